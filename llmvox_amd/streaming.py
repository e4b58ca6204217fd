"""Multi-queue streaming scheduler of the LLMVoX TTS hot path.

Two layers:

1. ``audio_generator_sync`` / ``route_text`` / ``audio_generator_async`` / ``clean_text`` —
   the reference's scheduler (streaming_server.py:106-149,184-469) with the same signature
   and behaviour, driving any ModelHandler-like object one token at a time (our
   ``llmvox_amd.ModelHandler``, the CPU oracle, or a scripted fake in tests).

2. ``SegmentMachine`` + ``FusedScheduler`` — the same per-stream semantics (dump schedule,
   EOA flush, reset, control signals) restated as a state machine that consumes greedy
   tokens produced in chunks by the fused HIP decode step (``lvx_ar_steps``) for many
   streams at once (continuous batching), with the codec decode of every dump batched
   across streams. Run-ahead past an end-of-audio token is rolled back exactly.
"""
from __future__ import annotations

import asyncio
import re
from collections import deque
from dataclasses import dataclass, field
from queue import Empty, Queue
from typing import Callable, Deque, Dict, List, Optional

import numpy as np

from . import config as C


def _cfg(config, key, default):
    if config is None:
        return default
    if hasattr(config, "get"):
        v = config.get(key, default)
    else:
        v = getattr(config, key, default)
    return default if v is None else v


# ---------------------------------------------------------------------------------------
# text cleaning / routing (streaming_server.py:106-149, 224-244)
# ---------------------------------------------------------------------------------------

def clean_text(text: str, eos_token: str = C.EOS_TOKEN) -> str:
    """Same substitutions, same order as the reference's clean_text."""
    text = text.strip().replace("**", "").replace("-", " ")
    text = re.sub(r"(\d)\.(?=\s|$)", r"\1", text)
    text = re.sub(r"\*", "", text)
    text = re.sub(r"#", " number ", text)
    text = re.sub(r"&", " and ", text)
    text = re.sub(r"@", " at ", text)
    text = re.sub(r"\s+", " ", text)
    text = re.sub(r"\.{3,}", " pause ", text)
    text = re.sub(r"(\d),(\d)", r"\1\2", text)
    text = re.sub(r"\/+", " slash ", text)
    text = re.sub(r"\\+", " backslash ", text)
    return text


def route_text(outputs, queues, eos: str = C.EOS_TOKEN):
    """text_streamer_producer's routing: skip '' / '-', strip, clean (unless it is the EOS
    token), put on the active queue, switch queue after a word that ends with '.'."""
    active = 0
    routed = []
    for out in outputs:
        if out in ("", "-"):
            continue
        out = out.strip()
        if out != eos:
            out = clean_text(out, eos)
        routed.append(out)
        if out:
            queues[active].put(out)
            if out.endswith("."):
                active = 1 - active
    return routed


# ---------------------------------------------------------------------------------------
# 1. the reference-shaped consumer (one token per model call)
# ---------------------------------------------------------------------------------------

def audio_generator_sync(index: int, dump_size: int, model_handler, text_token_queue: Queue,
                         audio_byte_queue: Queue, config=None):
    """Consumer thread of the multi-queue design (streaming_server.py:250-426).

    Extension: a ``None`` text token ends the loop (the reference loops forever); the
    generator then puts ``None`` on the audio queue, as the reference's unreachable tail does.
    """
    import torch
    import torch.nn.functional as F

    max_audio_len = _cfg(config, "max_audio_length", C.MAX_AUDIO_LENGTH)
    max_dump = _cfg(config, "max_dump_size", C.MAX_DUMP_SIZE)
    eos = _cfg(config, "eos_token", C.EOS_TOKEN)
    pad_token_id = _cfg(config, "pad_token_id", C.PAD_TOKEN_ID)
    eoa_token_id = _cfg(config, "eoa_token_id", C.EOA_TOKEN_ID)
    dev = model_handler.device
    bandwidth_id = torch.tensor([0]).to(dev)

    gen_index, cur_tok, kvcache = 0, None, None
    end_of_speech, end_generation = False, False
    speech_outputs: List[int] = []
    hist = None

    def grow(ds):
        return min(ds * 3, max_dump) if ds < max_dump else ds

    def emit(tokens):
        codes = torch.tensor([tokens]).to(dev)
        feats = model_handler.wavtokenizer.codes_to_features(codes)
        audio = model_handler.wavtokenizer.decode(feats, bandwidth_id=bandwidth_id).squeeze(0)
        audio_byte_queue.put(audio.detach().cpu().numpy().astype("float32").tobytes())

    with torch.inference_mode():
        while True:
            if not end_of_speech:
                word = text_token_queue.get()
                if word is None:
                    break
                if (eos in word) or (word[-1] == "."):
                    if eos in word:
                        end_generation = True
                    word = word.rstrip(eos)  # a character-set strip, as in the reference
                    end_of_speech = True
                else:
                    end_of_speech = False
                ids = model_handler.tokenizer(word.strip())["input_ids"]
                if end_of_speech:
                    ids = ids + [C.EOS_TEXT_ID]
                text_emb = model_handler.llm_model(torch.tensor(ids).unsqueeze(0).to(dev))
            else:
                text_emb = model_handler.llm_model(torch.tensor([pad_token_id]).unsqueeze(0).to(dev))

            for i in range(text_emb.shape[1]):
                if gen_index == 0:
                    speech = torch.zeros((1, 1, 512), device=dev)
                else:
                    tok_t = torch.tensor([[cur_tok]]).to(dev)
                    speech = model_handler.wavtokenizer.codes_to_features(tok_t).permute(0, 2, 1).to(dev)
                x = torch.cat([text_emb[:, i, :].unsqueeze(1), speech], dim=2)
                x = F.normalize(x, p=2, dim=2, eps=1e-8)
                if gen_index > 0:
                    x = torch.cat([hist, x], dim=1)
                logits, _, kvcache = model_handler.model(x, kvcache=kvcache)
                cur_tok = int(F.softmax(logits[:, -1, :], dim=-1).argmax(dim=-1).item())
                speech_outputs.append(cur_tok)
                hist = x
                gen_index += 1

                if len(speech_outputs) >= dump_size:
                    batch, speech_outputs = speech_outputs[:dump_size], speech_outputs[dump_size:]
                    emit(batch)
                    dump_size = grow(dump_size)
                elif eoa_token_id in speech_outputs:
                    emit(speech_outputs)
                    speech_outputs = []
                    dump_size = grow(dump_size)

                if cur_tok == eoa_token_id or len(speech_outputs) > max_audio_len:
                    if end_generation:
                        audio_byte_queue.put("end")
                    else:
                        audio_byte_queue.put(1 if index == 0 else 0)
                    gen_index, cur_tok, kvcache, hist = 0, None, None, None
                    end_of_speech, end_generation = False, False
                    speech_outputs = []
                    dump_size = grow(dump_size)
    audio_byte_queue.put(None)


def audio_chunks(queue_1: Queue, queue_2: Queue, timeout: float = 1.0, stop: Optional[Callable[[], bool]] = None):
    """Synchronous form of audio_generator_async (streaming_server.py:428-469): yields PCM
    byte chunks in speaking order, switching queues on the 0/1 signals; 'end' closes the
    stream (the reference yields None there, which ends the HTTP response by exception)."""
    qs = [queue_1, queue_2]
    cur = qs[0]
    while True:
        if stop is not None and stop():
            return
        try:
            item = cur.get(True, timeout)
        except Empty:
            continue
        if isinstance(item, str) and item == "end":
            return
        if isinstance(item, int) and not isinstance(item, bool) and item in (0, 1):
            cur = qs[item]
            continue
        if item is None:
            continue
        yield item


async def audio_generator_async(queue_1: Queue, queue_2: Queue):
    loop = asyncio.get_event_loop()
    qs = [queue_1, queue_2]
    cur = qs[0]
    while True:
        try:
            item = await loop.run_in_executor(None, cur.get, True, 1)
        except Empty:
            continue
        if isinstance(item, str) and item == "end":
            return
        if isinstance(item, int) and item in (0, 1):
            cur = qs[item]
            continue
        if item is None:
            continue
        yield item


# ---------------------------------------------------------------------------------------
# 2. token-level state machine of one replica stream (same semantics as above)
# ---------------------------------------------------------------------------------------

@dataclass
class Event:
    kind: str            # "audio" (tokens to decode) or "signal" (0 / 1 / "end")
    tokens: Optional[List[int]] = None
    signal: object = None


@dataclass
class SegmentMachine:
    """The per-token semantics of audio_generator_sync, with the model call factored out:
    ``next_text_id()`` says what the next decode step is fed, ``consume(token)`` applies the
    dump / EOA / reset rules and returns the events, exactly in the reference's order."""
    index: int = 0
    dump_size: int = C.INITIAL_DUMP_SIZE_1
    tokenizer: object = None
    max_audio_len: int = C.MAX_AUDIO_LENGTH
    max_dump: int = C.MAX_DUMP_SIZE
    eos: str = C.EOS_TOKEN
    pad_id: int = C.PAD_TOKEN_ID
    eoa_id: int = C.EOA_TOKEN_ID
    words: Deque[str] = field(default_factory=deque)
    pending: Deque[int] = field(default_factory=deque)
    gen_index: int = 0
    end_of_speech: bool = False
    end_generation: bool = False
    speech_outputs: List[int] = field(default_factory=list)
    closed: bool = False

    def __post_init__(self):
        if self.tokenizer is None:
            from .tokenizer import ByteTokenizer
            self.tokenizer = ByteTokenizer()

    # -- text side --
    def feed(self, word: Optional[str]):
        self.words.append(word)

    def _word_ids(self, word: str):
        eos = self.eos
        if (eos in word) or (word[-1] == "."):
            end_gen = eos in word
            word = word.rstrip(eos)
            eos_flag = True
        else:
            end_gen, eos_flag = False, False
        ids = self.tokenizer(word.strip())["input_ids"]
        if eos_flag:
            ids = ids + [C.EOS_TEXT_ID]
        return ids, eos_flag, end_gen

    def _refill(self) -> bool:
        """Make ``pending`` non-empty; False when the next word has not arrived yet."""
        if self.pending:
            return True
        if self.end_of_speech:
            self.pending.append(self.pad_id)
            return True
        if not self.words:
            return False
        word = self.words.popleft()
        if word is None:
            self.closed = True
            return False
        ids, self.end_of_speech, eg = self._word_ids(word)
        if eg:
            self.end_generation = True
        self.pending.extend(ids)
        return True

    def plan(self, n: int) -> List[int]:
        """The text ids of the next n steps if no end-of-audio occurs (no state change);
        shorter when text is not available yet."""
        out = list(self.pending)[:n]
        eos_flag, words = self.end_of_speech, list(self.words)
        wi = 0
        while len(out) < n:
            if eos_flag:
                out.extend([self.pad_id] * (n - len(out)))
                break
            if wi >= len(words) or words[wi] is None:
                break
            ids, eos_flag, _ = self._word_ids(words[wi])
            wi += 1
            out.extend(ids[: n - len(out)])
        return out

    def next_text_id(self) -> Optional[int]:
        if not self._refill():
            return None
        return self.pending[0]

    # -- token side --
    def _grow(self):
        if self.dump_size < self.max_dump:
            self.dump_size = min(self.dump_size * 3, self.max_dump)

    def consume(self, token: int) -> List[Event]:
        """Apply one greedy token of the step fed ``next_text_id()``."""
        if not self._refill():
            raise RuntimeError("consume() without an available text id")
        self.pending.popleft()
        ev: List[Event] = []
        self.speech_outputs.append(int(token))
        self.gen_index += 1
        if len(self.speech_outputs) >= self.dump_size:
            batch = self.speech_outputs[: self.dump_size]
            self.speech_outputs = self.speech_outputs[self.dump_size:]
            ev.append(Event("audio", tokens=batch))
            self._grow()
        elif self.eoa_id in self.speech_outputs:
            ev.append(Event("audio", tokens=self.speech_outputs))
            self.speech_outputs = []
            self._grow()
        if token == self.eoa_id or len(self.speech_outputs) > self.max_audio_len:
            sig = "end" if self.end_generation else (1 if self.index == 0 else 0)
            ev.append(Event("signal", signal=sig))
            self.gen_index = 0
            self.end_of_speech = False
            self.end_generation = False
            self.speech_outputs = []
            self._grow()
        return ev

    @property
    def position(self):
        return self.gen_index


# ---------------------------------------------------------------------------------------
# fused multi-stream scheduler on the HIP step
# ---------------------------------------------------------------------------------------

class FusedStream:
    def __init__(self, sched, slot, machine: SegmentMachine, sink: Optional[Queue] = None):
        self.sched = sched
        self.slot = slot
        self.m = machine
        self.sink = sink if sink is not None else Queue()
        self.events: List[object] = []   # decoded items in order: bytes or signals
        self.tokens: List[int] = []      # every greedy token consumed (diagnostics / tests)
        self.fed = False                 # a word has been fed (the service caps only fed streams)

    def feed(self, word):
        self.fed = True
        self.m.feed(word)

    def _out(self, item):
        self.events.append(item)
        self.sink.put(item)


class FusedScheduler:
    """Continuous batching of many replica streams on one Engine.

    Every ``run_chunk`` call: each stream with text available contributes its planned text
    ids for the next n steps (n ends at the earliest pending dump boundary, so the first
    chunk of a stream is decoded as soon as its tokens exist); the fused step runs n times
    for all rows (one HIP-graph replay per step, no host traffic); tokens are read back once;
    every stream's SegmentMachine consumes them in order; a stream that hits end-of-audio
    drops its run-ahead tokens and its slot is rewound to position 0; all dumps of the chunk
    are decoded (batched by length) and delivered in order.

    With ``overlap=True`` the codec of chunk c runs on a second HIP stream while the AR decode of
    chunk c+1 runs on the main one: chunk c's items are delivered by the next
    ``run_chunk`` right after it has launched chunk c+1, or by ``flush`` (called by
    ``run_until_idle`` and by an idle ``run_chunk``). Off by default: measured on MI355X, the
    latency-bound AR chain stalls while codec kernels from another queue are in flight, so the
    overlapped loop is slower than running the codec after the AR on one stream (25.5 vs
    23.6 ms per 256-token chunk at 1 stream, 65.2 vs 64.4 ms at 32; round 1).
    """

    def __init__(self, engine, max_chunk: int = 64, max_rows: Optional[int] = None, to_bytes: bool = True,
                 overlap: bool = False):
        import torch
        self.engine = engine
        self.torch = torch
        self.max_chunk = max_chunk
        self.max_rows = max_rows or engine.max_streams
        self.streams: List[FusedStream] = []
        self.free_slots = list(range(engine.max_streams - 1, -1, -1))
        self.to_bytes = to_bytes
        dev = engine.device
        R, n = self.max_rows, max_chunk
        self.slots_d = torch.full((R,), -1, dtype=torch.int32, device=dev)
        self.plan_d = torch.zeros((R, n), dtype=torch.int32, device=dev)
        self.rowstep_d = torch.zeros((R,), dtype=torch.int32, device=dev)
        self.tok_d = torch.zeros((R, n), dtype=torch.int32, device=dev)
        pin = torch.device(dev).type == "cuda"
        self.plan_h = torch.zeros((R, n), dtype=torch.int32, pin_memory=pin)
        self.slots_h = torch.full((R,), -1, dtype=torch.int32, pin_memory=pin)
        self.overlap = bool(overlap) and pin
        self.codec_stream = torch.cuda.Stream(device=dev) if self.overlap else None
        self.pcm_h = None      # pinned staging buffer of the decode in flight (grown on demand)
        self.pending = None    # (event, [(dump index, offset, samples)], order, ready) of the last chunk

    def open_stream(self, index=0, dump_size=C.INITIAL_DUMP_SIZE_1, sink=None, **kw) -> FusedStream:
        if not self.free_slots:
            raise RuntimeError("no free KV slot")
        slot = self.free_slots.pop()
        st = FusedStream(self, slot, SegmentMachine(index=index, dump_size=dump_size, **kw), sink)
        self.engine.reset_slot(slot)
        self.streams.append(st)
        return st

    def close_stream(self, st: FusedStream):
        self.streams.remove(st)
        self.free_slots.append(st.slot)

    def _steps_to_dump(self, m: SegmentMachine):
        return max(1, m.dump_size - len(m.speech_outputs))

    def run_chunk(self) -> int:
        """One chunk for all ready streams; returns the number of decode steps run (0 = idle)."""
        torch = self.torch
        ready = []
        for st in self.streams:
            if st.m.closed:
                continue
            if st.m.next_text_id() is None:
                continue
            ready.append(st)
        ready = ready[: self.max_rows]
        if not ready:
            self.flush()
            return 0
        n = min(self.max_chunk, min(self._steps_to_dump(st.m) for st in ready))
        plans = {}
        for st in ready:
            p = st.m.plan(n)
            plans[st] = p
            n = min(n, len(p))
        self.slots_h.fill_(-1)
        for r, st in enumerate(ready):
            self.slots_h[r] = st.slot
            self.plan_h[r, :n] = torch.tensor(plans[st][:n], dtype=torch.int32)
        B = len(ready)
        self.slots_d.copy_(self.slots_h, non_blocking=True)
        self.plan_d.copy_(self.plan_h, non_blocking=True)
        self.rowstep_d.zero_()
        self.engine.ar_steps(n, self.slots_d[:B], self.plan_d[:B], self.rowstep_d[:B], self.tok_d[:B])
        self.flush()  # the previous chunk's audio, decoded while this chunk's AR steps run
        toks = self.tok_d[:B, :n].cpu().numpy()
        # a KV-capacity error concerns only the rows that reached max_positions in this chunk (their
        # last positions were clamped); every other row's tokens are valid and are consumed, decoded
        # and delivered below before the error is raised, naming the streams at the edge
        cap_err, edge = None, set()
        try:
            self.engine.check_errors()
        except Exception as e:
            from ._lib import LvxCapacityError
            if not isinstance(e, LvxCapacityError):
                raise
            # a row that ran past max_positions had its last positions clamped: those tokens are
            # invalid. A row that ends exactly AT max_positions set the flag with the commit of its
            # last step, but all n of its tokens came from positions <= max_positions - 1: they are
            # valid and consumed below; the row is then reported at capacity with the others
            P = self.engine.max_positions
            edge = {st for st in ready if st.m.position + n > P}
            at_cap = {st for st in ready if st.m.position + n == P}
            if not edge and not at_cap:  # not a position overflow of a known row (e.g. a plan overrun)
                raise
            cap_err = e
            cap_err.streams = sorted(edge | at_cap, key=lambda st: st.slot)
        dumps = []  # (stream, tokens)
        order: Dict[FusedStream, List[tuple]] = {st: [] for st in ready}
        for r, st in enumerate(ready):
            if st in edge:
                continue
            for j in range(n):
                tok = int(toks[r, j])
                st.tokens.append(tok)
                reset = False
                for e in st.m.consume(tok):
                    if e.kind == "audio":
                        dumps.append((st, e.tokens))
                        order[st].append(("audio", len(dumps) - 1))
                    else:
                        order[st].append(("signal", e.signal))
                        reset = True
                if reset:
                    # run-ahead past end-of-audio: drop the rest, restart the slot at position 0
                    self.engine.set_slot(st.slot, 0, 0)
                    break
        if self.overlap:
            self._launch_decode(dumps, order, ready)
        else:
            self._deliver(self._decode(dumps), order, ready)
        if cap_err is not None:
            self.flush()
            raise cap_err
        return n

    def _deliver(self, pcm, order, ready):
        for st in ready:
            for kind, v in order[st]:
                st._out(pcm[v] if kind == "audio" else v)

    def _groups(self, dumps):
        """Dump indices batched by length (one codec call per group, within max_codec_frames)."""
        by_len: Dict[int, List[int]] = {}
        for i, (_, toks) in enumerate(dumps):
            by_len.setdefault(len(toks), []).append(i)
        for L, idx in by_len.items():
            cap = max(1, self.engine.max_codec_frames // L)
            for s in range(0, len(idx), cap):
                yield L, idx[s:s + cap]

    def _decode(self, dumps):
        torch = self.torch
        res: List[object] = [None] * len(dumps)
        for L, grp in self._groups(dumps):
            codes = torch.tensor([dumps[i][1] for i in grp], dtype=torch.int32, device=self.engine.device)
            out = self.engine.decode_codes(codes).cpu().numpy()
            for k, i in enumerate(grp):
                res[i] = out[k].astype("float32").tobytes() if self.to_bytes else out[k]
        return res

    def _launch_decode(self, dumps, order, ready):
        """Queue the chunk's decodes on the codec stream, PCM into pinned host memory; no wait."""
        torch = self.torch
        total = 320 * sum(len(t) for _, t in dumps)
        if self.pcm_h is None or self.pcm_h.numel() < total:
            self.pcm_h = torch.empty(max(total, 1 << 16) * 2, dtype=torch.float32, pin_memory=True)
        spans, off = [], 0
        with torch.cuda.stream(self.codec_stream):
            for L, grp in self._groups(dumps):
                codes = torch.tensor([dumps[i][1] for i in grp], dtype=torch.int32, device=self.engine.device)
                out = self.engine.decode_codes(codes)
                self.pcm_h[off:off + out.numel()].view(out.shape).copy_(out, non_blocking=True)
                for k, i in enumerate(grp):
                    spans.append((i, off + k * 320 * L, 320 * L))
                off += out.numel()
            ev = torch.cuda.Event()
            ev.record(self.codec_stream)
        self.pending = (ev, spans, order, ready, len(dumps))

    def flush(self):
        """Deliver the items of the chunk whose decode is in flight (overlap mode)."""
        if self.pending is None:
            return
        ev, spans, order, ready, nd = self.pending
        self.pending = None
        ev.synchronize()
        pcm: List[object] = [None] * nd
        for i, off, ln in spans:
            a = self.pcm_h[off:off + ln].numpy()
            pcm[i] = a.tobytes() if self.to_bytes else a.copy()
        self._deliver(pcm, order, ready)

    def run_until_idle(self, max_chunks: int = 1 << 30) -> int:
        total = 0
        for _ in range(max_chunks):
            n = self.run_chunk()
            if n == 0:
                break
            total += n
        self.flush()
        return total
