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
import atexit
import contextlib
import copy
import re
import threading
import weakref
from collections import deque
from dataclasses import dataclass, field
from queue import Empty, Queue
from typing import Callable, Deque, Dict, List, Optional

import numpy as np

from . import config as C
from .streams import side_stream


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
        """(ids, end of speech, end of generation) of a word; memoised (plan() re-reads the words ahead
        every chunk, and the regex tokenizer costs ~10 us a word)."""
        cache = self.__dict__.setdefault("_ids_cache", {})
        got = cache.get(word)
        if got is None:
            got = cache[word] = self._word_ids_uncached(word)
            if len(cache) > 4096:
                cache.clear()
        ids, eos_flag, end_gen = got
        return list(ids), eos_flag, end_gen

    def _word_ids_uncached(self, word: str):
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

    def consume_many(self, tokens) -> tuple:
        """``consume`` over a run of tokens, stopping after a segment end: (events, tokens consumed).
        A run without end-of-audio that stays within max_audio_length takes a batched path (the text
        ids popped at once, the dumps cut as consecutive dump-size slices: exactly what consume does one
        token at a time, since a dump empties the outputs whenever they reach the dump size)."""
        n = len(tokens)
        if self.eoa_id in tokens or len(self.speech_outputs) + n > self.max_audio_len:
            ev: List[Event] = []
            for j, t in enumerate(tokens):
                e = self.consume(int(t))
                ev += e
                if any(x.kind == "signal" for x in e):
                    return ev, j + 1
            return ev, n
        k = n
        while k:
            if not self.pending and self.end_of_speech:
                break  # the rest are PAD steps: _refill would push one PAD id per step and pop it
            if not self._refill():
                raise RuntimeError("consume() without an available text id")
            take = min(k, len(self.pending))
            for _ in range(take):
                self.pending.popleft()
            k -= take
        self.gen_index += n
        buf = self.speech_outputs + [int(t) for t in tokens]  # (ints: tokens may be numpy scalars)
        ev = []
        pos = 0
        while len(buf) - pos >= self.dump_size:
            ev.append(Event("audio", tokens=buf[pos:pos + self.dump_size]))
            pos += self.dump_size
            self._grow()
        self.speech_outputs = buf[pos:]
        return ev, n

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


def _copy_machine(m: SegmentMachine) -> SegmentMachine:
    """A speculative copy of a machine (its own word / id queues and speech outputs; the tokenizer
    is shared)."""
    c = copy.copy(m)
    c.words = deque(m.words)
    c.pending = deque(m.pending)
    c.speech_outputs = list(m.speech_outputs)
    return c


class _Chunk:
    """One launched AR chunk: its rows, steps, buffer set and completion event; ``bad`` holds the
    streams whose rows it must not consume (rolled back by an end-of-audio of an older chunk)."""

    def __init__(self, ready, n, buf, event, near=None):
        self.ready, self.n, self.buf, self.event, self.near = ready, n, buf, event, near
        self.bad = set()


_LIVE_DELIVERERS: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _close_deliverers():
    """Stop every delivery thread before the interpreter finalises: a daemon thread still inside a
    GIL-releasing torch call (Event.synchronize) when finalisation reclaims it unwinds through a C++
    destructor and the process aborts ("terminate called without an active exception")."""
    for d in list(_LIVE_DELIVERERS):
        d.close()


class _Deliverer:
    """The overlapped scheduler's delivery thread: jobs run in submission order; each waits for its
    codec event (if any), then hands its items to the streams, so a dump reaches its stream as soon
    as its codec call has finished, in the reference's per-stream order."""

    def __init__(self):
        self.q: Queue = Queue()
        self.cv = threading.Condition()
        self.pending = 0
        self.error: Optional[BaseException] = None
        self.thread = threading.Thread(target=self._run, name="lvx-deliver", daemon=True)
        self.thread.start()
        _LIVE_DELIVERERS.add(self)

    def put(self, event, fn):
        with self.cv:
            self.pending += 1
        self.q.put((event, fn))

    def _run(self):
        while True:
            ev, fn = self.q.get()
            if fn is None:
                return
            try:
                if ev is not None:
                    ev.synchronize()
                fn()
            except BaseException as e:  # surfaced on the scheduler thread (take_error)
                from ._lib import LvxStreamError
                if self.error is None:
                    self.error = e
                elif isinstance(self.error, LvxStreamError) and isinstance(e, LvxStreamError):
                    # two groups' codec errors before the scheduler took the first: one error naming both
                    self.error.streams = sorted(set(self.error.streams) | set(e.streams), key=lambda st: st.slot)
            with self.cv:
                self.pending -= 1
                self.cv.notify_all()

    def wait(self):
        with self.cv:
            while self.pending:
                self.cv.wait()

    def take_error(self):
        e, self.error = self.error, None
        if e is not None:
            raise e

    def close(self):
        if self.thread.is_alive():
            self.q.put((None, None))
            self.thread.join(timeout=30)
        _LIVE_DELIVERERS.discard(self)


class FusedScheduler:
    """Continuous batching of many replica streams on one Engine.

    A chunk: each stream with text available contributes its planned text ids for the next n steps
    (n ends at the earliest pending dump boundary, so the first chunk of a stream is decoded as soon
    as its tokens exist); the fused step runs n times for all rows (one HIP-graph replay per 16
    steps, no host traffic); tokens are read back once; every stream's SegmentMachine consumes them
    in order; a stream that hits end-of-audio drops its run-ahead tokens and its slot is rewound to
    position 0; all dumps of the chunk are decoded (batched by length) and delivered in order.

    ``overlap=True`` runs the schedule of the reference's two replicas and of the bench
    (streaming_server.py:357-376): chunk c + 1's decode steps are queued on the main
    stream BEFORE chunk c's tokens are read back (planned from the streams' speculative state after
    chunk c without an end-of-audio; a stream whose chunk c does end its segment has its chunk c + 1
    row discarded, and its slot rewound behind it); chunk c's codec runs on a second HIP stream, queued
    only once the host holds its tokens (host-paced: no queue ever waits on the other's event, which
    costs every dispatch of the AR chain ~1 us); each chunk's items are delivered by a
    delivery thread as soon as its codec event completes. Streams see the same items, in the same
    order, as without overlap (tests/test_gpu_streaming.py). Run-ahead is skipped for a chunk whose
    rows would cross max_positions (the capacity edge then behaves as without overlap). On a CPU
    stand-in engine the same run-ahead / rollback / ordering runs with synchronous decodes.

    ``stop_rule(stream, tokens, position)`` (optional): True when a stream must not be planned once it
    has consumed ``tokens`` tokens and stands at ``position`` (the service's max_tokens / capacity
    stop), applied to the speculative state too, so run-ahead never decodes past a stop.

    Joining streams: a chunk longer than ``tail`` steps is queued as two calls with an event between
    them, ``tail`` steps before its end; the next chunk is planned once that event has passed, so a
    stream opened while a chunk runs joins the very next chunk (with run-ahead planned at the chunk's
    start it would wait a whole extra chunk), and the tail steps cover the host's planning.
    ``waiter(event)`` (optional) replaces every host wait on a device event: the service passes one that
    releases its lock meanwhile, so requests are admitted while the scheduler waits for the device.
    ``stream`` (optional): the HIP stream of the decode steps and slot updates, whatever thread calls
    (default: the calling thread's current stream). Decode steps on the legacy null stream run
    without graphs and serialise with every other stream, so the service gives each device one.
    """

    def __init__(self, engine, max_chunk: int = 32, max_rows: Optional[int] = None, to_bytes: bool = True,
                 overlap: bool = False, stop_rule=None, waiter=None, tail: int = 8, stream=None,
                 codec_stream: bool = True):
        import torch
        self.engine = engine
        self.torch = torch
        self.max_chunk = max_chunk
        self.max_rows = max_rows or engine.max_streams
        self.streams: List[FusedStream] = []
        self.free_slots = list(range(engine.max_streams - 1, -1, -1))
        self.to_bytes = to_bytes
        self.stop_rule = stop_rule
        self.waiter = waiter
        self.tail = max(1, int(tail))
        self.ar_stream = stream
        dev = engine.device
        self.cuda = torch.device(dev).type == "cuda"
        self.overlap = bool(overlap)
        # the codec's stream is checked to run beside the decode stream (streams.side_stream: two streams
        # on one hardware queue run in order, and the overlap would be silently lost)
        self.codec_stream = (side_stream(dev, [stream]) if codec_stream else (stream or torch.cuda.current_stream(dev))) \
            if (self.overlap and self.cuda) else None
        self.take = self.cuda and hasattr(engine, "take_errors")
        self.codec_take = hasattr(engine, "take_errors")  # (host-synchronous decodes: any engine with the words)
        self.bufs = [self._alloc() for _ in range(2 if self.overlap else 1)]
        self._bi = 0
        self.inflight: Deque[_Chunk] = deque()
        self.deliverer = _Deliverer() if self.overlap else None
        # streams whose dump failed in the codec (its error word): nothing more is delivered to them,
        # so a client never receives audio after a hole (the error names them; the caller closes them;
        # weak: kept past close_stream, for the jobs of chunks still queued behind the failure)
        self.failed = weakref.WeakSet()

    def _alloc(self):
        torch, dev = self.torch, self.engine.device
        R, n = self.max_rows, self.max_chunk
        pin = self.cuda
        return {"slots_d": torch.full((R,), -1, dtype=torch.int32, device=dev),
                "plan_d": torch.zeros((R, n), dtype=torch.int32, device=dev),
                "rowstep_d": torch.zeros((R,), dtype=torch.int32, device=dev),
                "tok_d": torch.zeros((R, n), dtype=torch.int32, device=dev),
                "err_d": torch.zeros((1,), dtype=torch.int32, device=dev),
                "plan_h": torch.zeros((R, n), dtype=torch.int32, pin_memory=pin),
                "slots_h": torch.full((R,), -1, dtype=torch.int32, pin_memory=pin),
                "tok_h": torch.zeros((R, n), dtype=torch.int32, pin_memory=pin),
                "err_h": torch.zeros((1,), dtype=torch.int32, pin_memory=pin)}

    def open_stream(self, index=0, dump_size=C.INITIAL_DUMP_SIZE_1, sink=None, **kw) -> FusedStream:
        if not self.free_slots:
            raise RuntimeError("no free KV slot")
        slot = self.free_slots.pop()
        st = FusedStream(self, slot, SegmentMachine(index=index, dump_size=dump_size, **kw), sink)
        with self._on_ar():
            self.engine.reset_slot(slot)  # (stream-ordered behind any chunk in flight on the slot)
        self.streams.append(st)
        return st

    def close_stream(self, st: FusedStream):
        self.streams.remove(st)
        self.free_slots.append(st.slot)

    def close(self):
        """Stop the delivery thread (after delivering what is queued)."""
        if self.deliverer is not None:
            self.deliverer.wait()
            self.deliverer.close()
            self.deliverer = None

    def _on_ar(self):
        return self.torch.cuda.stream(self.ar_stream) if self.ar_stream is not None else contextlib.nullcontext()

    def _steps_to_dump(self, m: SegmentMachine):
        return max(1, m.dump_size - len(m.speech_outputs))

    # -- planning ---------------------------------------------------------------------------
    def _speculative(self):
        """Each stream of the chunk in flight, advanced over that chunk as if it ended no segment:
        {stream: (machine copy or None when the chunk ends its segment anyway, tokens consumed)}."""
        spec = {}
        for ch in self.inflight:
            for st in ch.ready:
                if st in ch.bad or st not in self.streams:
                    continue
                m0, ntok = spec.get(st, (st.m, len(st.tokens)))
                if m0 is None:
                    continue
                m = _copy_machine(m0)
                dummy = 0 if m.eoa_id != 0 else 1
                try:
                    ev, used = m.consume_many([dummy] * ch.n)
                    ends = used < ch.n or any(e.kind == "signal" for e in ev)  # (a max_audio_length reset)
                except RuntimeError:
                    ends = True
                spec[st] = (None if ends else m, ntok + ch.n)
        return spec

    def _launch_next(self) -> int:
        """Plan and queue the next chunk (from the speculative state of the chunk in flight, if any);
        returns its steps, 0 when nothing is ready or run-ahead would cross the capacity edge."""
        torch = self.torch
        if self.inflight and self.inflight[-1].near is not None:
            self._wait(self.inflight[-1].near)  # `tail` steps before the chunk in flight ends
            self.inflight[-1].near = None
        spec = self._speculative() if self.inflight else {}
        ready = []
        for st in self.streams:
            m, ntok = spec.get(st, (st.m, len(st.tokens)))
            if m is None or m.closed or m.next_text_id() is None:
                continue
            if self.stop_rule is not None and self.stop_rule(st, ntok, m.position):
                continue
            ready.append((st, m))
        ready = ready[: self.max_rows]
        if not ready:
            return 0
        n = min(self.max_chunk, min(self._steps_to_dump(m) for _, m in ready))
        plans = []
        for st, m in ready:
            p = m.plan(n)
            plans.append(p)
            n = min(n, len(p))
        if self.inflight and any(m.position + n > self.engine.max_positions for _, m in ready):
            return 0  # the capacity edge: complete the chunk in flight first (no run-ahead)
        with self._on_ar():
            return self._launch(ready, plans, n)

    def _launch(self, ready, plans, n) -> int:
        torch = self.torch
        buf = self.bufs[self._bi]
        self._bi = (self._bi + 1) % len(self.bufs)
        B = len(ready)
        sl = buf["slots_h"].numpy()
        sl[:] = -1
        sl[:B] = [st.slot for st, _ in ready]
        buf["plan_h"].numpy()[:B, :n] = np.array([p[:n] for p in plans], dtype=np.int32)
        buf["slots_d"].copy_(buf["slots_h"], non_blocking=True)
        buf["plan_d"].copy_(buf["plan_h"], non_blocking=True)
        buf["rowstep_d"].zero_()
        args = (buf["slots_d"][:B], buf["plan_d"][:B], buf["rowstep_d"][:B], buf["tok_d"][:B])
        near = None
        if self.overlap and self.cuda and n >= 2 * self.tail:  # (a short chunk is planned behind at once)
            # (round 5, measured worse: the head rounded down to whole 16-step graph replays moved the
            # planning point up to 16 steps before the chunk's end, and a request arriving in that window
            # waits for the whole next chunk: loaded first chunk p50 11.2 / 13.8 vs 9.0 / 10.2 ms,
            # tools/latency_ab.py 32)
            head = n - self.tail
            self.engine.ar_steps(head, *args)
            near = torch.cuda.Event()
            near.record(torch.cuda.current_stream(self.engine.device))
            self.engine.ar_steps(n - head, *args)
        else:
            self.engine.ar_steps(n, *args)
        ev = None
        if self.cuda:
            buf["tok_h"].copy_(buf["tok_d"], non_blocking=True)
            if self.take:
                from . import _lib
                self.engine.take_errors(_lib.ERRW_AR, buf["err_d"])
                buf["err_h"].copy_(buf["err_d"], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.engine.device))
        self.inflight.append(_Chunk([st for st, _ in ready], n, buf, ev, near))
        return n

    def _wait(self, ev):
        if self.waiter is not None:
            self.waiter(ev)
        else:
            ev.synchronize()

    # -- completion --------------------------------------------------------------------------
    def _chunk_error(self, ch):
        if not self.take:  # a stand-in engine: its own (synchronous) check
            try:
                self.engine.check_errors()
            except Exception as e:
                return e
            return None
        bits = int(ch.buf["err_h"][0])
        if not bits:
            return None
        from . import _lib
        return _lib.error_for(self.engine.lib.lvx_error_status(bits), bits)

    def _complete(self, ch: _Chunk) -> int:
        """Read back the chunk's tokens (waits for its event only), consume them, queue its decodes."""
        if ch.event is not None:
            self._wait(ch.event)
        B, n = len(ch.ready), ch.n
        toks = (ch.buf["tok_h"] if self.cuda else ch.buf["tok_d"])[:B, :n].numpy()
        err = self._chunk_error(ch)
        # a KV-capacity error concerns only the rows that reached max_positions in this chunk (their
        # last positions were clamped); every other row's tokens are valid and are consumed, decoded
        # and delivered below before the error is raised, naming the streams at the edge. A fused-MLP
        # range error (B <= 2) invalidates the logits of this chunk's rows: they are named the same way
        from ._lib import LvxCapacityError, LvxNumericError
        edge, at_cap = set(), set()
        live = [st for st in ch.ready if st in self.streams and st not in ch.bad]  # (rows still consumed)
        if err is not None:
            if isinstance(err, LvxCapacityError):
                # a row that ran past max_positions had its last positions clamped: those tokens are
                # invalid. A row that ends exactly AT max_positions set the flag with the commit of
                # its last step, but all n of its tokens came from positions <= max_positions - 1:
                # they are consumed below, then the row is reported at capacity
                P = self.engine.max_positions
                bits = getattr(err, "bits", 0) or 0  # (device bits: 1 KV capacity, 2 a plan overrun)
                if bits & 2:
                    raise err
                # the rows at the edge among the live ones (a discarded row's machine was rewound by its
                # end of audio: its host position no longer says where its device row ran)
                if not any(st.m.position + n >= P for st in live):
                    if len(live) == len(ch.ready):
                        raise err  # no row can have reached the edge: not a capacity condition of ours
                    err = None  # only discarded rows can have run into it: their tokens are dropped anyway
                else:
                    edge = {st for st in live if st.m.position + n > P}
                    at_cap = {st for st in live if st.m.position + n == P}
            elif isinstance(err, LvxNumericError):
                edge = set(live)
            else:
                raise err
            # the named streams' rows in newer chunks (planned assuming this chunk was consumed) are not
            # consumed either: the caller ends those streams
            for st in edge | at_cap:
                for newer in self.inflight:
                    newer.bad.add(st)
            # (an error of rows already discarded -- a closed stream, a run-ahead row rolled back --
            # concerns no live stream: nothing is raised for it below)
        dumps = []  # (stream, tokens)
        order: Dict[FusedStream, List[tuple]] = {st: [] for st in ch.ready}
        ended = set()
        for r, st in enumerate(ch.ready):
            if st in edge or st in ch.bad or st not in self.streams:
                continue
            row = toks[r].tolist()
            evs, used = st.m.consume_many(row)
            st.tokens.extend(row[:used])
            reset = False
            for e in evs:
                if e.kind == "audio":
                    dumps.append((st, e.tokens))
                    order[st].append(("audio", len(dumps) - 1))
                else:
                    order[st].append(("signal", e.signal))
                    reset = True
            if reset:
                # run-ahead past end-of-audio: drop the rest, restart the slot at position 0
                # (queued behind any newer chunk in flight, whose row of this stream is discarded)
                with self._on_ar():
                    self.engine.set_slot(st.slot, 0, 0)
                for newer in self.inflight:
                    newer.bad.add(st)
                ended.add(st)
        # a row that reached the capacity exactly AND ended its segment in this chunk was rewound to
        # position 0 by the end of audio: it continues, as the reference would
        at_cap -= ended
        codec_err = None
        if self.overlap:
            self._launch_decode(dumps, order, ch.ready)
        else:
            pcm, codec_err = self._decode(dumps)
            self._deliver(pcm, order, ch.ready)
        if err is not None:
            if self.deliverer is not None:
                self.deliverer.wait()
            err.streams = sorted(edge | at_cap | set(codec_err.streams if codec_err else ()), key=lambda st: st.slot)
            if err.streams:
                raise err
        if codec_err is not None:
            raise codec_err
        return n

    def run_chunk(self) -> int:
        """Serial: one chunk for all ready streams, its items delivered on return. Overlap: queue the
        next chunk, then complete the one in flight before it (its items are delivered when its codec
        call ends). Returns the steps queued or completed (0 = idle: everything delivered)."""
        if self.deliverer is not None:
            self.deliverer.take_error()
        launched = self._launch_next()
        if self.inflight and (len(self.inflight) > 1 or not launched or not self.overlap):
            done = self._complete(self.inflight.popleft())
            return launched or done
        if not launched:
            self.flush()
        return launched

    def _deliver(self, pcm, order, ready):
        for st in ready:
            if st in self.failed:
                continue
            for kind, v in order[st]:
                st._out(pcm[v] if kind == "audio" else v)

    def _codec_failure(self, exc, streams):
        """A codec call's error word was set: the streams of its dumps get nothing more (``failed``) and
        the error is re-raised as an LvxStreamError naming them (the service ends only their requests);
        an error of a call that carries no stream's dump (decode_now) is returned as it was."""
        from ._lib import LvxStreamError
        streams = [st for st in streams if st is not None]
        if not streams:
            return exc
        for st in streams:
            self.failed.add(st)
        se = LvxStreamError(getattr(exc, "code", -2), f"codec error word: {exc}")
        se.bits = getattr(exc, "bits", 0)
        se.streams = sorted(set(streams), key=lambda st: st.slot)
        return se

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
        """Every dump decoded now (one call per length group), host-synchronous. Returns (PCM per dump,
        None or the LvxStreamError naming the streams of the groups whose codec error word was set:
        the other groups' PCM is valid and delivered)."""
        torch = self.torch
        res: List[object] = [None] * len(dumps)
        first, bad = None, []
        for L, grp in self._groups(dumps):
            codes = torch.tensor([dumps[i][1] for i in grp], dtype=torch.int32, device=self.engine.device)
            out = self.engine.decode_codes(codes).cpu().numpy()
            for k, i in enumerate(grp):
                res[i] = out[k].astype("float32").tobytes() if self.to_bytes else out[k]
            if self.codec_take:  # the codec's own error word, per group
                from . import _lib
                e = torch.zeros((1,), dtype=torch.int32, device=self.engine.device)
                self.engine.take_errors(_lib.ERRW_CODEC, e)
                try:
                    _lib.check_bits(int(e.item()))
                except _lib.LvxError as exc:
                    first = first or exc
                    bad += [dumps[i][0] for i in grp]
        return res, (self._codec_failure(first, bad) if first is not None else None)

    def decode_now(self, tokens: List[int]):
        """One dump decoded and returned at once, on the codec stream when overlapping, so it does not
        queue behind the decode chunk in flight (raises for the codec's error word)."""
        torch = self.torch
        with (torch.cuda.stream(self.codec_stream) if self.codec_stream is not None else contextlib.nullcontext()):
            res, err = self._decode([(None, tokens)])
        if err is not None:
            raise err
        return res[0]

    def queue_tail(self, st: FusedStream, tokens: List[int]):
        """The stream's undumped tail decoded as one last dump and delivered AFTER every item already
        queued for it (the service's end of a request). Overlap: queued on the codec stream, delivered by
        the delivery thread behind its event (the caller never waits for the device); serial: now."""
        if self.deliverer is None:
            st._out(self.decode_now(tokens))
            return
        self._launch_decode([(st, tokens)], {st: [("audio", 0)]}, [st])

    def after_delivered(self, fn):
        """fn() once every item queued so far has been delivered (in the delivery order)."""
        if self.deliverer is None:
            fn()
        else:
            self.deliverer.put(None, fn)

    def _launch_decode(self, dumps, order, ready):
        """Queue the chunk's decodes on the codec stream (codes from the host: no wait on the AR
        stream), one call per dump length, shortest first, each with its PCM copied into pinned host
        memory and a delivery job behind its own event: a stream's items go out with the job of its
        (last) dump as soon as that call ends; a 10-frame first dump does not wait for a 1,280-frame one
        of the same chunk. Streams without a dump in the chunk are served by the first job."""
        torch = self.torch
        if not self.cuda:  # a stand-in engine: decode now, deliver in order through the same thread
            pcm, err = self._decode(dumps)

            def job():
                self._deliver(pcm, order, ready)
                if err is not None:
                    raise err
            self.deliverer.put(None, job)
            return
        groups = sorted(self._groups(dumps), key=lambda g: g[0])
        if not groups:
            self.deliverer.put(None, lambda: self._deliver([], order, ready))
            return
        from . import _lib
        dev = self.engine.device
        gi = {i: g for g, (_, grp) in enumerate(groups) for i in grp}
        last = {}  # stream -> the group whose job delivers its items
        for st in ready:
            idx = [gi[v] for kind, v in order[st] if kind == "audio"]
            last[st] = max(idx) if idx else 0
        to_bytes, nd = self.to_bytes, len(dumps)
        pcm: List[object] = [None] * nd  # filled by the jobs, in order
        for g, (L, grp) in enumerate(groups):
            host = torch.empty(len(grp) * 320 * L, dtype=torch.float32, pin_memory=True)
            err_h = torch.zeros((1,), dtype=torch.int32, pin_memory=True)
            codes = torch.tensor([dumps[i][1] for i in grp], dtype=torch.int32).pin_memory()
            with torch.cuda.stream(self.codec_stream):
                out = self.engine.decode_codes(codes.to(dev, non_blocking=True))
                host.view(out.shape).copy_(out, non_blocking=True)
                err_d = torch.zeros((1,), dtype=torch.int32, device=dev)
                self.engine.take_errors(_lib.ERRW_CODEC, err_d)
                err_h.copy_(err_d, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.codec_stream)
            sts = [st for st in ready if last[st] == g]

            def deliver(host=host, err_h=err_h, grp=grp, L=L, sts=sts, codes=codes):  # (codes: kept alive)
                # a set codec error word fails this group's streams only: the
                # other streams of the job, and the other groups' jobs, are still delivered
                exc = None
                try:
                    _lib.check_bits(int(err_h[0]))
                except _lib.LvxError as e:
                    exc = self._codec_failure(e, [dumps[i][0] for i in grp])
                if exc is None:
                    for k, i in enumerate(grp):
                        a = host[k * 320 * L:(k + 1) * 320 * L].numpy()
                        pcm[i] = a.tobytes() if to_bytes else a.copy()
                self._deliver(pcm, order, sts)
                if exc is not None:
                    raise exc

            self.deliverer.put(ev, deliver)

    def flush(self):
        """Complete every chunk in flight and deliver everything queued."""
        while self.inflight:
            self._complete(self.inflight.popleft())
        if self.deliverer is not None:
            self.deliverer.wait()
            self.deliverer.take_error()

    def run_until_idle(self, max_chunks: int = 1 << 30) -> int:
        total = 0
        for _ in range(max_chunks):
            n = self.run_chunk()
            if n == 0:
                break
            total += n
        self.flush()
        return total
