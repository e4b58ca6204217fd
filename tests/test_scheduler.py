"""a12: dump / EOA / reset / control-signal semantics against traces of the reference's own
audio_generator_sync (tests/golden/sched_golden.json, scripted model + codec fakes)."""
import json
import os
import threading
from queue import Queue

import numpy as np
import pytest
import torch

from llmvox_amd import streaming as S
from llmvox_amd.tokenizer import ByteTokenizer

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TRACES = json.load(open(os.path.join(GOLDEN, "sched_golden.json")))


class _Stop(Exception):
    pass


class ScriptModel:
    def __init__(self, script):
        self.script, self.i = list(script), 0

    def __call__(self, emb, kvcache=None, targets=None):
        if self.i >= len(self.script):
            raise _Stop()
        tok = self.script[self.i]
        self.i += 1
        lg = torch.zeros(1, 1, 4096)
        lg[0, 0, tok] = 10.0
        return lg, None, (kvcache or []) + [emb.shape[1]]


class FakeWav:
    def codes_to_features(self, codes):
        if codes.dim() == 2:
            codes = codes.unsqueeze(1)
        f = torch.zeros(codes.shape[1], 512, codes.shape[2])
        f[:, 0, :] = codes[0].float()
        return f

    def decode(self, features, bandwidth_id=None):
        return features[:, 0, :].clone()


class FakeHandler:
    def __init__(self, script):
        self.device = torch.device("cpu")
        self.model = ScriptModel(script)
        self.wavtokenizer = FakeWav()
        self.llm_model = lambda ids: torch.zeros(1, ids.shape[1], 256)
        self.tokenizer = ByteTokenizer()


def _record(items):
    rec = []
    for it in items:
        if isinstance(it, (bytes, bytearray)):
            rec.append({"audio": np.frombuffer(it, dtype=np.float32).astype(int).tolist()})
        else:
            rec.append({"signal": it})
    return rec


@pytest.mark.parametrize("name", sorted(TRACES))
def test_dropin_generator_matches_reference_trace(name):
    tr = TRACES[name]
    h = FakeHandler(tr["script"])
    tq, aq = Queue(), Queue()
    for w in tr["words"]:
        tq.put(w)
    done = threading.Event()

    def body():
        try:
            S.audio_generator_sync(tr["index"], tr["dump_size"], h, tq, aq)
        except _Stop:
            pass
        finally:
            done.set()

    th = threading.Thread(target=body, daemon=True)
    th.start()
    # the reference blocks on the text queue when it runs out of words; so does the mirror
    done.wait(3.0)
    items = []
    while not aq.empty():
        items.append(aq.get())
    assert _record(items) == tr["items"]
    assert h.model.i == tr["model_calls"]


@pytest.mark.parametrize("name", sorted(TRACES))
def test_segment_machine_matches_reference_trace(name):
    tr = TRACES[name]
    m = S.SegmentMachine(index=tr["index"], dump_size=tr["dump_size"])
    for w in tr["words"]:
        m.feed(w)
    rec, calls = [], 0
    for tok in tr["script"]:
        if m.next_text_id() is None:
            break
        calls += 1
        for e in m.consume(tok):
            if e.kind == "audio":
                rec.append({"audio": list(e.tokens)})
            else:
                rec.append({"signal": e.signal})
    assert rec == tr["items"]
    assert calls == tr["model_calls"]


def test_plan_is_the_text_id_sequence():
    m = S.SegmentMachine(index=0, dump_size=10)
    for w in ["The", "quick", "bank."]:
        m.feed(w)
    plan = m.plan(30)
    t = ByteTokenizer()
    expect = t("The")["input_ids"] + t("quick")["input_ids"] + t("bank.")["input_ids"] + [385]
    assert plan[:len(expect)] == expect
    assert plan[len(expect):] == [384] * (30 - len(expect))
    got = []
    for _ in range(30):
        got.append(m.next_text_id())
        m.consume(7)
    assert got == plan


def test_plan_stops_when_text_missing():
    m = S.SegmentMachine(index=0, dump_size=10)
    m.feed("ab")
    assert m.plan(10) == [100, 101, 1]


def test_clean_text_and_routing():
    g = json.load(open(os.path.join(GOLDEN, "clean_text_golden.json")))
    for text, expect in g.items():
        assert S.clean_text(text) == expect, text
    q1, q2 = Queue(), Queue()
    S.route_text(["Hello", "world.", "", "-", "Next", "one.", "<|eot_id|>"], [q1, q2])
    assert [q1.get() for _ in range(q1.qsize())] == ["Hello", "world.", "<|eot_id|>"]
    assert [q2.get() for _ in range(q2.qsize())] == ["Next", "one."]


def test_audio_chunks_queue_switching():
    q1, q2 = Queue(), Queue()
    for it in [b"a", 1, b"x"]:
        q1.put(it)
    for it in [b"b", 0]:
        q2.put(it)
    q1.put("end")
    assert list(S.audio_chunks(q1, q2, timeout=0.05)) == [b"a", b"b", b"x"]


# ---- the fused scheduler's bookkeeping on a scripted engine (no GPU) ----------------------

class ScriptEngine:
    """Stands in for llmvox_amd.Engine: every ar_steps row gets the next tokens of its slot's
    script; decode_codes returns the codes as floats."""

    def __init__(self, scripts, max_streams=4):
        self.device = torch.device("cpu")
        self.max_streams = max_streams
        self.max_codec_frames = 4096
        self.scripts = {k: list(v) for k, v in scripts.items()}
        self.calls = {k: 0 for k in scripts}
        self.set_calls = []

    def reset_slot(self, slot):
        pass

    def set_slot(self, slot, pos, prev=0):
        self.set_calls.append((slot, pos))

    def ar_steps(self, n, slots, plan, rowstep, tok, margin=None):
        for r, s in enumerate(slots.tolist()):
            if s < 0:
                continue
            for j in range(n):
                i = self.calls[s]
                tok[r, j] = self.scripts[s][i] if i < len(self.scripts[s]) else 0
                self.calls[s] += 1

    def decode_codes(self, codes, bandwidth_id=0, out=None):
        return codes.float()

    def check_errors(self):
        pass


@pytest.mark.parametrize("name", ["eoa_mid", "dump_then_eoa", "eoa_exact_dump", "grow_dumps", "end_generation"])
def test_fused_scheduler_matches_reference_trace(name):
    tr = TRACES[name]
    eng = ScriptEngine({0: _consumed_script(tr)})
    sch = S.FusedScheduler(eng, max_chunk=7, to_bytes=False)
    st = sch.open_stream(index=tr["index"], dump_size=tr["dump_size"])
    for w in tr["words"]:
        st.feed(w)
    sch.run_until_idle(max_chunks=200)
    rec = []
    for it in st.events:
        if isinstance(it, np.ndarray):
            rec.append({"audio": it.astype(int).tolist()})
        else:
            rec.append({"signal": it})
    n = len(tr["items"])
    assert rec[:n] == tr["items"]


def _consumed_script(tr):
    """The fused scheduler runs ahead and rolls back after an end-of-audio: it consumes the
    same tokens as the reference, so give each slot exactly the reference's consumed tokens
    followed by filler that never ends a segment."""
    m = tr["model_calls"]
    return tr["script"][:m] + [5] * 400


def test_fused_scheduler_rewinds_after_eoa():
    eng = ScriptEngine({0: [3, 3, 453] + [4] * 300})
    sch = S.FusedScheduler(eng, max_chunk=16, to_bytes=False)
    st = sch.open_stream(index=0, dump_size=10)
    for w in ["abcdef."]:
        st.feed(w)
    sch.run_chunk()
    assert (0, 0) in eng.set_calls  # slot rewound to position 0 after the EOA at step 2
    assert st.events[-1] == 1  # replica 0 signals the switch to replica 1


def test_mirror_scheduler_on_oracle_reproduces_reference_stream():
    """Our audio_generator_sync mirror driving the CPU oracle reproduces the reference's own
    end-to-end stream (first 3 dumps: 10, 30, 90 tokens) bit for bit."""
    from llmvox_amd import weights as LW
    from oracle.scheduler_cpu import OracleHandler
    g = np.load(os.path.join(GOLDEN, "stream_golden.npz"))
    gw, cw, tt = LW.synthetic_all(1234)
    h = OracleHandler(gw, cw, tt, tokenizer=ByteTokenizer())
    real = h.model
    calls = {"n": 0}

    def counted(*a, **k):
        if calls["n"] >= int(g["model_calls"]):
            raise _Stop()
        calls["n"] += 1
        return real(*a, **k)

    h.model = counted
    tq, aq = Queue(), Queue()
    for w in "The quick brown fox jumps over the lazy dog near the river bank.".split(" "):
        tq.put(w)
    try:
        S.audio_generator_sync(0, 10, h, tq, aq)
    except _Stop:
        pass
    chunks = [np.frombuffer(aq.get(), dtype=np.float32) for _ in range(aq.qsize())]
    assert [len(c) for c in chunks] == g["sizes"].tolist()
    for i in range(3):
        np.testing.assert_array_equal(chunks[i], g[f"chunk{i}"])
