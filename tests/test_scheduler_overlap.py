"""FusedScheduler's overlapped schedule (AR run-ahead by one chunk, rollback of a run-ahead row after an
end-of-audio, delivery by the delivery thread) on a CPU stand-in engine: every stream receives exactly
the items of the serial schedule, in the same order (reference semantics: streaming_server.py:357-422)."""
import numpy as np
import pytest

from llmvox_amd import streaming as S
from test_service_multidevice import StateEngine

TEXTS = ["The quick brown fox jumps over the lazy dog near the river bank.",
         "Hello there, how are you today? Fine.", "One sentence. Two sentences. Three.",
         "a b c d e f g h i j k l m n o p q r s t u v w x y z.", "Short."]


def _run(overlap, max_chunk, eoa, n_streams=5):
    eng = StateEngine(max_streams=8, max_positions=4096, eoa=eoa)
    sch = S.FusedScheduler(eng, max_chunk=max_chunk, to_bytes=False, overlap=overlap,
                           stop_rule=lambda st, ntok, pos: ntok >= 700)  # (without end of audio: no idle)
    sts = []
    for i in range(n_streams):
        st = sch.open_stream(index=i % 2, dump_size=10 if i % 2 == 0 else 160, eoa_id=eoa or 453)
        for w in TEXTS[i % len(TEXTS)].split(" "):
            st.feed(w)
        sts.append(st)
    # both schedules run to idle (every text spoken to its end), so their whole event lists compare
    # (a common-prefix comparison would pass an overlap that drops trailing items)
    assert sch.run_until_idle(max_chunks=5000) > 0
    assert sch.run_chunk() == 0 and not sch.inflight
    out = []
    for st in sts:
        ev = [("pcm", x.astype(int).tolist()) if isinstance(x, np.ndarray) else ("sig", x) for x in st.events]
        out.append((ev, list(st.tokens)))
    sch.close()
    return out


@pytest.mark.parametrize("max_chunk", [7, 16, 64])
@pytest.mark.parametrize("eoa", [None, 4000])
def test_overlap_delivers_the_serial_items(max_chunk, eoa):
    """eoa 4000: the stand-in emits it at every position divisible by 41, so segments end mid-chunk
    and the run-ahead rows of those streams are rolled back."""
    ser = _run(False, max_chunk, eoa)
    ovl = _run(True, max_chunk, eoa)
    assert len(ser) == len(ovl)
    for (ev_s, tok_s), (ev_o, tok_o) in zip(ser, ovl):
        assert len(ev_s) >= 2
        assert ev_o == ev_s
        assert tok_o == tok_s
    if eoa is not None:
        assert any(k == "sig" for ev, _ in ser for k, _ in ev)  # segments did end


def test_overlap_stop_rule_never_plans_past_a_stop():
    """A stream that the rule stops after its in-flight chunk is not planned by the run-ahead: it
    consumes exactly the tokens of the serial schedule."""
    got = []
    for overlap in (False, True):
        eng = StateEngine(max_streams=4)
        sch = S.FusedScheduler(eng, max_chunk=8, to_bytes=False, overlap=overlap,
                               stop_rule=lambda st, ntok, pos: ntok >= 30)
        st = sch.open_stream(index=0, dump_size=10)
        for w in TEXTS[0].split(" "):
            st.feed(w)
        sch.run_until_idle(max_chunks=100)
        got.append(list(st.tokens))
        sch.close()
    assert len(got[0]) == 34  # chunks 8 + 2 (dump at 10) + 8 + 8 + 8: the first count >= 30
    assert got[1] == got[0]


@pytest.mark.parametrize("seed", range(6))
def test_consume_many_equals_per_token_consume(seed):
    """The batched consume path gives the events, state and stop point of consume() token by token."""
    rng = np.random.default_rng(seed)
    words = TEXTS[seed % len(TEXTS)].split(" ") * 3
    a = S.SegmentMachine(index=seed % 2, dump_size=int(rng.choice([4, 10, 160])), eoa_id=453)
    b = S.SegmentMachine(index=seed % 2, dump_size=a.dump_size, eoa_id=453)
    for w in words:
        a.feed(w)
        b.feed(w)
    for _ in range(60):
        n = int(rng.integers(1, 40))
        toks = rng.integers(0, 4096, size=n)
        if rng.random() < 0.15:
            toks[rng.integers(0, n)] = 453
        if a.next_text_id() is None:
            break
        ev_a, used = a.consume_many(toks.tolist())
        ev_b = []
        for t in toks.tolist()[:used]:
            ev_b += b.consume(t)
        assert used == n or any(e.kind == "signal" for e in ev_a)
        assert [(e.kind, e.tokens, e.signal) for e in ev_a] == [(e.kind, e.tokens, e.signal) for e in ev_b]
        assert (a.speech_outputs, a.dump_size, a.gen_index, list(a.pending), list(a.words), a.end_of_speech) == \
            (b.speech_outputs, b.dump_size, b.gen_index, list(b.pending), list(b.words), b.end_of_speech)
