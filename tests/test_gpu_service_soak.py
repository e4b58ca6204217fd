"""The service under concurrent load against the same requests served one at a time.

In the fp32 parity mode a stream's greedy tokens do not depend on which other streams share its
decode steps (every batch size runs the bit-exact fp32 step), so a request must get the same tokens
and the same dumps whether it runs alone or joins seven others at random moments of the chunk in
flight (admission between chunks, run-ahead rollback, slots reused across waves, codec calls grouped
with other requests' dumps). Only the tail may differ: a stream stops at the first chunk end past
max_tokens, and chunk ends depend on the other streams' dump points, so the last item (the decode of
the undumped tail) is excluded."""
import random
import threading

import numpy as np
import pytest

TEXTS = [
    "The quick brown fox. Jumps over the lazy dog.",
    "Streaming speech needs low latency. Every chunk counts.",
    "A second sentence follows the first. Then a third one ends it.",
    "Numbers like one two three are words too. They are spoken.",
    "Short one. Short two.",
    "Replica zero speaks this sentence. Replica one speaks the next.",
    "The weather is fine today. Tomorrow it may rain.",
    "Hello there, how are you doing. I am doing well, thanks.",
]


def _serve(svc, text, peak=None):
    s = svc.submit(text)
    if peak is not None:
        peak.append(len(svc.sessions))
    items = [bytes(x) for x in svc.chunks(s, timeout=0.01)]
    return items, [list(st.tokens) for st in s.streams]


def _compare(solo, conc, text):
    (ia, ta), (ib, tb) = solo, conc
    for k, (a, b) in enumerate(zip(ta, tb)):  # replica k's tokens: one greedy sequence (every text
        # has a sentence for each replica)
        n = min(len(a), len(b))
        assert n >= 64, (text, k, len(a), len(b))
        assert a[:n] == b[:n], (text, k)
    n = min(len(ia), len(ib)) - 1  # every item but each run's last (the tail decode)
    assert n >= 1, (text, len(ia), len(ib))
    for j in range(n):
        x, y = np.frombuffer(ia[j], np.float32), np.frombuffer(ib[j], np.float32)
        assert x.shape == y.shape, (text, j, x.shape, y.shape)
        assert np.abs(x - y).max() < 1e-5, (text, j)


@pytest.mark.gpu
def test_concurrent_requests_match_solo_requests():
    from llmvox_amd.engine import build_engine
    from llmvox_amd.server import TTSService
    eng = build_engine(0, "fp32", "fp32", max_streams=16, max_positions=512, max_codec_frames=16 * 256)
    svc = TTSService(eng, max_chunk=32, max_tokens=100)
    try:
        solo = {t: _serve(svc, t) for t in TEXTS}
        rng = random.Random(7)
        peak = []
        for wave in range(3):  # slots freed by one wave are reused by the next
            got, errs = {}, []

            def client(text, delay):
                try:
                    threading.Event().wait(delay)
                    got[text] = _serve(svc, text, peak)
                except BaseException as e:  # noqa: BLE001 (reported below)
                    errs.append((text, e))
            order = TEXTS[:]
            rng.shuffle(order)
            th = [threading.Thread(target=client, args=(t, rng.uniform(0.0, 0.04))) for t in order]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=120)
            assert not any(t.is_alive() for t in th), f"wave {wave}: a request did not finish"
            assert not errs, errs
            for t in TEXTS:
                _compare(solo[t], got[t], t)
            assert svc.sessions == [] and svc.error is None
        assert max(peak) >= 4, peak  # the requests did overlap
    finally:
        svc.shutdown()
        eng.close()
