"""The headline's overlapped schedule (bench.run_chunks with codec_overlap: chunk c's codec on a second
HIP stream beside chunk c + 1's decode, host-paced, tokens / PCM double-buffered) produces bit for bit
the tokens and PCM of the serial schedule (codec after each chunk's decode on one stream). VERDICT r04
"what's weak" 6: the driver times only this schedule, and the buffer pacing is where a race would hide."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _plans(S, utt, n_utt):
    import bench
    rng = np.random.default_rng(1234)
    plans = np.zeros((S, n_utt * utt), dtype=np.int32)
    for g in range(S):
        for u in range(n_utt):
            ids = bench.sentence_ids(bench.SENTENCE if (g == 0 and u == 0) else bench.random_sentence(rng))
            plans[g, u * utt:(u + 1) * utt] = bench.plan_for(ids, 0, utt)
    return plans


@pytest.mark.parametrize("dtype,kv", [("bf16", "bf16"), ("bf16", "fp8")])
def test_overlapped_bench_schedule_equals_serial(dtype, kv):
    import bench
    from llmvox_amd.engine import build_engine
    S, chunk, K, reset_every = 4, 64, 4, 2
    eng = build_engine(0, dtype, kv, max_streams=S, max_positions=8192, max_codec_frames=S * chunk)
    prev = torch.cuda.current_stream()
    torch.cuda.set_stream(torch.cuda.Stream())  # graph replay, as bench.py runs
    try:
        mine = torch.from_numpy(_plans(S, reset_every * chunk, K // reset_every)).to(eng.device)
        recs = {}
        for overlap in (False, True):
            rec = []
            bench.run_chunks(eng, mine, S, chunk, K, 1, reset_every, codec_overlap=overlap, record=rec)
            torch.cuda.synchronize()
            recs[overlap] = [(t.cpu(), p.cpu()) for t, p in rec]
        assert len(recs[False]) == len(recs[True]) == K
        for c, ((ts, ps), (to, po)) in enumerate(zip(recs[False], recs[True])):
            assert torch.equal(ts, to), f"chunk {c}: tokens differ"
            assert torch.equal(ps, po), f"chunk {c}: PCM differs"
            assert ps.abs().max() > 0
        # the utterance reset every 2 chunks restarts each stream's sentence: chunk 2 repeats chunk 0
        # only for streams whose second utterance is the same text (none here), so just check the
        # chunks are not all identical (the reset / plan columns moved)
        assert not torch.equal(recs[False][0][0], recs[False][1][0])
    finally:
        torch.cuda.set_stream(prev)
        eng.close()
