"""The multi-GPU exchange on RCCL itself (reference: the two replicas'
text in and PCM out, streaming_server.py:162-169,241-244,521-534). A one-rank NCCL (= RCCL on ROCm)
process group is created in this process (an in-process store, no rendezvous, no re-launch), and the
code the 8-GPU run takes goes through it on device tensors:

* bench.run_chunks with the async PCM gather (parallel.ChunkGather: the gather on its own communicator
  stream, issued once the host has seen the codec event, completion polled with Work.is_completed())
  gives tokens and PCM bit-identical to dist=None, and what the gather delivered equals each chunk's
  local PCM;
* the synchronous gather of the serial schedule, the same;
* scatter_plans / scatter_texts / gather_bytes on device tensors return exactly what was sent.
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.fixture(scope="module")
def rccl():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    try:
        yield dist
    finally:
        torch.cuda.synchronize()
        dist.destroy_process_group()


def _plans(S, utt, n_utt):
    import bench
    rng = np.random.default_rng(77)
    plans = np.zeros((S, n_utt * utt), dtype=np.int32)
    for g in range(S):
        for u in range(n_utt):
            ids = bench.sentence_ids(bench.SENTENCE if (g == 0 and u == 0) else bench.random_sentence(rng))
            plans[g, u * utt:(u + 1) * utt] = bench.plan_for(ids, 0, utt)
    return plans


def test_scatter_and_gather_on_device_tensors(rccl):
    from llmvox_amd.parallel import gather_bytes, gather_pcm, scatter_plans, scatter_texts
    dev = torch.device("cuda:0")
    full = torch.from_numpy(_plans(3, 64, 2))
    mine = scatter_plans(full, 3, full.shape[1], dev, rccl, 0)
    assert mine.device.type == "cuda" and torch.equal(mine.cpu(), full)
    texts = ["The quick brown fox.", "", "naïve café — ünïcödé ✓"]
    assert scatter_texts(texts, 3, dev, rccl, 0, 1) == texts
    items = [b"", bytes(range(256)) * 3, np.arange(1001, dtype=np.float32).tobytes()]
    got = gather_bytes(items, dev, rccl, 0, 1)
    assert got == [items]
    pcm = torch.randn(3, 320 * 16, device=dev)
    out = gather_pcm(pcm, rccl, 0, 1)
    assert len(out) == 1 and torch.equal(out[0], pcm)
    out, work = gather_pcm(pcm, rccl, 0, 1, async_op=True)
    assert work is not None
    work.wait()
    torch.cuda.synchronize()
    assert torch.equal(out[0], pcm)


@pytest.mark.parametrize("overlap", [True, False])
def test_run_chunks_through_rccl_equals_local(rccl, overlap):
    import bench
    from llmvox_amd.engine import build_engine
    S, chunk, K, reset_every = 4, 64, 4, 2
    eng = build_engine(0, "bf16", "bf16", max_streams=S, max_positions=8192, max_codec_frames=S * chunk)
    prev = torch.cuda.current_stream()
    torch.cuda.set_stream(torch.cuda.Stream())  # graph replay, as bench.py runs
    try:
        mine = torch.from_numpy(_plans(S, reset_every * chunk, K // reset_every)).to(eng.device)
        recs, gathered = {}, []
        for d in (None, rccl):
            rec = []
            bench.run_chunks(eng, mine, S, chunk, K, 1, reset_every, dist=d, rank=0, world=1,
                             codec_overlap=overlap, record=rec, gathered=gathered if d is not None else None)
            torch.cuda.synchronize()
            recs[d is not None] = [(t.cpu(), p.cpu()) for t, p in rec]
        assert len(recs[False]) == len(recs[True]) == K
        for c, ((tl, pl), (tr, pr)) in enumerate(zip(recs[False], recs[True])):
            assert torch.equal(tl, tr), f"chunk {c}: tokens differ with the RCCL group"
            assert torch.equal(pl, pr), f"chunk {c}: PCM differs with the RCCL group"
            assert pl.abs().max() > 0
        if overlap:
            # every timed chunk's PCM reached rank 0 through the async gather, in issue order
            assert len(gathered) == K
            for c, g in enumerate(gathered):
                assert len(g) == 1 and torch.equal(g[0], recs[True][c][1]), f"chunk {c}: gathered PCM differs"
        else:
            assert gathered == []
    finally:
        torch.cuda.set_stream(prev)
        eng.close()
