"""Stream sharding: rank 0 scatters text plans and gathers PCM (gloo, world size 2, CPU)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from llmvox_amd.parallel import gather_pcm, scatter_plans, shard_of
    S, n_pos = 3, 16
    full = torch.arange(world * S * n_pos, dtype=torch.int32).view(world * S, n_pos) if rank == 0 else None
    mine = scatter_plans(full, S, n_pos, "cpu", dist, rank)
    pcm = mine.float() * 2  # stand-in for this rank's decode
    got = gather_pcm(pcm, dist, rank, world)
    if rank == 0:
        q.put((torch.cat(got).tolist(), [shard_of(g, S) for g in range(world * S)]))
    dist.barrier()
    dist.destroy_process_group()


def test_scatter_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    gathered, shards = q.get(timeout=10)
    expect = (torch.arange(2 * 3 * 16, dtype=torch.float32).view(6, 16) * 2).tolist()
    assert gathered == expect
    assert shards == [0, 0, 0, 1, 1, 1]


def _worker_texts(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from llmvox_amd.parallel import gather_bytes, scatter_texts
    S = 2
    texts = [f"sentence {g}: caf\u00e9 " + "x" * (7 * g) + "." for g in range(world * S)] if rank == 0 else None
    mine = scatter_texts(texts, S, "cpu", dist, rank, world)
    # stand-in PCM of each stream: variable length, derived from its text
    pcm = [(t * (1 + rank)).encode("utf-8") + bytes(range(len(t) % 7)) for t in mine]
    got = gather_bytes(pcm, "cpu", dist, rank, world)
    if rank == 0:
        q.put((mine, got))
    else:
        q.put((mine, None))
    dist.barrier()
    dist.destroy_process_group()


def test_scatter_texts_gather_variable_bytes_world2():
    """configs[3]'s exchange (bench.py run_config3): rank 0 scatters the request texts, every rank
    returns its streams' variable-length PCM bytes to rank 0 (sizes first)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 7) % 1000
    ps = [ctx.Process(target=_worker_texts, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    texts = [f"sentence {g}: caf\u00e9 " + "x" * (7 * g) + "." for g in range(4)]
    mines = sorted(r[0] for r in res)
    assert mines == [texts[:2], texts[2:]]
    got = [r[1] for r in res if r[1] is not None][0]
    want = [[(t * (1 + r)).encode("utf-8") + bytes(range(len(t) % 7)) for t in texts[2 * r:2 * r + 2]] for r in range(2)]
    assert got == want
