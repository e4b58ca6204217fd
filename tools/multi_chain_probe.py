"""Development probe: do independent decode chains overlap on one GPU inside one process?
Each chain is its own engine (own weights, KV pool and scratch) on its own HIP stream; all run
256 AR steps from position 0 concurrently. Prints speech tokens/s for 1 chain of B rows vs
n chains of B/n rows. usage: python tools/multi_chain_probe.py"""
import sys
import time

import torch

sys.path.insert(0, ".")
from llmvox_amd.engine import build_engine  # noqa: E402

N = 256
engines = [build_engine(0, "bf16", "bf16", max_streams=32, max_positions=512, max_codec_frames=64)
           for _ in range(4)]
dev = engines[0].device
streams = [torch.cuda.Stream(device=dev) for _ in engines]


def run(n_chains, B):
    bufs = []
    for e, s in zip(engines[:n_chains], streams):
        with torch.cuda.stream(s):
            plan = torch.full((B, N), 100, dtype=torch.int32, device=dev)
            slots = torch.arange(B, dtype=torch.int32, device=dev)
            rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
            tok = torch.zeros(B, N, dtype=torch.int32, device=dev)
            bufs.append((plan, slots, rowstep, tok))
    best = None
    for rep in range(3):
        for (e, s), (plan, slots, rowstep, tok) in zip(zip(engines, streams), bufs):
            with torch.cuda.stream(s):
                for b in range(B):
                    e.reset_slot(b)
                rowstep.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for (e, s), (plan, slots, rowstep, tok) in zip(zip(engines, streams), bufs):
            with torch.cuda.stream(s):
                e.ar_steps(N, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if rep and (best is None or dt < best):  # rep 0 captures the graphs
            best = dt
    for e in engines[:n_chains]:
        e.check_errors()
    tps = n_chains * B * N / best
    print(f"{n_chains} chain(s) x B = {B:2d}: {best / N * 1e6:7.1f} us/step  {tps:9.0f} tok/s", flush=True)


for n, B in [(1, 1), (2, 1), (4, 1), (1, 2), (1, 4), (4, 8), (1, 8), (2, 16), (1, 32), (4, 4), (1, 16)]:
    run(n, B)
