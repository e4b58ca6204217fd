"""Development probe: do independent decode chains overlap on one GPU once every chain's stream is
checked to run beside the others (llmvox_amd.streams.side_stream)? Round 1's multi_chain_probe used
unchecked pool streams. Each chain is its own engine on its own stream; all run 256 AR steps from
position P0 concurrently (HIP graph replay). Prints us per step of the whole group and tokens/s.
usage: python tools/chain_overlap_probe.py P0 'n x B' ...   e.g. 384 1x32 2x16 1x16 4x8"""
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from llmvox_amd.engine import build_engine  # noqa: E402
from llmvox_amd.streams import side_stream  # noqa: E402

P0 = int(sys.argv[1])
specs = [tuple(int(x) for x in s.split("x")) for s in sys.argv[2:]]
N = 256
maxn = max(n for n, _ in specs)
maxb = max(b for _, b in specs)
dev = torch.device("cuda", 0)
streams = []
for _ in range(maxn):
    streams.append(side_stream(dev, [None] + streams))
engines = [build_engine(0, "bf16", "bf16", max_streams=maxb, max_positions=P0 + 512, max_codec_frames=64)
           for _ in range(maxn)]


def run(n, B):
    bufs = []
    for e, s in zip(engines[:n], streams):
        with torch.cuda.stream(s):
            plan = torch.full((B, P0 + N), 100, dtype=torch.int32, device=dev)
            slots = torch.arange(B, dtype=torch.int32, device=dev)
            rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
            tok = torch.zeros(B, P0 + N, dtype=torch.int32, device=dev)
            bufs.append((plan, slots, rowstep, tok))
    ts = []
    for rep in range(4):
        for e, s, (plan, slots, rowstep, tok) in zip(engines, streams, bufs):
            with torch.cuda.stream(s):
                for b in range(B):
                    e.set_slot(b, P0, 5)
                rowstep.zero_()
                if rep == 0:
                    e.ar_steps(16, slots, plan, rowstep, tok)
                    for b in range(B):
                        e.set_slot(b, P0, 5)
                    rowstep.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for e, s, (plan, slots, rowstep, tok) in zip(engines, streams, bufs):
            with torch.cuda.stream(s):
                e.ar_steps(N, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    for e in engines[:n]:
        e.check_errors()
    dt = statistics.median(ts[1:])
    print(f"P0={P0} {n} chain(s) x B = {B:2d}: {dt / N * 1e6:7.1f} us per group step  "
          f"{n * B * N / dt:9.0f} tok/s  (reps {', '.join(f'{t / N * 1e6:.1f}' for t in ts)})", flush=True)


for n, B in specs:
    run(n, B)
