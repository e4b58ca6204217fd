"""Development probe: per-step time of 256 AR steps launched one by one on the null stream, as
graph replays on a side stream, and launched one by one on a side stream (B = 1, 2, 32)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from llmvox_amd.engine import build_engine  # noqa: E402

N = 256
e = build_engine(0, "bf16", "bf16", max_streams=32, max_positions=512, max_codec_frames=64)
dev = e.device
side = torch.cuda.Stream(device=dev)
for B in (1, 2, 32):
    plan = torch.full((B, N), 100, dtype=torch.int32, device=dev)
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
    tok = torch.zeros(B, N, dtype=torch.int32, device=dev)
    res = {}
    for rep in range(3):
        for name, stream, graphs in [("null/launched", None, True), ("side/graphs", side, True),
                                     ("side/launched", side, False)]:
            e.set_graphs(graphs)
            with torch.cuda.stream(stream):
                for b in range(B):
                    e.reset_slot(b)
                rowstep.zero_()
                e.ar_steps(16, slots, plan, rowstep, tok)  # capture / warm
                for b in range(B):
                    e.reset_slot(b)
                rowstep.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                e.ar_steps(N, slots, plan, rowstep, tok)
                torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / N * 1e6
            res[name] = min(res.get(name, 1e9), us)
    e.set_graphs(True)
    print(f"B = {B:2d}: " + "  ".join(f"{k} {v:6.1f} us/step" for k, v in res.items()), flush=True)
e.check_errors()
