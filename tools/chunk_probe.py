"""Development probe: B=1 AR chunk time (256 steps) vs starting position, and the bench-style loop."""
import time
import torch
from llmvox_amd.engine import build_engine

e = build_engine(0, "bf16", "bf16", max_streams=4, max_positions=8192, max_codec_frames=1024)
dev = e.device
n = 256
plan = torch.full((1, n), 100, dtype=torch.int32, device=dev)
slots = torch.zeros(1, dtype=torch.int32, device=dev)
rowstep = torch.zeros(1, dtype=torch.int32, device=dev)
tok = torch.zeros(1, n, dtype=torch.int32, device=dev)
e.reset_slot(0); e.ar_steps(n, slots, plan, rowstep, tok); torch.cuda.synchronize()
for p0 in (0, 256, 512, 768, 1024, 2048, 4096):
    ts = []
    for r in range(3):
        e.set_slot(0, p0, 5); rowstep.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.ar_steps(n, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"chunk at positions {p0}..{p0 + n - 1}: {min(ts):.3f} ms ({min(ts) / n * 1e3:.1f} us/step)")
