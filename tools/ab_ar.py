"""In-process A/B of AR step variants (development tool): python tools/ab_ar.py opt v0 v1 ..."""
import os, sys, time
import torch
from llmvox_amd.engine import build_engine

opt = sys.argv[1]
vals = [int(v) for v in sys.argv[2:]] or [0, 1]
e = build_engine(0, "bf16", "bf16", max_streams=max(8, int(os.environ.get("AB_B", "1"))), max_positions=2048, max_codec_frames=256)
dev = e.device
B, stride, n = int(os.environ.get("AB_B", "1")), 512, 256
plan = torch.full((B, stride), 100, dtype=torch.int32, device=dev)
slots = torch.arange(B, dtype=torch.int32, device=dev)
rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
tok = torch.zeros((B, stride), dtype=torch.int32, device=dev)
res = {v: [] for v in vals}
toks = {}
for rep in range(4):
    for v in vals:
        e.set_option(opt, v)
        e.reset_slot(0); rowstep.zero_()
        e.ar_steps(16, slots, plan, rowstep, tok)  # capture + warm
        torch.cuda.synchronize()
        e.reset_slot(0); rowstep.zero_()
        t0 = time.perf_counter()
        e.ar_steps(n, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) / n * 1e6)
        toks[v] = tok[0, :n].clone()
for v in vals:
    print(f"{opt}={v}: us/step min {min(res[v]):.1f} med {sorted(res[v])[len(res[v])//2]:.1f}  same_tokens={bool((toks[v]==toks[vals[0]]).all())}")
