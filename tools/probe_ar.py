"""Quick timing probe of the AR step and codec decode (development tool)."""
import sys, time
import torch
from llmvox_amd.engine import build_engine

wd = sys.argv[1] if len(sys.argv) > 1 else "bf16"
e = build_engine(0, wd, wd, max_streams=64, max_positions=2048, max_codec_frames=1280)
dev = e.device
for B in (1, 32):
    stride = 1024
    plan = torch.full((B, stride), 100, dtype=torch.int32, device=dev)
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
    tok = torch.zeros((B, stride), dtype=torch.int32, device=dev)
    for s in range(B):
        e.reset_slot(s)
    e.ar_steps(8, slots, plan, rowstep, tok)
    torch.cuda.synchronize()
    for s in range(B):
        e.reset_slot(s)
    rowstep.zero_()
    t0 = time.perf_counter()
    e.ar_steps(512, slots, plan, rowstep, tok)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{wd} B={B}: {dt/512*1e6:.1f} us/step, {B*512/dt:.0f} tok/s", flush=True)
for L in (10, 256, 1280):
    codes = torch.randint(0, 4096, (1, L), device=dev)
    e.decode_codes(codes)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        e.decode_codes(codes)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"{wd} codec L={L}: {dt*1e3:.2f} ms, {320*L/dt/1e6:.2f} Msamples/s", flush=True)
