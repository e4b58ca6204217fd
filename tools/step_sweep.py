"""us per AR step (HIP graph replay, all kernels) at positions [P0, P0+256) for B streams under
option sets; each config measured 3 times (median).
usage: python tools/step_sweep.py B P0 'opt=v,...' ['opt=v' ...]
LVX_SWEEP_STREAM=1: run on a torch side stream (the library then replays 16-step HIP graphs; on the
default (null) stream it launches every kernel). LVX_SWEEP_KV=fp8: fp8 KV cache (configs[4]).
LVX_SWEEP_W=fp32: the fp32 parity mode (fp32 weights and KV)."""
import os, statistics, sys, time
import torch
from llmvox_amd.engine import build_engine

B, P0 = int(sys.argv[1]), int(sys.argv[2])
WD = os.environ.get("LVX_SWEEP_W", "bf16")
e = build_engine(0, WD, "fp32" if WD == "fp32" else os.environ.get("LVX_SWEEP_KV", "bf16"), max_streams=B, max_positions=P0 + 512, max_codec_frames=256)
dev = e.device
plan = torch.full((B, P0 + 256), 100, dtype=torch.int32, device=dev)
slots = torch.arange(B, dtype=torch.int32, device=dev)
tok = torch.zeros(B, P0 + 256, dtype=torch.int32, device=dev)
side = torch.cuda.Stream(device=dev) if os.environ.get("LVX_SWEEP_STREAM") == "1" else None
if side is not None:
    torch.cuda.set_stream(side)
for spec in sys.argv[3:] or [""]:
    opts = [kv.split("=") for kv in spec.split(",") if kv]
    for k, v in opts:
        e.set_option(k, int(v))
    ts = []
    for rep in range(3):
        for s in range(B):
            e.set_slot(s, P0, 5)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        e.ar_steps(16, slots, plan, rowstep, tok)  # warm / capture
        torch.cuda.synchronize()
        for s in range(B):
            e.set_slot(s, P0, 5)
        rowstep.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.ar_steps(256, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / 256 * 1e6)
    us = statistics.median(ts)
    print(f"B={B} P={P0}.. [{spec}]: {us:7.1f} us/step  {B / us * 1e6:9.0f} tok/s", flush=True)
    for k, v in opts:
        e.set_option(k, {"bt": 1, "defer_select": 1, "fuse_mlp": 1, "codec_g2": 1, "codec_g3": 1, "codec_skinny": 1, "f32b": 1, "ln_max": 8, "l0q": 1}.get(k, 0))
