"""Codec decode time (ms) for S x L frames under option settings (HIP events, 10 reps)."""
import sys
import torch
from llmvox_amd.engine import build_engine
e = build_engine(0, "bf16", "bf16", max_streams=2, max_positions=64, max_codec_frames=16384)
cases = [(1, 10), (1, 256), (1, 1280), (8, 256), (32, 256), (64, 256)]
opts = [dict(codec_g2_min=1024), dict(codec_g2_min=1), dict(codec_g2=0)]
for S, L in cases:
    codes = torch.randint(0, 4096, (S, L), device=e.device)
    for o in opts:
        for k, v in o.items():
            e.set_option(k, v)
        e.decode_codes(codes)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            e.decode_codes(codes)
        b.record()
        b.synchronize()
        print(f"S={S:3d} L={L:5d} {o}: {a.elapsed_time(b) / 10:.3f} ms", flush=True)
        e.set_option("codec_g2", 1)
        e.set_option("codec_g2_min", 1024)
