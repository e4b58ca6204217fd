"""Codec decode time (ms) for S x L frames under option sets (HIP events, 10 reps).
usage: python tools/codec_sweep.py 'S:L,S:L' 'opt=v,...' ['opt=v' ...]"""
import sys
import torch
from llmvox_amd.engine import build_engine
cases = [tuple(int(x) for x in c.split(":")) for c in (sys.argv[1] if len(sys.argv) > 1 else "1:256,32:256").split(",")]
e = build_engine(0, "bf16", "bf16", max_streams=2, max_positions=64, max_codec_frames=max(S * L for S, L in cases))
specs = sys.argv[2:] or [""]
DEFAULTS = {"codec_g2": 1, "codec_g2_min": 128, "codec_xcd": 1, "codec_bm256": 0}
for S, L in cases:
    codes = torch.randint(0, 4096, (S, L), device=e.device)
    for spec in specs:
        opts = [kv.split("=") for kv in spec.split(",") if kv]
        for k, v in opts:
            e.set_option(k, int(v))
        e.decode_codes(codes)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            e.decode_codes(codes)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / 10
        print(f"S={S:3d} L={L:5d} [{spec}]: {ms:.3f} ms  {S * L * (125_566_976 + 3072 * L) / ms / 1e9:.1f} TFLOP/s", flush=True)
        for k, v in opts:
            e.set_option(k, DEFAULTS.get(k, 0))
