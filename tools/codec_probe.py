"""Codec decode timing (HIP events on the stream the decode runs on): batched 32 x 256 frames (the
configs[2] chunk), 1 x 256 (configs[1]) and 1 x 10 (the first dump). Also the PMC target of
tools/gpu_codec_pmc.sh. usage: python tools/codec_probe.py [reps] [dtype] [opt=v,...]"""
import sys

import torch

sys.path.insert(0, ".")
from llmvox_amd.engine import build_engine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dt = sys.argv[2] if len(sys.argv) > 2 else "bf16"
# dtype "fp8": bf16 context with fp8 codec weights (configs[4])
e = build_engine(0, "bf16" if dt == "fp8" else dt, "bf16" if dt == "fp8" else dt, max_streams=32, max_positions=64,
                 max_codec_frames=8192, codec_dtype="fp8" if dt == "fp8" else None)
opts = sys.argv[3] if len(sys.argv) > 3 else ""
for kv in filter(None, opts.split(",")):
    k, v = kv.split("=")
    e.set_option(k, int(v))
g = torch.Generator().manual_seed(0)
s = torch.cuda.current_stream()
CASES = ((32, 256), (1, 256), (2, 160), (1, 90), (1, 30), (1, 10))
if len(sys.argv) > 4:  # extra "BxL,BxL"
    CASES = tuple(tuple(int(v) for v in c.split("x")) for c in sys.argv[4].split(","))
for B, L in CASES:
    codes = torch.randint(0, 4096, (B, L), generator=g, dtype=torch.int32).to(e.device)
    out = torch.empty(B, 320 * L, device=e.device)
    e.decode_codes(codes, 0, out=out)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        e.decode_codes(codes, 0, out=out)
    b.record(s)
    b.synchronize()
    ms = a.elapsed_time(b) / reps
    fl = B * L * (125_566_976 + 3_072 * L)
    print(f"{dt} [{opts}] {B} x {L} frames: {ms:.3f} ms  {fl / ms / 1e9:.1f} TFLOP/s", flush=True)
e.check_errors()
