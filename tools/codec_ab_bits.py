"""Bit-identity of the codec decode under an option change (development A/B): decodes the same codes
with option NAME at 0 and at VALUE and compares the PCM. usage: python tools/codec_ab_bits.py NAME VALUE [dtype]"""
import sys

import torch

sys.path.insert(0, ".")
from llmvox_amd.engine import build_engine  # noqa: E402

name, val = sys.argv[1], int(sys.argv[2])
dt = sys.argv[3] if len(sys.argv) > 3 else "bf16"
e = build_engine(0, dt, dt, max_streams=32, max_positions=64, max_codec_frames=8192)
g = torch.Generator().manual_seed(0)
for B, L in ((32, 256), (1, 256), (2, 160), (1, 90), (1, 10), (1, 1), (3, 7)):
    codes = torch.randint(0, 4096, (B, L), generator=g, dtype=torch.int32).to(e.device)
    e.set_option(name, 0)
    a = e.decode_codes(codes, 0).clone()
    e.set_option(name, val)
    b = e.decode_codes(codes, 0).clone()
    e.set_option(name, 0)
    print(f"{dt} {B} x {L}: {name}={val} vs 0: bit-equal {torch.equal(a, b)}  max|d| {(a - b).abs().max().item():.3e}", flush=True)
e.check_errors()
