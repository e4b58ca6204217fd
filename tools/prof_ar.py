"""Profile target: fixed AR steps + codec decodes (run under rocprofv3)."""
import sys
import torch
from llmvox_amd.engine import build_engine

wd = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
e = build_engine(0, wd, wd, max_streams=64, max_positions=2048, max_codec_frames=1280)
dev = e.device
stride = 512
plan = torch.full((B, stride), 100, dtype=torch.int32, device=dev)
slots = torch.arange(B, dtype=torch.int32, device=dev)
rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
tok = torch.zeros((B, stride), dtype=torch.int32, device=dev)
e.ar_steps(256, slots, plan, rowstep, tok)
codes = torch.randint(0, 4096, (1, 256), device=dev)
for _ in range(3):
    e.decode_codes(codes)
torch.cuda.synchronize()
print("done")
