"""Profile target: codec decodes of S streams x L frames (run under rocprofv3).
argv: wdtype L S [option=value ...]"""
import sys
import torch
from llmvox_amd.engine import build_engine
wd = sys.argv[1] if len(sys.argv) > 1 else "bf16"
L = int(sys.argv[2]) if len(sys.argv) > 2 else 256
S = int(sys.argv[3]) if len(sys.argv) > 3 else 1
e = build_engine(0, wd, wd, max_streams=2, max_positions=64, max_codec_frames=max(S * L, 256))
for kv in sys.argv[4:]:
    k, v = kv.split("=")
    e.set_option(k, int(v))
codes = torch.randint(0, 4096, (S, L), device=e.device)
for _ in range(3):
    e.decode_codes(codes)
torch.cuda.synchronize()
print("done")
