"""PMC target: bench.py's roofline probes (probe_kernels) on a small engine (KV capacity max(1024, POS)),
for rocprofv3 --pmc passes that segfault in the profiler on the full bench (large KV pool).
usage: python tools/probe_pmc.py STREAMS POS [kv_dtype]"""
import sys
import torch
sys.path.insert(0, ".")
from bench import probe_kernels
from llmvox_amd.engine import build_engine

S, P = int(sys.argv[1]), int(sys.argv[2])
kvd = sys.argv[3] if len(sys.argv) > 3 else "bf16"
e = build_engine(0, "bf16", kvd, max_streams=S, max_positions=max(1024, P), max_codec_frames=256)
slots = torch.arange(S, dtype=torch.int32, device=e.device)
for s in range(S):
    e.set_slot(s, P - 1, 0)
r = probe_kernels(e, slots, P, 2, {"bf16": 2, "fp8": 1}[kvd])
for v in r.values():
    print(f"{v['name']:34s} {v['avg_us']:7.2f} us {v['gbs']:8.1f} GB/s")
