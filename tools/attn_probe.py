"""Development probe: the decode attention alone (lvx_probe_kernel op 1, HIP events) at several
KV positions for B = 1 and B = 32, bf16 KV. usage: python tools/attn_probe.py [reps]"""
import sys
import torch
from llmvox_amd.engine import build_engine

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
e = build_engine(0, "bf16", "bf16", max_streams=32, max_positions=4096, max_codec_frames=256)
s = torch.cuda.current_stream()
for B in (1, 32):
    slots = torch.arange(B, dtype=torch.int32, device=e.device)
    for t in (512, 1024, 2048, 4096):
        for b in range(B):
            e.set_slot(b, t - 1, 0)
        e.probe_kernel(1, slots, 5)
        best = 1e9
        for _ in range(3):
            a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            e.probe_kernel(1, slots, reps)
            c.record(s)
            c.synchronize()
            best = min(best, a.elapsed_time(c) * 1e3 / reps)
        gbs = B * 3072 * t / best / 1e3
        print(f"B={B:2d} t={t:5d} attention {best:7.2f} us  {gbs:7.0f} GB/s", flush=True)
