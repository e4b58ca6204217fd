"""Per-op timing of the decode step (HIP events, back-to-back launches) for several B and t."""
import sys
import torch
from llmvox_amd.engine import build_engine

wd = sys.argv[1] if len(sys.argv) > 1 else "bf16"
maxpos = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
e = build_engine(0, wd, wd, max_streams=64, max_positions=maxpos, max_codec_frames=256)
names = ["c_attn", "attn", "c_proj+merge", "c_fc", "mlp_proj", "lm_head"]
s = torch.cuda.current_stream()
for B in (1, 8, 32):
    slots = torch.arange(B, dtype=torch.int32, device=e.device)
    for t in (64, 256, 1024):
        for b in range(B):
            e.set_slot(b, t - 1, 0)
        row = []
        for k in range(6):
            e.probe_kernel(k, slots, 5)
            a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            e.probe_kernel(k, slots, 50)
            c.record(s)
            c.synchronize()
            row.append(a.elapsed_time(c) * 1e3 / 50)
        step = 4 * sum(row[:5]) + row[5]
        print(f"B={B:2d} t={t:4d} " + " ".join(f"{n}={v:6.2f}" for n, v in zip(names, row)) + f"  ~step={step:6.1f}us", flush=True)
