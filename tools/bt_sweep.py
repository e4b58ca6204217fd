"""Sweep the batched-path options: us per AR step at positions 256..511 for several B."""
import itertools, sys, time
import torch
from llmvox_amd.engine import build_engine

e = build_engine(0, "bf16", "bf16", max_streams=64, max_positions=1024, max_codec_frames=256)
dev = e.device
Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,16,32,64").split(",")]
configs = [dict(bt=0)] + [dict(bt=1, bt_rows=r, bt_merge=m) for r, m in itertools.product([16, 32], [0, 1])]
for B in Bs:
    plan = torch.full((B, 512), 100, dtype=torch.int32, device=dev)
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    tok = torch.zeros(B, 512, dtype=torch.int32, device=dev)
    for cfg in configs:
        if cfg["bt"] == 0 and B > 32:
            continue
        for k, v in cfg.items():
            e.set_option(k, v)
        for s in range(B):
            e.reset_slot(s)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        e.ar_steps(256, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.ar_steps(256, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / 256 * 1e6
        print(f"B={B:3d} {cfg}: {us:7.1f} us/step  {B / us * 1e6:9.0f} tok/s", flush=True)
e.set_option("bt", 1)
