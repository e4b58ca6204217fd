"""Development probe: B = 1 step time vs the engine's max_streams / max_positions (layout only)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from llmvox_amd.engine import build_engine  # noqa: E402

N = 256
for ms, mp in [(1, 8192), (1, 512), (32, 512), (32, 8192), (2, 512), (8, 512)]:
    e = build_engine(0, "bf16", "bf16", max_streams=ms, max_positions=mp, max_codec_frames=64)
    dev = e.device
    plan = torch.full((1, N), 100, dtype=torch.int32, device=dev)
    slots = torch.zeros(1, dtype=torch.int32, device=dev)
    rowstep = torch.zeros(1, dtype=torch.int32, device=dev)
    tok = torch.zeros(1, N, dtype=torch.int32, device=dev)
    best = 1e9
    for rep in range(3):
        e.reset_slot(0)
        rowstep.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.ar_steps(N, slots, plan, rowstep, tok)
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / N * 1e6)
    e.check_errors()
    print(f"max_streams {ms:2d} max_positions {mp:5d}: B = 1 {best:6.1f} us/step", flush=True)
    e.close()
    del e
    torch.cuda.empty_cache()
