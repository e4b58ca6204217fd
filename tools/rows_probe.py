"""Development check: are equal batch rows bit-identical for each B / kernel variant?"""
import numpy as np, torch
from llmvox_amd.engine import build_engine
g = np.load("tests/golden/ar_golden.npz")
text = g["text_ids"].tolist()
e = build_engine(0, "bf16", "bf16", max_streams=8, max_positions=1024, max_codec_frames=512)
dev = e.device
for opt, vals in (("fuse_mlp", (0, 1)), ("cproj_b1", (0, 1))):
    for v in vals:
        e.set_option(opt, v)
        for B in (1, 2, 3, 4):
            for n in (1, 8):
                plan = torch.full((B, n), 384, dtype=torch.int32); plan[:, :len(text[:n])] = torch.tensor(text[:n], dtype=torch.int32)
                plan = plan.to(dev); slots = torch.arange(B, dtype=torch.int32, device=dev)
                rowstep = torch.zeros(B, dtype=torch.int32, device=dev); tok = torch.zeros(B, n, dtype=torch.int32, device=dev)
                for s in range(B): e.reset_slot(s)
                e.ar_steps(n, slots, plan, rowstep, tok)
                lg = e.last_logits(B).cpu().numpy()
                d = max(float(np.abs(lg[b] - lg[0]).max()) for b in range(B))
                print(f"{opt}={v} B={B} n={n} max row diff {d:.3g}")
    e.set_option(opt, 1)
