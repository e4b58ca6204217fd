import numpy as np, torch
from llmvox_amd.engine import build_engine
g = np.load("tests/golden/ar_golden.npz")
text = g["text_ids"].tolist()
for kv in ("bf16", "fp8"):
    e = build_engine(0, "bf16", kv, max_streams=32, max_positions=1024, max_codec_frames=512)
    for B in (1, 2, 8):
        n = 32
        dev = e.device
        plan = torch.full((B, n), 384, dtype=torch.int32); plan[:, :len(text[:n])] = torch.tensor(text[:n], dtype=torch.int32)
        plan = plan.to(dev); slots = torch.arange(B, dtype=torch.int32, device=dev)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev); tok = torch.zeros(B, n, dtype=torch.int32, device=dev)
        for s in range(B): e.reset_slot(s)
        e.ar_steps(1, slots, plan, rowstep, tok)
        lg = e.last_logits(B).cpu().numpy()
        d0 = np.abs(lg[0] - g["logits"][0]).max() / np.abs(g["logits"][0]).max()
        e.ar_steps(n - 1, slots, plan, rowstep, tok)
        t = tok.cpu().numpy()
        agree = int(np.argmax(t[0] != g["ids"][:n])) if (t[0] != g["ids"][:n]).any() else n
        print(kv, B, "step0 rel dev %.4f" % d0, "agree_until", agree, "rows_equal", all((t[b] == t[0]).all() for b in range(B)))
    e.close()
