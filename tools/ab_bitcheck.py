"""Development check: an option A/B (lvx_set_option) must leave the decode bit-identical: tokens,
margins and final logits of N steps from position 0, bf16 weights + bf16 KV.
usage: python tools/ab_bitcheck.py OPT VALUE [B ...]   (LVX_AB_W=fp32: fp32 weights + fp32 KV, the parity mode;
LVX_AB_KV=fp8: bf16 weights with the fp8 KV cache)"""
import os
import sys
import torch
from llmvox_amd.engine import build_engine

opt, val = sys.argv[1], int(sys.argv[2])
Bs = [int(x) for x in sys.argv[3:]] or [4, 16, 17, 24, 32]
W = os.environ.get("LVX_AB_W", "bf16")
KV = os.environ.get("LVX_AB_KV", W)
e = build_engine(0, W, KV, max_streams=max(Bs), max_positions=1024, max_codec_frames=256)
e.set_option("fuse_mlp", 0)  # the fused MLP (B <= 2) adds with fp32 atomics: run-to-run noise
dev = e.device
n = 320
torch.manual_seed(0)
bad = 0
for B in Bs:
    plan = torch.randint(3, 380, (B, n), dtype=torch.int32, device=dev)
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    res = []
    for v in (0, val):
        e.set_option(opt, v)
        for s in range(B):
            e.reset_slot(s)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        tok = torch.zeros(B, n, dtype=torch.int32, device=dev)
        mar = torch.zeros(B, n, dtype=torch.float32, device=dev)
        e.ar_steps(n, slots, plan, rowstep, tok, mar)
        lg = e.last_logits(B)
        torch.cuda.synchronize()
        e.check_errors()
        res.append((tok.cpu(), mar.cpu(), lg.cpu()))
    e.set_option(opt, 0)
    same = all(torch.equal(a, b) for a, b in zip(*res))
    extra = ""
    if not same:  # how far apart: token agreement and the final logits
        (t0, _, l0), (t1, _, l1) = res
        extra = (f" (tokens equal {float((t0 == t1).float().mean()):.4f}, first differing step "
                 f"{int((t0 != t1).any(0).float().argmax()) if (t0 != t1).any() else -1}, "
                 f"max |dlogit| {float((l0 - l1).abs().max()):.3g} of max |logit| {float(l0.abs().max()):.3g})")
    print(f"B={B:2d} {opt}={val}: {'bit-identical' if same else 'DIFFERENT'}{extra}", flush=True)
    bad += not same
sys.exit(1 if bad else 0)
