"""Teacher-forced parity of the performance modes (bf16 weights + bf16 KV, bf16 + fp8 KV) against
the reference's 256 golden decode steps (tests/golden/ar_golden.npz, streaming_server.py:323-346).

Each step i runs the production fused decode step (lvx_ar_steps, the bench / server path) with the
slot rewound to position i and its previous token set to the REFERENCE's token i-1, so every step
sees the reference's history and errors cannot compound: step i's greedy pick is compared with the
reference's id i. Picks must agree wherever the reference's top1-top2 margin exceeds the mode's
logit error bound (stated per mode below); the agreement rate over all 256 steps is reported, and
the logits are compared with the reference's at the 8 recorded steps."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")

# max |logit - reference logit| allowed at the recorded steps, and the margin above which the pick
# must equal the reference's (2 x the logit bound: neither top-2 logit can cross the other)
BOUNDS = {("bf16", "bf16"): 0.03, ("bf16", "fp8"): 0.15}


# B: rows per step. B = 1 runs the single-stream kernels (configs[1]); B = 32 the batched MFMA path
# of the bench's default workload (configs[2]); B = 8 the fp8-KV batched path of configs[4]. Every
# row of a step gets the same teacher-forced history (its own slot), so all rows must also agree.
@pytest.mark.parametrize("wd,kvd,B", [("bf16", "bf16", 1), ("bf16", "bf16", 32), ("bf16", "fp8", 1), ("bf16", "fp8", 8)],
                         ids=["bf16-B1", "bf16-B32", "bf16-kvfp8-B1", "bf16-kvfp8-B8"])
def test_teacher_forced_256_steps(wd, kvd, B):
    from llmvox_amd.engine import build_engine
    g = np.load(os.path.join(GOLDEN, "ar_golden.npz"))
    ids, margins, text = g["ids"], g["margins"], g["text_ids"].tolist()
    n = len(ids)
    e = build_engine(0, wd, kvd, max_streams=B, max_positions=512, max_codec_frames=16)
    dev = e.device
    try:
        slots = torch.arange(B, dtype=torch.int32, device=dev)
        plan = torch.zeros(B, 2, dtype=torch.int32, device=dev)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        tok = torch.zeros(B, 2, dtype=torch.int32, device=dev)
        marg = torch.zeros(B, 2, dtype=torch.float32, device=dev)
        picks, gm, kept, rows_ok = [], [], {}, True
        keep = g["logit_steps"].tolist()
        for i in range(n):
            for b in range(B):
                e.set_slot(b, i, int(ids[i - 1]) if i > 0 else 0)
            plan.fill_(text[i] if i < len(text) else 384)
            rowstep.zero_()
            e.ar_steps(1, slots, plan, rowstep, tok, marg)
            if i in keep:
                lg = e.last_logits(B).cpu().numpy()
                kept[i] = lg[0]
                rows_ok &= bool(np.abs(lg - lg[0]).max() < 1e-5)
            picks.append(tok[:, 0].clone())
            gm.append(marg[0, 0].clone())
        e.check_errors()
        allp = torch.stack(picks).cpu().numpy()  # [n][B]
        picks = allp[:, 0]
        gm = torch.stack(gm).cpu().numpy()
    finally:
        e.close()
    bound = BOUNDS[(wd, kvd)]
    err = max(float(np.abs(kept[s] - g["logits"][k]).max()) for k, s in enumerate(keep))
    agree = float((picks == ids).mean())
    must = margins > 2 * bound
    print(f"\n[teacher-forced {wd}/kv {kvd} B={B}] agreement {agree:.4f} over {n} steps; "
          f"max |dlogit| at recorded steps {err:.4g} (bound {bound}); steps with margin > {2 * bound}: "
          f"{int(must.sum())}, mismatches there: {int((picks != ids)[must].sum())}; "
          f"mismatch steps {np.nonzero(picks != ids)[0].tolist()} (golden margins "
          f"{[round(float(margins[k]), 4) for k in np.nonzero(picks != ids)[0]]})")
    assert err < bound
    assert rows_ok and (allp == allp[:, :1]).all(), "rows with the same history disagree"
    np.testing.assert_array_equal(picks[must], ids[must])
    assert agree >= 0.95
