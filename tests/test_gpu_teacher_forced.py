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


def _teacher_forced(wd, kvd, B, ids, text, keep, max_positions):
    """Run len(ids) teacher-forced steps; returns (picks [n][B], logits at the `keep` steps (row 0),
    whether every row of a kept step agreed with row 0 to 1e-5)."""
    from llmvox_amd.engine import build_engine
    n = len(ids)
    e = build_engine(0, wd, kvd, max_streams=B, max_positions=max_positions, max_codec_frames=16)
    dev = e.device
    try:
        slots = torch.arange(B, dtype=torch.int32, device=dev)
        plan = torch.zeros(B, 2, dtype=torch.int32, device=dev)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        tok = torch.zeros(B, 2, dtype=torch.int32, device=dev)
        picks, kept, rows_ok = [], {}, True
        for i in range(n):
            for b in range(B):
                e.set_slot(b, i, int(ids[i - 1]) if i > 0 else 0)
            plan.fill_(text[i] if i < len(text) else 384)
            rowstep.zero_()
            e.ar_steps(1, slots, plan, rowstep, tok)
            if i in keep:
                lg = e.last_logits(B).cpu().numpy()
                kept[i] = lg[0]
                rows_ok &= bool(np.abs(lg - lg[0]).max() < 1e-5)
            picks.append(tok[:, 0].clone())
        e.check_errors()
        allp = torch.stack(picks).cpu().numpy()  # [n][B]
    finally:
        e.close()
    return allp, kept, rows_ok


def _check(tag, allp, kept, rows_ok, ids, margins, ref_logits, keep, bound):
    picks = allp[:, 0]
    n = len(ids)
    err = max(float(np.abs(kept[s] - ref_logits[k]).max()) for k, s in enumerate(keep))
    agree = float((picks == ids).mean())
    must = margins > 2 * bound
    print(f"\n[teacher-forced {tag}] agreement {agree:.4f} over {n} steps; "
          f"max |dlogit| at recorded steps {err:.4g} (bound {bound}); steps with margin > {2 * bound}: "
          f"{int(must.sum())}, mismatches there: {int((picks != ids)[must].sum())}; "
          f"mismatch steps {np.nonzero(picks != ids)[0].tolist()} (golden margins "
          f"{[round(float(margins[k]), 4) for k in np.nonzero(picks != ids)[0]]})")
    assert err < bound
    assert rows_ok and (allp == allp[:, :1]).all(), "rows with the same history disagree"
    np.testing.assert_array_equal(picks[must], ids[must])
    assert agree >= 0.95


# B: rows per step. B = 1 runs the single-stream kernels (configs[1]); B = 32 the batched MFMA path
# of the bench's default workload (configs[2]); B = 8 the fp8-KV batched path of configs[4]. Every
# row of a step gets the same teacher-forced history (its own slot), so all rows must also agree.
@pytest.mark.parametrize("wd,kvd,B", [("bf16", "bf16", 1), ("bf16", "bf16", 32), ("bf16", "fp8", 1), ("bf16", "fp8", 8)],
                         ids=["bf16-B1", "bf16-B32", "bf16-kvfp8-B1", "bf16-kvfp8-B8"])
def test_teacher_forced_256_steps(wd, kvd, B):
    g = np.load(os.path.join(GOLDEN, "ar_golden.npz"))
    ids, margins, text = g["ids"], g["margins"], g["text_ids"].tolist()
    keep = g["logit_steps"].tolist()
    allp, kept, rows_ok = _teacher_forced(wd, kvd, B, ids, text, keep, 512)
    _check(f"{wd}/kv {kvd} B={B}", allp, kept, rows_ok, ids, margins, g["logits"], keep, BOUNDS[(wd, kvd)])


# the bench's whole KV range: configs[2] decodes positions 0..1,023 of each utterance
# (16 KV chunks of 64 positions) in an engine of 8,192 positions per slot (the bench's layout). The
# reference's own stream (stream_long_golden.npz: its audio_generator_sync ids and top1-top2
# margins) is teacher-forced through position 1,023; logits are held against the reference's at
# positions 511 / 767 / 1,023 (ar_long_golden.npz) plus the first two recorded steps of ar_golden.
@pytest.mark.parametrize("wd,kvd,B", [("bf16", "bf16", 32), ("bf16", "fp8", 8), ("bf16", "bf16", 1)],
                         ids=["bf16-B32", "bf16-kvfp8-B8", "bf16-B1"])
def test_teacher_forced_through_position_1023(wd, kvd, B):
    lg = np.load(os.path.join(GOLDEN, "stream_long_golden.npz"))
    ll = np.load(os.path.join(GOLDEN, "ar_long_golden.npz"))
    g = np.load(os.path.join(GOLDEN, "ar_golden.npz"))
    n = 1024
    ids, margins, text = lg["ids"][:n], lg["margins"][:n], lg["text_ids"].tolist()
    np.testing.assert_array_equal(ll["ids"], ids)
    keep = g["logit_steps"].tolist()[:2] + ll["logit_steps"].tolist()
    ref = np.concatenate([g["logits"][:2], ll["logits"]])
    allp, kept, rows_ok = _teacher_forced(wd, kvd, B, ids, text, keep, 8192)
    _check(f"{wd}/kv {kvd} B={B}, positions 0..{n - 1}", allp, kept, rows_ok, ids, margins, ref, keep,
           BOUNDS[(wd, kvd)])
