"""The reference's greedy select (streaming_server.py:342-346, torch CPU fp32 softmax -> argmax) against
the closed-form tie rule the HIP selects implement (ar_kernels.hip softmax_ties): the pick is the first
index whose logit is within 2^-25 of the maximum. Pins the rule on this host's torch before the GPU
selects are checked against it (tests/test_gpu_select.py)."""
import numpy as np
import torch

from oracle import reference_cpu as R
from tests.select_cases import near_tie_rows, tie_rule


def test_rule_matches_torch_softmax_argmax_on_near_ties():
    rows = near_tie_rows(400, seed=11)
    picks = [R.greedy_token(torch.from_numpy(r).view(1, 1, -1)) for r in rows]
    assert picks == [tie_rule(r) for r in rows]
    # the cases do exercise the rule: some rows pick an index that is not the first maximum
    assert sum(p != int(np.argmax(r)) for p, r in zip(picks, rows)) >= 20


def test_rule_boundary_is_two_to_minus_25():
    base = np.full(4096, -5.0, dtype=np.float32)
    for m in (np.float32(0.1), np.float32(0.3)):
        ulp = np.spacing(m)
        for k in range(1, 8):
            x = base.copy()
            x[10] = m - np.float32(k * ulp)  # earlier index, k ulps below the maximum
            x[20] = m
            tied = float(m - x[10]) <= 2.0 ** -25
            got = R.greedy_token(torch.from_numpy(x).view(1, 1, -1))
            assert got == (10 if tied else 20), (m, k)
