"""Constructed near-tie logits for the greedy select (streaming_server.py:342-346: the reference takes
argmax(softmax(logits)) on the CPU in fp32, first index on equal probabilities).

``tie_rule`` restates what that select does without the softmax: probabilities are equal exactly when
exp(x - max) rounds to 1.0f, i.e. x - max >= -2^-25, so the pick is the first such index. It is
checked against torch itself (tests/test_select_rule.py) before the GPU selects are checked against
both (tests/test_gpu_select.py)."""
from __future__ import annotations

import numpy as np

TIE = np.float32(2.0 ** -25)


def tie_rule(row) -> int:
    x = np.asarray(row, dtype=np.float32)
    m = x.max()
    return int(np.nonzero((x - m) >= -TIE)[0][0])


def near_tie_rows(n_rows: int, seed: int = 0, vocab: int = 4096) -> np.ndarray:
    """Rows whose maximum has rivals 0..6 ulps (and up to ~3 x 2^-25) below it, placed before and
    after it, with maxima of magnitude 0.003..20 (their ulp spans 2^-32..2^-19) and exact ties."""
    rng = np.random.default_rng(seed)
    out = np.empty((n_rows, vocab), dtype=np.float32)
    for r in range(n_rows):
        m = np.float32(rng.choice([0.003, 0.01, 0.1, 0.3, 0.45, 0.7, 1.0, 3.0, 7.9, 20.0, -0.4, -2.0])
                       * rng.uniform(0.8, 1.2))
        row = (rng.standard_normal(vocab) * rng.uniform(0.1, 3.0) + m - rng.uniform(0.5, 6.0)).astype(np.float32)
        row = np.minimum(row, np.float32(m - np.float32(1e-3)))
        j = int(rng.integers(0, vocab))
        row[j] = m
        ulp = np.float32(np.spacing(np.abs(m)))
        kmax = max(2, int(3 * TIE / ulp) + 2)
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(0, vocab))
            if i == j:
                continue
            c = m
            for _ in range(int(rng.integers(0, kmax + 1))):
                c = np.nextafter(c, np.float32(-np.inf), dtype=np.float32)
            row[i] = c
        out[r] = row
    return out
