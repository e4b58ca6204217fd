"""Diagnostic: batched-path row determinism (same order twice, permuted order, with/without prefix)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
from test_gpu_batched import _run, _texts
from llmvox_amd.engine import build_engine

e = build_engine(0, "bf16", "bf16", max_streams=64, max_positions=512, max_codec_frames=256)
for B, pre_step, npre in [(32, 2, 20), (32, 0, 0), (16, 0, 0), (32, 2, 1), (8, 0, 0)]:
    texts = _texts(B, 64)
    prefix = set(range(0, B, pre_step)) if pre_step else set()
    order = list(range(B))
    ta, la = _run(e, order, texts, prefix, npre, 12)
    tb, lb = _run(e, order, texts, prefix, npre, 12)
    perm = np.random.default_rng(B).permutation(B).tolist()
    tc, lc = _run(e, perm, texts, prefix, npre, 12)
    rep = [r for r in range(B) if not np.array_equal(la[r], lb[r])]
    prm = [r for r in range(B) if not np.array_equal(la[r], lc[r])]
    print(f"B={B} prefix={sorted(prefix)[:4]}.. npre={npre}: repeat-diff rows {rep}, perm-diff rows {prm} "
          f"(perm pos {[perm.index(r) for r in prm]}), tok eq {np.array_equal(ta, tb)} {np.array_equal(ta, tc)}")
    for r in prm[:2]:
        d = np.abs(la[r] - lc[r])
        print("   row", r, "max diff", d.max(), "n diff", int((d > 0).sum()))
