"""Batched bf16 decode path (3 <= B <= 64, MFMA GEMMs with fused LayerNorm / merge prologues).

Rows are independent streams: a row's result may depend on B (the attention split count is sized
by B) but never on which batch row or KV slot carries it, nor on what the other rows hold. The
permutation tests check exactly that, bit for bit, with distinct texts and ragged positions
(catches any row/slot mix-up). Numerics against the fp32 oracle use the bf16 tolerance of
test_gpu_bf16.py; the v3 path is also held against the previous batched path (option bt=0).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", params=[1, 2], ids=["default", "v3-all-B"])
def eng(request):
    """default options (v2 for B <= 32, v3 above) and v3 forced for every batched B"""
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", "bf16", max_streams=64, max_positions=512, max_codec_frames=256)
    e.set_option("bt", request.param)
    e.bt_mode = request.param
    yield e
    e.close()


def _texts(B, n, seed=7):
    rng = np.random.default_rng(seed)
    return rng.integers(3, 384, size=(B, n)).astype(np.int32)


def _run(e, order, texts, prefix_rows, n_prefix, n_main, between=None):
    """Rows `order` (text index per batch row) in slots `order`; the rows whose text index is in
    prefix_rows first run n_prefix steps alone (ragged positions), then all rows n_main steps
    (`between` is called before the main phase)."""
    dev = e.device
    B = len(order)
    n = n_prefix + n_main
    for s in range(e.max_streams):
        e.reset_slot(s)
    out_tok = np.zeros((B, n), dtype=np.int32)
    out_tok[:] = -1
    pre = [i for i, r in enumerate(order) if r in prefix_rows]
    if pre:
        Bp = len(pre)
        plan = torch.from_numpy(texts[[order[i] for i in pre], :n].copy()).to(dev)
        slots = torch.tensor([order[i] for i in pre], dtype=torch.int32, device=dev)
        rowstep = torch.zeros(Bp, dtype=torch.int32, device=dev)
        tok = torch.zeros(Bp, n, dtype=torch.int32, device=dev)
        e.ar_steps(n_prefix, slots, plan, rowstep, tok)
        t = tok.cpu().numpy()
        for j, i in enumerate(pre):
            out_tok[i, :n_prefix] = t[j, :n_prefix]
    if between is not None:
        between()
    plan = torch.from_numpy(texts[order, :n].copy()).to(dev)
    slots = torch.tensor(order, dtype=torch.int32, device=dev)
    rowstep = torch.tensor([n_prefix if r in prefix_rows else 0 for r in order], dtype=torch.int32, device=dev)
    tok = torch.zeros(B, n, dtype=torch.int32, device=dev)
    e.ar_steps(n_main, slots, plan, rowstep, tok)
    e.check_errors()
    t = tok.cpu().numpy()
    lg = e.last_logits(B).cpu().numpy()
    for i, r in enumerate(order):
        s0 = n_prefix if r in prefix_rows else 0
        out_tok[i, s0:s0 + n_main] = t[i, s0:s0 + n_main]
    # back to text order
    inv = np.argsort(order)
    return out_tok[inv], lg[inv]


@pytest.mark.parametrize("B", [5, 32, 37, 64])
def test_rows_are_independent_of_batch_position(eng, B):
    texts = _texts(B, 64)
    prefix = set(range(0, B, 2))  # >= 3 rows: the B <= 2 fused MLP adds in arrival order
    order = list(range(B))
    tok_a, lg_a = _run(eng, order, texts, prefix, 20, 12)
    rng = np.random.default_rng(B)
    perm = rng.permutation(B).tolist()
    tok_b, lg_b = _run(eng, perm, texts, prefix, 20, 12)
    np.testing.assert_array_equal(tok_a, tok_b)
    np.testing.assert_array_equal(lg_a, lg_b)


@pytest.mark.parametrize("B", [8, 32, 48])
def test_v3_close_to_v2_batched_path(eng, B):
    """Same v3 prefix (ragged, multi-split attention), then one step on v3 vs on the v2 path."""
    texts = _texts(B, 80, seed=3)
    order = list(range(B))
    pre = set(range(0, B, 2))
    eng.set_option("bt", 2)
    _, lg3 = _run(eng, order, texts, pre, 70, 1)
    try:
        _, lg2 = _run(eng, order, texts, pre, 70, 1, between=lambda: eng.set_option("bt", 0))
    finally:
        eng.set_option("bt", eng.bt_mode)
    assert np.abs(lg3 - lg2).max() < 0.03 * np.abs(lg2).max()


@pytest.mark.parametrize("B", [3, 16, 48])
def test_first_step_matches_fp32_oracle_per_row(eng, B):
    from llmvox_amd import weights as LW
    from oracle import reference_cpu as R
    gw, cw, tt = LW.synthetic_all(1234)
    W = R.to_torch(gw)
    table = torch.from_numpy(tt)
    texts = _texts(B, 4, seed=11)
    _, lg = _run(eng, list(range(B)), texts, set(), 0, 1)
    for b in range(0, B, max(1, B // 6)):
        x = R.build_input(table[int(texts[b, 0])].view(1, 1, -1), torch.zeros(1, 1, 512))
        ref, _ = R.gpt_forward(W, x, None)
        ref = ref.reshape(-1).numpy()
        assert np.abs(lg[b] - ref).max() < 0.03 * np.abs(ref).max(), b


@pytest.mark.parametrize("B", [16, 32])
def test_v3_path_agrees_with_v2(eng, B):
    """The batched path v3 (one kernel per op: option bt = 2 at B <= 32) computes the same step as
    v2 after a shared ragged prefix, within bf16 rounding (the cross-check of the two paths)."""
    texts = _texts(B, 80, seed=13)
    order = list(range(B))
    pre = set(range(0, B, 2))
    eng.set_option("bt", 1)
    try:
        _, ref = _run(eng, order, texts, pre, 40, 1)
        _, got = _run(eng, order, texts, pre, 40, 1, between=lambda: eng.set_option("bt", 2))
    finally:
        eng.set_option("bt", eng.bt_mode)
    assert np.abs(got - ref).max() < 0.02 * np.abs(ref).max()


@pytest.mark.parametrize("B,kv", [(8, "bf16"), (8, "fp8"), (6, "bf16")])
def test_rows_structure_at_small_b(B, kv):
    """Option ln_max below B runs a small batch on the rows-kernel structure (rows kernel + c_attn
    + 16-row-tile GEMMs) instead of the GEMMs that normalise in their own prologue: another
    summation order, so the logits agree to bf16 rounding and the tokens where the margin allows.
    (Layer 0's c_attn as the GEMM on both sides, option l0q 0: the tables are held to it in
    test_layer0_tables_agree_with_the_gemm.)"""
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", kv, max_streams=64, max_positions=512, max_codec_frames=256)
    try:
        e.set_option("fuse_mlp", 0)
        e.set_option("l0q", 0)
        texts = _texts(B, 64, seed=21)
        order = list(np.random.default_rng(B + 7).permutation(B))
        res = []
        for lm in (8, 4):
            e.set_option("ln_max", lm)
            res.append(_run(e, order, texts, set(range(0, B, 3)), 16, 1))
        e.set_option("ln_max", 8)
        e.set_option("fuse_mlp", 1)
        ref, got = res[0][1], res[1][1]
        assert np.abs(got - ref).max() < 0.02 * np.abs(ref).max()
    finally:
        e.close()


@pytest.mark.parametrize("B,kv", [(4, "bf16"), (8, "fp8"), (9, "bf16"), (16, "bf16"), (32, "bf16"), (32, "fp8")])
def test_layer0_tables_agree_with_the_gemm(B, kv):
    """Layer 0's c_attn from the q0 tables with the select (ar_q0_rows_kernel, option l0q, B >= 4)
    against the c_attn GEMM (B > 8: after the embedding kernel; 4 <= B <= 8: the GEMM whose prologue
    commits the select from lm_head's granules and builds the embedding rows), after a shared ragged
    prefix: the same step up to
    the GEMM's bf16 rounding of the LayerNorm'd operand (the tables multiply it unrounded), so the
    logits agree within the bf16 path's bound, every row's state advances alike, and one step's
    tokens agree wherever the margin exceeds twice the logit difference."""
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", kv, max_streams=32, max_positions=512, max_codec_frames=256)
    try:
        texts = _texts(B, 64, seed=29)
        order = list(np.random.default_rng(B + 3).permutation(B))
        pre = set(range(0, B, 3))
        res = []
        for q in (0, 1):  # the prefix on the GEMM form both times: one step apart
            e.set_option("l0q", 0)
            res.append(_run(e, order, texts, pre, 24, 1, between=lambda q=q: e.set_option("l0q", q)))
        (t0, ref), (t1, got) = res
        col = np.array([24 if r in pre else 0 for r in range(B)])  # the main step's column (text order)
        np.testing.assert_array_equal(t1[:, :24][col == 24], t0[:, :24][col == 24])  # same prefix
        d = np.abs(got - ref).max()
        # bf16 KV: bf16 rounding; fp8 KV: a k / v value that moves by rounding can land on the next e4m3
        # step, so the fp8 mode's own bound (0.15 against the reference, test_gpu_teacher_forced.py)
        assert d < (0.02 if kv == "bf16" else 0.06) * np.abs(ref).max(), d
        srt = np.sort(ref, axis=1)
        sure = (srt[:, -1] - srt[:, -2]) > 2 * d
        assert sure.any()
        main0, main1 = t0[np.arange(B), col], t1[np.arange(B), col]
        np.testing.assert_array_equal(main1[sure], main0[sure])
    finally:
        e.set_option("l0q", 1)
        e.close()


@pytest.mark.parametrize("S", [12, 20])
def test_fragment_packed_rows_with_odd_engine_size(S):
    """max_streams not a multiple of 16: the fragment-packed operand rows (xn, xb, hb) are
    written and read in whole 16-row tiles, so the engine allocates them rounded up to 16 rows. The S
    streams of an S-slot engine must decode bit for bit as the same streams in a 32-slot engine (rows
    are independent of the engine's size and of their batch position), and nothing may fault. (Round 6:
    the row-major operand rows this was compared with, option exp bit 4, were removed.)"""
    from llmvox_amd.engine import build_engine
    texts = _texts(S, 64, seed=S)
    order = list(np.random.default_rng(S).permutation(S))
    res = []
    for slots in (S, 32):
        e = build_engine(0, "bf16", "bf16", max_streams=slots, max_positions=256, max_codec_frames=256)
        try:
            e.set_option("fuse_mlp", 0)
            res.append(_run(e, order, texts, set(range(0, S, 3)), 20, 36))
        finally:
            e.close()
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])


@pytest.mark.parametrize("B", [8, 32])
def test_table_path_idle_row_and_batch_composition(B):
    """The default bf16 path (layer 0 from the q0 tables inside the select launch, ar_q0_rows_kernel)
    with an idle row (slot -1) in the batch, over several lvx_ar_steps calls replayed as graphs on a
    side stream: the idle row's plan step and token buffer stay untouched, and the live rows' tokens
    and last logits are bit-equal to the same rows decoded without the idle row (B - 1 rows: the rows
    are independent of the batch they run in)."""
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", "bf16", max_streams=B, max_positions=256, max_codec_frames=64)
    dev = e.device
    texts = _texts(B, 40, seed=41)
    idle = B // 2
    calls = [3, 17, 1, 16]
    n = sum(calls)

    def run(slots):
        for s in range(B):
            e.reset_slot(s)
        plan = torch.from_numpy(texts[[max(s, 0) for s in slots], :n].copy()).to(dev)
        st = torch.tensor(slots, dtype=torch.int32, device=dev)
        rowstep = torch.zeros(len(slots), dtype=torch.int32, device=dev)
        tok = torch.full((len(slots), n), -7, dtype=torch.int32, device=dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for c in calls:
                e.ar_steps(c, st, plan, rowstep, tok)
            e.check_errors()
            lg = e.last_logits(len(slots))
        torch.cuda.current_stream(dev).wait_stream(side)
        return tok.cpu().numpy(), rowstep.cpu().numpy(), lg.cpu().numpy()

    try:
        with_idle = list(range(B))
        with_idle[idle] = -1
        tok_i, rs_i, lg_i = run(with_idle)
        live = [s for s in range(B) if s != idle]
        tok_l, rs_l, lg_l = run(live)
    finally:
        e.close()
    assert rs_i[idle] == 0 and (tok_i[idle] == -7).all()
    rows = [b for b in range(B) if b != idle]
    assert (rs_i[rows] == n).all() and (rs_l == n).all()
    np.testing.assert_array_equal(tok_i[rows], tok_l)
    np.testing.assert_array_equal(lg_i[rows], lg_l)
