"""Deferred greedy select (option "defer_select", B <= 2 GEMV step): lm_head leaves per-block
top1/top2 granules and the next step's c_attn layer 0 commits them (ar_select_final_kernel commits
the last step of each lvx_ar_steps call). The state it produces must be bit-identical to the
separate ar_argmax_kernel path (option off): tokens, margins, plan steps, slot positions and the
last logits, across graph replays (16-step graphs + 1-step graphs), eager launches, an idle row and
several calls in a row (the pending select never leaks across calls). The bf16 B <= 2 fused MLP
adds its partial sums in arrival order (fp32 atomics), so with it on two runs of the same path
differ in the last bits: bit-equality is checked with it off, and with it on tokens must agree
wherever the top1-top2 margin exceeds that noise.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["bf16", "fp32"])
def eng(request):
    from llmvox_amd.engine import build_engine
    e = build_engine(0, request.param, request.param, max_streams=4, max_positions=256, max_codec_frames=64)
    yield e
    e.close()


def _run(e, B, slots, calls, graphs):
    dev = e.device
    rng = np.random.default_rng(B * 31 + len(calls))
    n = sum(calls)
    plan = torch.from_numpy(rng.integers(3, 384, size=(B, n)).astype(np.int32)).to(dev)
    for s in range(4):
        e.reset_slot(s)
    st = torch.tensor(slots, dtype=torch.int32, device=dev)
    rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
    tok = torch.full((B, n), -7, dtype=torch.int32, device=dev)
    margin = torch.zeros(B, n, dtype=torch.float32, device=dev)
    e.set_graphs(graphs)
    # graphs are captured only on a non-default stream (the library launches the steps one by
    # one on the legacy null stream): the graph case runs on a stream of its own
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev) if graphs else None
    if side is not None:
        side.wait_stream(main)
    try:
        with torch.cuda.stream(side):
            for c in calls:
                e.ar_steps(c, st, plan, rowstep, tok, margin)
            e.check_errors()
            pos = [e.slot_position(s) for s in slots if s >= 0]
            logits = e.last_logits(B)
    finally:
        e.set_graphs(True)
    if side is not None:
        main.wait_stream(side)
    return tok.cpu().numpy(), margin.cpu().numpy(), rowstep.cpu().numpy(), pos, logits.cpu().numpy()


@pytest.mark.parametrize("fuse_mlp", [0, 1], ids=["exact", "fused-mlp"])
@pytest.mark.parametrize("graphs", [True, False], ids=["graphs", "eager"])
@pytest.mark.parametrize("B,slots", [(1, [2]), (2, [0, 3]), (2, [1, -1])], ids=["B1", "B2", "B2-idle"])
def test_deferred_select_matches_argmax_kernel(eng, B, slots, graphs, fuse_mlp):
    # (layer 0's c_attn as the GEMV on both paths, option l0q 0: with the q0 tables the select runs
    # in the embedding + select kernel, held to this form by test_small_b_tables_agree_with_the_gemv)
    calls = [3, 17, 1, 16]
    eng.set_option("fuse_mlp", fuse_mlp)
    eng.set_option("l0q", 0)
    try:
        eng.set_option("defer_select", 0)
        try:
            ref = _run(eng, B, slots, calls, graphs)
        finally:
            eng.set_option("defer_select", 1)
        got = _run(eng, B, slots, calls, graphs)
    finally:
        eng.set_option("fuse_mlp", 1)
        eng.set_option("l0q", 1)
    if fuse_mlp == 0 or eng.weight_dtype == "fp32":  # no arrival-order sums on this path
        live = [b for b, s in enumerate(slots) if s >= 0]  # (an idle row's logits are not outputs)
        for a, b, name in zip(got, ref, ["tokens", "margins", "rowstep", "positions", "logits"]):
            if name == "logits":
                a, b = a[live], b[live]
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b), err_msg=name)
    else:
        # a near-tie may flip a token, and the stream diverges from there: compare up to the
        # first step whose margin is within the noise, and the logits only if there is none
        tied = False
        for b, s in enumerate(slots):
            if s < 0:
                continue
            close = np.nonzero(ref[1][b] < 1e-3)[0]
            k = close[0] if len(close) else ref[0].shape[1]
            tied |= bool(len(close))
            np.testing.assert_array_equal(got[0][b, :k], ref[0][b, :k])
        np.testing.assert_array_equal(got[2], ref[2])
        assert got[3] == ref[3]
        if not tied:
            np.testing.assert_allclose(got[4], ref[4], atol=1e-3 * np.abs(ref[4]).max())
    tok, _, rowstep, pos, _ = got
    n = sum(calls)
    for b, s in enumerate(slots):
        if s >= 0:
            assert rowstep[b] == n and (tok[b] >= 0).all()
        else:
            assert rowstep[b] == 0 and (tok[b] == -7).all()
    assert pos == [n] * len(pos)


@pytest.fixture(scope="module")
def eng_batched():
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", "bf16", max_streams=48, max_positions=256, max_codec_frames=64)
    yield e
    e.close()


@pytest.mark.parametrize("B,ref_mode", [(4, 0), (8, 0), (32, 0), (48, 0), (4, 2), (5, 2), (8, 2)])
def test_batched_deferred_select_matches_argmax_kernel(eng_batched, B, ref_mode):
    """Batched steps (MFMA / v3 paths): the select runs in the next step's first kernel (4 <= B <= 8:
    c_attn layer 0 reduces lm_head's granules; larger B: the embedding rows kernel), ar_argmax_kernel
    after the last step. Against the argmax kernel after every lm_head (ref_mode 0) and, at B <= 8,
    against the embedding + select kernel (option defer_select 2). These paths have no arrival-order
    sums: bit-equal, with one idle row. (Layer 0's c_attn as the GEMM on every path, option l0q 0:
    the argmax-kernel path has no table form; the l0q kernel's select is this same code, held to
    the reference's picks by tests/test_gpu_teacher_forced.py at B = 32.)"""
    e = eng_batched
    e.set_option("l0q", 0)
    slots = list(range(B))
    slots[B // 2] = -1
    calls = [3, 17, 1, 16]

    def run():
        dev = e.device
        rng = np.random.default_rng(B)
        n = sum(calls)
        plan = torch.from_numpy(rng.integers(3, 384, size=(B, n)).astype(np.int32)).to(dev)
        for s in range(48):
            e.reset_slot(s)
        st = torch.tensor(slots, dtype=torch.int32, device=dev)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        tok = torch.full((B, n), -7, dtype=torch.int32, device=dev)
        margin = torch.zeros(B, n, dtype=torch.float32, device=dev)
        for c in calls:
            e.ar_steps(c, st, plan, rowstep, tok, margin)
        e.check_errors()
        pos = [e.slot_position(s) for s in slots if s >= 0]
        return tok.cpu().numpy(), margin.cpu().numpy(), rowstep.cpu().numpy(), pos, e.last_logits(B).cpu().numpy()

    e.set_option("defer_select", ref_mode)
    try:
        ref = run()
        e.set_option("defer_select", 1)
        got = run()
    finally:
        e.set_option("defer_select", 1)
        e.set_option("l0q", 1)
    live = [b for b in range(B) if b != B // 2]  # the idle row's logits are whatever its garbage x gives
    for a, b, name in zip(got, ref, ["tokens", "margins", "rowstep", "positions", "logits"]):
        if name == "logits":
            a, b = a[live], b[live]
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b), err_msg=name)
    n = sum(calls)
    assert got[2][B // 2] == 0 and (got[0][B // 2] == -7).all()
    assert all(got[2][b] == n for b in range(B) if b != B // 2)


@pytest.mark.parametrize("B,slots", [(1, [2]), (2, [0, 3]), (2, [1, -1])], ids=["B1", "B2", "B2-idle"])
def test_small_b_tables_agree_with_the_gemv(eng, B, slots):
    """B <= 2, bf16 (round 6): layer 0's c_attn from the q0 tables (ar_q0_gran_kernel: 9 blocks that
    each commit-reduce lm_head's granules and compute 256 of the 2,304 outputs) against the GEMV whose
    prologue does the same select before multiplying (option l0q 0), over several calls with graph
    replays and eager launches: the same state machine (plan steps, positions, idle rows untouched),
    the tokens equal up to the first step whose margin is within the noise (the two forms differ in
    fp32 rounding only: the GEMV multiplies the fp32 LayerNorm'd row), the graph replay bit-equal to
    the eager launches, and the logits within the bf16 bound."""
    if eng.weight_dtype != "bf16":
        pytest.skip("the q0 tables are a bf16-weight form")
    calls = [3, 17, 1, 16]
    eng.set_option("l0q", 0)
    try:
        ref = _run(eng, B, slots, calls, True)
    finally:
        eng.set_option("l0q", 1)
    got = _run(eng, B, slots, calls, True)
    eager = _run(eng, B, slots, calls, False)
    for a, b, name in zip(eager, got, ["tokens", "margins", "rowstep", "positions", "logits"]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b), err_msg=f"eager vs graphs: {name}")
    n = sum(calls)
    tied = False
    for b, s in enumerate(slots):
        if s < 0:
            assert got[2][b] == 0 and (got[0][b] == -7).all()
            continue
        assert got[2][b] == n and (got[0][b] >= 0).all()
        close = np.nonzero(ref[1][b] < 0.05)[0]
        k = close[0] if len(close) else n
        tied |= bool(len(close))
        np.testing.assert_array_equal(got[0][b, :k], ref[0][b, :k])
    assert got[3] == ref[3]
    if not tied:
        live = [b for b, s in enumerate(slots) if s >= 0]
        assert np.abs(got[4][live] - ref[4][live]).max() < 0.02 * np.abs(ref[4][live]).max()


@pytest.mark.parametrize("B,slots", [(1, [2]), (2, [0, 3]), (2, [1, -1])], ids=["B1", "B2", "B2-idle"])
def test_graph_replay_matches_eager(eng, B, slots):
    """16-step + 1-step graph replays on a side stream == the same steps launched one by one
    (deterministic path: fused MLP off)."""
    calls = [3, 17, 1, 16]
    eng.set_option("fuse_mlp", 0)
    try:
        eager = _run(eng, B, slots, calls, False)
        graph = _run(eng, B, slots, calls, True)
    finally:
        eng.set_option("fuse_mlp", 1)
    for a, b, name in zip(graph, eager, ["tokens", "margins", "rowstep", "positions", "logits"]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b), err_msg=name)


@pytest.mark.parametrize("B", [1, 4])
def test_kernel_probe_graphs(eng, B):
    """bench.py's roofline probe: every op's launches replay as one graph (captured on the
    context's own stream for a null-stream caller); the fused mlp c_proj reports LVX_E_STATE;
    the decode state stays valid."""
    from llmvox_amd._lib import LvxError
    dev = eng.device
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    for s in range(B):
        eng.set_slot(s, 100, 7)
    ran = 0
    for _ in range(2):  # capture, then replay the cached graph
        for k in range(6):
            try:
                eng.probe_kernel(k, slots, 20)
                ran += 1
            except LvxError as e:
                assert e.code == -2 and k == 4, (k, e.code)
    torch.cuda.synchronize()
    eng.check_errors()
    assert ran >= 10
    with pytest.raises(LvxError):
        eng.probe_kernel(6, slots, 20)


@pytest.mark.parametrize("path,B", [(0, 1), (0, 8), (1, 1), (1, 2), (1, 4), (2, 4), (2, 16), (3, 4), (3, 8)],
                         ids=["argmax-B1", "argmax-B8", "granules-B1", "granules-B2", "granules-B4",
                              "batched-B4", "batched-B16", "granules16-B4", "granules16-B8"])
def test_select_paths_reproduce_softmax_argmax(eng_batched, path, B):
    """Every production select path over constructed near-tie logits (rivals 0..6 ulps and up to
    3 x 2^-25 below the maximum, before and after it) picks what the reference's
    softmax -> argmax picks on the same fp32 logits (oracle greedy_token = torch CPU), and the
    margin is top1 - top2. Rows are committed as a decode step commits them."""
    from oracle import reference_cpu as R
    from tests.select_cases import near_tie_rows
    e = eng_batched
    dev = e.device
    picked, want = [], []
    for rep in range(12):
        rows = near_tie_rows(B, seed=1000 * path + 10 * B + rep)
        for s in range(B):
            e.set_slot(s, 5, 0)
        slots = torch.arange(B, dtype=torch.int32, device=dev)
        plan = torch.full((B, 4), 97, dtype=torch.int32, device=dev)
        rowstep = torch.ones(B, dtype=torch.int32, device=dev)
        tok = torch.full((B, 4), -7, dtype=torch.int32, device=dev)
        marg = torch.zeros(B, 4, dtype=torch.float32, device=dev)
        e.select_probe(path, slots, torch.from_numpy(rows), plan, rowstep, tok, marg)
        torch.cuda.synchronize()
        t, m, rs = tok.cpu().numpy(), marg.cpu().numpy(), rowstep.cpu().numpy()
        for b in range(B):
            ref = R.greedy_token(torch.from_numpy(rows[b]).view(1, 1, -1))
            top2 = np.sort(rows[b])[-2:]
            picked.append(int(t[b, 1]))
            want.append(ref)
            assert m[b, 1] == np.float32(top2[1] - top2[0])
            assert rs[b] == 2 and t[b, 0] == -7 and t[b, 2] == -7
        assert [e.slot_position(s) for s in range(B)] == [6] * B
    assert picked == want


@pytest.mark.parametrize("B", [4, 8])
def test_granule_select_fp8_kv_matches_embed_select(B):
    """configs[4]'s path (bf16 weights, fp8 KV, one 8-wave attention split): the 4 <= B <= 8 select
    folded into c_attn layer 0 (defer_select 1) against the embedding + select kernel (defer_select 2)
    and the argmax kernel after lm_head (0), across several lvx_ar_steps calls and graph replays on a
    side stream, with an idle row: tokens, margins, plan steps, positions and the live rows' logits
    bit-equal. (Layer 0's c_attn as the GEMM, option l0q 0: with the q0 tables the 4 <= B <= 8 select
    runs in ar_q0_rows_kernel, held to the GEMM form in
    tests/test_gpu_batched.py::test_layer0_tables_agree_with_the_gemm.)"""
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", "fp8", max_streams=8, max_positions=512, max_codec_frames=64)
    e.set_option("l0q", 0)
    dev = e.device
    slots = list(range(B))
    slots[1] = -1
    calls = [5, 16, 1, 33]
    n = sum(calls)

    def run():
        rng = np.random.default_rng(7 * B)
        plan = torch.from_numpy(rng.integers(3, 384, size=(B, n)).astype(np.int32)).to(dev)
        for s in range(8):
            e.reset_slot(s)
        st = torch.tensor(slots, dtype=torch.int32, device=dev)
        rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
        tok = torch.full((B, n), -7, dtype=torch.int32, device=dev)
        margin = torch.zeros(B, n, dtype=torch.float32, device=dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for c in calls:
                e.ar_steps(c, st, plan, rowstep, tok, margin)
            e.check_errors()
            pos = [e.slot_position(s) for s in slots if s >= 0]
            logits = e.last_logits(B)
        torch.cuda.current_stream(dev).wait_stream(side)
        return tok.cpu().numpy(), margin.cpu().numpy(), rowstep.cpu().numpy(), pos, logits.cpu().numpy()

    try:
        res = {}
        for mode in (2, 0, 1):
            e.set_option("defer_select", mode)
            res[mode] = run()
    finally:
        e.close()
    live = [b for b in range(B) if slots[b] >= 0]
    for ref in (2, 0):
        for a, b, name in zip(res[1], res[ref], ["tokens", "margins", "rowstep", "positions", "logits"]):
            if name == "logits":
                a, b = a[live], b[live]
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b), err_msg=f"{name} vs defer_select {ref}")
    assert res[1][2][1] == 0 and (res[1][0][1] == -7).all()
    assert all(res[1][2][b] == n for b in live)
