"""The persistent dataflow decode step (ar_persist_kernel: one launch per step at 17 <= B <= 32, bf16
weights + bf16 KV) against the 26-launch batched path it replaces (option
persist = 0). Every task runs the launch path's arithmetic in the same order, so tokens, margins
and logits must agree bit for bit, with permuted slots, ragged positions, partly filled 16-row
batch tiles and KV histories crossing 64-position chunks; and the headline mode must still hold
the reference's ids (teacher-forced bounds of test_gpu_teacher_forced.py run on this path)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(e, order, texts, prefix_rows, n_prefix, n_main):
    dev = e.device
    B = len(order)
    n = n_prefix + n_main
    for s in range(e.max_streams):
        e.reset_slot(s)
    out_tok = np.full((B, n), -1, dtype=np.int32)
    out_m = np.zeros((B, n), dtype=np.float32)
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
    plan = torch.from_numpy(texts[order, :n].copy()).to(dev)
    slots = torch.tensor(order, dtype=torch.int32, device=dev)
    rowstep = torch.tensor([n_prefix if r in prefix_rows else 0 for r in order], dtype=torch.int32, device=dev)
    tok = torch.zeros(B, n, dtype=torch.int32, device=dev)
    marg = torch.zeros(B, n, dtype=torch.float32, device=dev)
    e.ar_steps(n_main, slots, plan, rowstep, tok, marg)
    e.check_errors()
    t, mg = tok.cpu().numpy(), marg.cpu().numpy()
    lg = e.last_logits(B).cpu().numpy()
    for i, r in enumerate(order):
        s0 = n_prefix if r in prefix_rows else 0
        out_tok[i, s0:s0 + n_main] = t[i, s0:s0 + n_main]
        out_m[i, s0:s0 + n_main] = mg[i, s0:s0 + n_main]
    inv = np.argsort(order)
    return out_tok[inv], out_m[inv], lg[inv]


@pytest.fixture(scope="module")
def eng():
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", "bf16", max_streams=40, max_positions=1024, max_codec_frames=256)
    e.set_option("persist", 1)
    yield e
    e.set_option("persist", 0)
    e.close()


@pytest.mark.parametrize("B", [17, 24, 32])
def test_persistent_step_bit_identical_to_launch_path(eng, B):
    rng = np.random.default_rng(B)
    texts = rng.integers(3, 384, size=(B, 160)).astype(np.int32)
    order = list(rng.permutation(B))
    prefix = set(range(0, B, 3))
    res = []
    for opt in (1, 0):
        eng.set_option("persist", opt)
        res.append(_run(eng, order, texts, prefix, 37, 110))
    eng.set_option("persist", 1)
    for k, what in enumerate(("tokens", "margins", "logits")):
        np.testing.assert_array_equal(res[0][k], res[1][k], err_msg=what)


def test_persistent_step_repeatable(eng):
    """two runs of the same batch: bit-equal (no arrival-order arithmetic anywhere in the step)"""
    B = 32
    rng = np.random.default_rng(77)
    texts = rng.integers(3, 384, size=(B, 96)).astype(np.int32)
    a = _run(eng, list(range(B)), texts, set(), 0, 96)
    b = _run(eng, list(range(B)), texts, set(), 0, 96)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_persistent_step_many_launches_state_reset(eng):
    """~600 consecutive persistent launches (graph replays of 16 steps and single steps): the
    dependency counters are re-zeroed by every launch, so the last steps still match the launch path"""
    B = 20
    rng = np.random.default_rng(5)
    texts = rng.integers(3, 384, size=(B, 640)).astype(np.int32)
    res = []
    for opt in (1, 0):
        eng.set_option("persist", opt)
        res.append(_run(eng, list(range(B)), texts, set(), 0, 601))
    eng.set_option("persist", 1)
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][2], res[1][2])
