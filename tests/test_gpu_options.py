"""Kernel options are per context: lvx_set_option on one engine must not change
another engine's kernels. Two engines on device 0; engine B decodes a stream in two calls while
engine A switches options (to a variant with another summation order) between them and decodes with
them: B's tokens, margins and logits must equal a clean run bit for bit, on the launch-by-launch
path (null stream) and on the HIP-graph replay path (a side stream), and A's results must show that
its option did take effect."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 48


def _engine():
    from llmvox_amd.engine import build_engine
    return build_engine(0, "bf16", "bf16", max_streams=4, max_positions=512, max_codec_frames=16)


def _run(e, texts, halves, between=None):
    """Decode N steps of stream 0 (B = 1: the fused-MLP path that option fuse_mlp switches) in
    `halves` calls; `between()` runs between the calls."""
    dev = e.device
    e.reset_slot(0)
    slots = torch.zeros(1, dtype=torch.int32, device=dev)
    toks, margs = [], []
    n = N // halves
    for h in range(halves):
        plan = texts[:, h * n:(h + 1) * n].contiguous()
        tok = torch.zeros(1, n, dtype=torch.int32, device=dev)
        marg = torch.zeros(1, n, dtype=torch.float32, device=dev)
        e.ar_steps(n, slots, plan, torch.zeros(1, dtype=torch.int32, device=dev), tok, marg)
        e.check_errors()
        toks.append(tok.cpu().numpy())
        margs.append(marg.cpu().numpy())
        if between is not None and h + 1 < halves:
            between()
    return np.concatenate(toks, 1), np.concatenate(margs, 1), e.last_logits(1).cpu().numpy()


@pytest.mark.parametrize("graphs", [False, True])
def test_option_on_one_engine_leaves_the_other_bit_identical(graphs):
    ea, eb = _engine(), _engine()
    rng = np.random.default_rng(7)
    texts = torch.from_numpy(rng.integers(3, 384, size=(1, N)).astype(np.int32)).to(ea.device)
    side = torch.cuda.Stream(device=ea.device) if graphs else None
    try:
        with torch.cuda.stream(side) if side is not None else torch.cuda.device(ea.device):
            ref = _run(eb, texts, 1)
            a_default = _run(ea, texts, 1)

            def switch_a():
                ea.set_option("fuse_mlp", 0)   # B <= 2: the two-kernel MLP (another summation order)
                ea.set_option("exp", 8)        # a batched fp32 variant (B's dtype and size never use it)
                ea.set_option("codec_exp", 1)
                _run(ea, texts, 2)             # A launches (and captures) with its own options

            got = _run(eb, texts, 2, between=switch_a)
            a_switched = _run(ea, texts, 1)
        torch.cuda.synchronize()
        for k in range(3):
            np.testing.assert_array_equal(got[k], ref[k])
        np.testing.assert_array_equal(a_default[2], ref[2])  # same default options: same bits
        assert not np.array_equal(a_switched[2], ref[2]), "engine A's option had no effect"
        # B still decodes with the defaults after A's change (its graphs were not flushed or mixed)
        again = _run(eb, texts, 1)
        for k in range(3):
            np.testing.assert_array_equal(again[k], ref[k])
    finally:
        ea.close()
        eb.close()
