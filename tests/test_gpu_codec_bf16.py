"""Codec decode in bf16 mode (bf16 weights and bf16 GEMM operands, fp32 accumulation and fp32
residual stream). No bit-exactness claim against the fp32 reference; the bar is a relative RMS
error of the waveform, measured against the fp32 parity-mode engine (itself pinned to the
reference's golden PCM by test_gpu_parity.py) and against the golden PCM directly. The large-M
GEMM (gemm_bf16_kernel, 128x128 tiles), the small-M tile GEMM and the skinny GEMM (M <= 384)
must agree to bf16 summation-order noise.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def engs():
    from llmvox_amd.engine import build_engine
    e16 = build_engine(0, "bf16", "bf16", max_streams=2, max_positions=64, max_codec_frames=4096)
    e32 = build_engine(0, "fp32", "fp32", max_streams=2, max_positions=64, max_codec_frames=4096)
    yield e16, e32
    e16.close()
    e32.close()


def _rel_rms(a, b):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / np.sqrt(np.mean(b ** 2)))


@pytest.mark.parametrize("L", [10, 90])
def test_bf16_decode_close_to_golden(engs, L):
    e16, _ = engs
    c = np.load(os.path.join(GOLDEN, "codec_golden.npz"))
    codes = torch.from_numpy(c[f"codes_{L}"]).to(e16.device)
    pcm = e16.decode_codes(codes).cpu().numpy()
    err = _rel_rms(pcm, c[f"pcm_{L}"])
    print(f"bf16 codec L={L} rel RMS vs golden {err:.4f}")
    assert err < 0.02


@pytest.mark.parametrize("S,L", [(8, 256), (16, 128), (3, 700)])
def test_bf16_large_m_close_to_fp32(engs, S, L):
    e16, e32 = engs
    g = torch.Generator().manual_seed(S * 1000 + L)
    codes = torch.randint(0, 4096, (S, L), generator=g).to(e16.device)
    p16 = e16.decode_codes(codes).cpu().numpy()
    p32 = e32.decode_codes(codes).cpu().numpy()
    for b in range(S):
        assert _rel_rms(p16[b], p32[b]) < 0.02, b


def test_large_m_gemm_agrees_with_small_m_gemm(engs):
    e16, _ = engs
    g = torch.Generator().manual_seed(5)
    codes = torch.randint(0, 4096, (8, 256), generator=g).to(e16.device)
    big = e16.decode_codes(codes).cpu().numpy()
    e16.set_option("codec_g2", 0)
    try:
        small = e16.decode_codes(codes).cpu().numpy()
    finally:
        e16.set_option("codec_g2", 1)
    assert _rel_rms(big, small) < 5e-3


@pytest.mark.parametrize("S,L", [(16, 256), (5, 700)])
def test_lds_dma_gemm_agrees_with_register_staged_gemm(engs, S, L):
    """gemm_glds_kernel (LDS-DMA staging, 128 x 192 tiles, 16x16x32 MFMA; M >= ~4,096 frames, and
    the N = 2,304 GEMMs from ~2,048) against gemm_bf16_kernel (register staging, 32x32x16 MFMA):
    the same bf16 products, summed in another order. (5, 700): M = 3,500, a partial last M tile
    and A_CONV windows crossing stream boundaries inside a tile."""
    e16, e32 = engs
    g = torch.Generator().manual_seed(S + L)
    codes = torch.randint(0, 4096, (S, L), generator=g).to(e16.device)
    dma = e16.decode_codes(codes).cpu().numpy()
    e16.set_option("codec_g3", 0)
    try:
        reg = e16.decode_codes(codes).cpu().numpy()
    finally:
        e16.set_option("codec_g3", 1)
    assert _rel_rms(dma, reg) < 5e-3
    p32 = e32.decode_codes(codes[:2]).cpu().numpy()
    for b in range(2):
        assert _rel_rms(dma[b], p32[b]) < 0.02, b


@pytest.mark.parametrize("S,L", [(1, 10), (1, 30), (1, 90), (1, 256), (2, 160), (3, 100)])
def test_skinny_gemm_close_to_fp32(engs, S, L):
    """M = S x L <= 384: the codec's weight GEMMs run on gemm_skinny_kernel (K split over the
    block's waves, A_CONV windows crossing stream boundaries at S > 1)"""
    e16, e32 = engs
    g = torch.Generator().manual_seed(S * 7 + L)
    codes = torch.randint(0, 4096, (S, L), generator=g).to(e16.device)
    p16 = e16.decode_codes(codes).cpu().numpy()
    p32 = e32.decode_codes(codes).cpu().numpy()
    for b in range(S):
        assert _rel_rms(p16[b], p32[b]) < 0.02, b


@pytest.mark.parametrize("S,L", [(1, 10), (1, 90), (2, 160)])
def test_skinny_gemm_agrees_with_tile_kernels(engs, S, L):
    e16, _ = engs
    g = torch.Generator().manual_seed(11 + L)
    codes = torch.randint(0, 4096, (S, L), generator=g).to(e16.device)
    sk = e16.decode_codes(codes).cpu().numpy()
    e16.set_option("codec_skinny", 0)
    try:
        tile = e16.decode_codes(codes).cpu().numpy()
    finally:
        e16.set_option("codec_skinny", 1)
    assert _rel_rms(sk, tile) < 5e-3


def test_bf16_streams_independent_small_m(engs):
    """as below, on the skinny-GEMM path (M = 300: 32-frame tiles straddle the streams)"""
    e16, _ = engs
    g = torch.Generator().manual_seed(19)
    codes = torch.randint(0, 4096, (3, 100), generator=g).to(e16.device)
    a = e16.decode_codes(codes).cpu().numpy()
    perm = [2, 0, 1]
    b = e16.decode_codes(codes[perm]).cpu().numpy()
    for i, p in enumerate(perm):
        np.testing.assert_array_equal(b[i], a[p])


def test_bf16_streams_independent(engs):
    """a stream decoded inside a batch == the same stream decoded in a batch of other content
    (same M, so the same kernels and split-K choices): bit-equal"""
    e16, _ = engs
    g = torch.Generator().manual_seed(9)
    codes = torch.randint(0, 4096, (6, 200), generator=g).to(e16.device)
    a = e16.decode_codes(codes).cpu().numpy()
    perm = [3, 0, 5, 1, 4, 2]
    b = e16.decode_codes(codes[perm]).cpu().numpy()
    for i, p in enumerate(perm):
        np.testing.assert_array_equal(b[i], a[p])


@pytest.fixture(scope="module")
def eng_fp8():
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "bf16", "bf16", max_streams=2, max_positions=64, max_codec_frames=4096, codec_dtype="fp8")
    yield e
    e.close()


@pytest.mark.parametrize("S,L", [(1, 10), (1, 90), (8, 256)])
def test_fp8_codec_weights_close_to_fp32(engs, eng_fp8, S, L):
    """configs[4]: e4m3fn codec weights with per-row scales (W8A16). Weight rounding error is
    ~2^-4 relative per weight; the waveform stays within 8 % relative RMS of the fp32 decode."""
    _, e32 = engs
    g = torch.Generator().manual_seed(S * 77 + L)
    codes = torch.randint(0, 4096, (S, L), generator=g).to(e32.device)
    p8 = eng_fp8.decode_codes(codes).cpu().numpy()
    p32 = e32.decode_codes(codes).cpu().numpy()
    errs = [_rel_rms(p8[b], p32[b]) for b in range(S)]
    print("fp8 codec rel RMS", max(errs))
    assert max(errs) < 0.08



def test_bf16_decode_at_the_bench_shape():
    """configs[2]'s codec call exactly as bench.py makes it: 32 streams x 256 frames = 8,192 frames
    in one batched decode (gemm_glds_kernel at 2 blocks per CU). Every stream within 2 % relative RMS
    of the fp32 parity engine's decode of the same codes (this shape was never compared)."""
    from llmvox_amd.engine import build_engine
    e16 = build_engine(0, "bf16", "bf16", max_streams=2, max_positions=64, max_codec_frames=32 * 256)
    e32 = build_engine(0, "fp32", "fp32", max_streams=2, max_positions=64, max_codec_frames=32 * 256)
    try:
        g = torch.Generator().manual_seed(3256)
        codes = torch.randint(0, 4096, (32, 256), generator=g).to(torch.int32).to(e16.device)
        p16 = e16.decode_codes(codes).cpu().numpy()
        p32 = e32.decode_codes(codes).cpu().numpy()
    finally:
        e16.close()
        e32.close()
    errs = [_rel_rms(p16[b], p32[b]) for b in range(32)]
    print(f"bf16 codec 32 x 256 frames: max rel RMS vs fp32 {max(errs):.4f}, mean {np.mean(errs):.4f}")
    assert max(errs) < 0.02


def _golden_rel(pcm, g, name):
    """relative RMS of pcm against the reference's golden samples (head, tail, every 64th sample)"""
    d = np.concatenate([pcm[:512] - g[f"{name}_head"], pcm[-512:] - g[f"{name}_tail"], pcm[::64] - g[f"{name}_s64"]])
    r = np.concatenate([g[f"{name}_head"], g[f"{name}_tail"], g[f"{name}_s64"]])
    return float(np.sqrt(np.mean(d.astype(np.float64) ** 2)) / np.sqrt(np.mean(r.astype(np.float64) ** 2)))


@pytest.mark.parametrize("L", [270, 480, 810, 1280])
def test_fp8_codec_against_reference_pcm(eng_fp8, L):
    """configs[4]'s codec against the REFERENCE's PCM directly (codec_large_golden.npz, from the imported
    reference, fp32), not only against the HIP fp32 engine. Each dump is decoded in
    a batch of >= 2,048 frames (copies of the same codes: streams are independent), the shape of
    configs[4]'s batched chunk decode, where pwconv1 runs fp8 x fp8 on the block-scaled MFMA
    (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3 activations with per-frame scales); option codec_exp bit 32
    gives the fp8-weight bf16 GEMM (W8A16) for comparison. Bounds: measured 2 x (printed)."""
    g = np.load(os.path.join(GOLDEN, "codec_large_golden.npz"))
    k = -(-2048 // L)
    codes = torch.from_numpy(np.repeat(g[f"codes_{L}"], k, axis=0)).to(eng_fp8.device)
    res = {}
    for name, exp in (("w8a8_mfma", 0), ("w8a16", 32)):
        eng_fp8.set_option("codec_exp", exp)
        try:
            pcm = eng_fp8.decode_codes(codes).cpu().numpy()
        finally:
            eng_fp8.set_option("codec_exp", 0)
        for b in range(1, k):  # identical streams in one batch: identical PCM
            assert np.array_equal(pcm[b], pcm[0])
        res[name] = _golden_rel(pcm[0], g, f"pcm_{L}")
    print(f"fp8 codec vs reference PCM, L = {L} in a batch of {k}: rel RMS {res}")
    assert res["w8a8_mfma"] < 0.12 and res["w8a16"] < 0.08


def test_bf16_codec_at_the_bench_kernels_against_reference_pcm():
    """The bf16 codec on the kernels of the bench's batched decode (gemm_glds at two blocks per CU: >
    256 tiles) against the REFERENCE's PCM directly (codec_large_golden.npz), not only against the HIP
    fp32 engine: six copies of the reference's 1,280-frame dump in one call (7,680 frames,
    720 pwconv1 tiles), every stream within 2 % relative RMS of the reference's samples."""
    from llmvox_amd.engine import build_engine
    g = np.load(os.path.join(GOLDEN, "codec_large_golden.npz"))
    e16 = build_engine(0, "bf16", "bf16", max_streams=2, max_positions=64, max_codec_frames=6 * 1280)
    try:
        codes = torch.from_numpy(np.repeat(g["codes_1280"], 6, axis=0)).to(e16.device)
        pcm = e16.decode_codes(codes).cpu().numpy()
    finally:
        e16.close()
    for b in range(1, 6):
        assert np.array_equal(pcm[b], pcm[0])
    rel = _golden_rel(pcm[0], g, "pcm_1280")
    print(f"bf16 codec (7,680-frame call) vs reference PCM: rel RMS {rel:.4f}")
    assert rel < 0.02
