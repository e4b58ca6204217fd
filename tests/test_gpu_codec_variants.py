"""Codec kernel variants that must leave the PCM bit-identical (round 3, option "codec_exp"): the
one-round GroupNorm kernel against the general one (bit 0), and the dwconv + AdaLN kernel at 4 frames
per block against 16 / 32 / 8 (bits 1-2), in bf16 and in the fp32 parity mode, over the bench's
batched shape and the small first-dump shapes."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = ((32, 256), (1, 256), (2, 160), (1, 10), (3, 7))


@pytest.fixture(scope="module", params=["bf16", "fp32"])
def eng(request):
    from llmvox_amd.engine import build_engine
    e = build_engine(0, request.param, request.param, max_streams=32, max_positions=64, max_codec_frames=8192)
    yield e
    e.close()


@pytest.mark.parametrize("val", [1, 2, 4, 6])
def test_codec_variant_bit_identical(eng, val):
    g = torch.Generator().manual_seed(val)
    try:
        for B, L in SHAPES:
            codes = torch.randint(0, 4096, (B, L), generator=g, dtype=torch.int32).to(eng.device)
            eng.set_option("codec_exp", 0)
            a = eng.decode_codes(codes, 0).clone()
            eng.set_option("codec_exp", val)
            b = eng.decode_codes(codes, 0).clone()
            assert torch.equal(a, b), (B, L, float((a - b).abs().max()))
        eng.check_errors()
    finally:
        eng.set_option("codec_exp", 0)
