"""The CPU oracle against the golden vectors produced by the reference itself
(tests/golden/make_golden.py). This pins the oracle before it is trusted as the checker."""
import os

import numpy as np
import pytest
import torch

from llmvox_amd import weights as LW
from oracle import reference_cpu as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def W():
    gw, cw, tt = LW.synthetic_all(1234)
    return R.to_torch(gw), R.to_torch(cw), torch.from_numpy(tt)


def test_ar_ids_and_logits_bitexact(W):
    g = np.load(os.path.join(GOLDEN, "ar_golden.npz"))
    Wg, Wc, tt = W
    n = 96  # keep the CPU suite fast; the full 256 are checked on the GPU
    ids, margins, logits = R.ar_decode(Wg, tt, Wc[R.CODEBOOK_KEY], g["text_ids"].tolist(), n, record_logits=True)
    assert ids == g["ids"][:n].tolist()
    np.testing.assert_allclose(margins, g["margins"][:n], rtol=0, atol=0)
    for k, step in enumerate(g["logit_steps"]):
        if step < n:
            np.testing.assert_array_equal(logits[step].numpy(), g["logits"][k])


def test_teacher_forced_equals_kv_decode(W):
    """Second, independent oracle: the training-form causal full-sequence pass."""
    g = np.load(os.path.join(GOLDEN, "ar_golden.npz"))
    Wg, Wc, tt = W
    n = 80
    lg = R.teacher_forced_logits(Wg, tt, Wc[R.CODEBOOK_KEY], g["text_ids"].tolist(), g["ids"][:n].tolist())
    assert lg.argmax(-1).tolist() == g["ids"][:n].tolist()
    for k, step in enumerate(g["logit_steps"]):
        if step < n:
            assert np.abs(lg[step].numpy() - g["logits"][k]).max() < 1e-5


@pytest.mark.parametrize("L", [1, 2, 10, 30])
def test_codec_pcm_bitexact(W, L):
    c = np.load(os.path.join(GOLDEN, "codec_golden.npz"))
    _, Wc, _ = W
    pcm = R.decode_codes(Wc, torch.from_numpy(c[f"codes_{L}"]).long()).numpy()
    np.testing.assert_array_equal(pcm, c[f"pcm_{L}"])


def test_codec_intermediates(W):
    c = np.load(os.path.join(GOLDEN, "codec_golden.npz"))
    _, Wc, _ = W
    feats = R.codes_to_features(Wc, torch.from_numpy(c["codes_10"]).long())
    np.testing.assert_array_equal(feats.numpy(), c["features_10"])
    np.testing.assert_array_equal(R.backbone(Wc, feats).numpy(), c["backbone_10"])


def test_codes_to_features_rejects_batched_2d(W):
    """The reference reads a 2-D input as (K, L): [B>1, L] indexes past the single codebook."""
    _, Wc, _ = W
    with pytest.raises(IndexError):
        R.codes_to_features(Wc, torch.zeros(2, 5, dtype=torch.long))


def test_istft_envelope_and_length(W):
    spec = torch.randn(1, 641, 7, dtype=torch.complex64)
    y = R.istft_same(spec)
    assert y.shape == (1, 7 * 320)


@pytest.mark.parametrize("L", [270, 1280])
def test_codec_large_dumps_bitexact(W, L):
    """configs[3]'s dump sizes (streaming_server.py:373-375): the oracle against the reference's PCM
    summaries (tests/golden/codec_large_golden.npz)."""
    g = np.load(os.path.join(GOLDEN, "codec_large_golden.npz"))
    _, Wc, _ = W
    pcm = R.decode_codes(Wc, torch.from_numpy(g[f"codes_{L}"]).long()).numpy()[0]
    assert pcm.size == int(g[f"pcm_{L}_len"])
    np.testing.assert_array_equal(pcm[:512], g[f"pcm_{L}_head"])
    np.testing.assert_array_equal(pcm[-512:], g[f"pcm_{L}_tail"])
    np.testing.assert_array_equal(pcm[::64], g[f"pcm_{L}_s64"])


def test_long_stream_ids_through_smallest_margin(W):
    """The reference's long stream (2,490 calls): the oracle reproduces its ids bit for bit through
    step 520, past the stream's smallest top1-top2 margin (2.1e-6 at step 498)."""
    g = np.load(os.path.join(GOLDEN, "stream_long_golden.npz"))
    Wg, Wc, tt = W
    n = 520
    ids, margins, _ = R.ar_decode(Wg, tt, Wc[R.CODEBOOK_KEY], g["text_ids"].tolist(), n)
    assert ids == g["ids"][:n].tolist()
    np.testing.assert_array_equal(np.float32(margins), g["margins"][:n])


def test_encoder_oracle_matches_reference_encode_infer():
    """8f.4: the oracle's SEANet encoder + quantiser against the reference's own encode_infer
    (tests/golden/make_golden_encoder.py): codes and the pre-quantisation embedding bit for bit."""
    g = np.load(os.path.join(GOLDEN, "encoder_golden.npz"))
    We = R.to_torch(LW.encoder_effective(LW.synthetic_encoder(1234)))
    cb = torch.from_numpy(LW.synthetic_codec(1234)[LW.CODEBOOK_KEY])
    tags = sorted(k[len("codes_"):] for k in g.files if k.startswith("codes_"))
    assert len(tags) == 5
    for tag in tags:
        audio = torch.from_numpy(g[f"audio_{tag}"])
        feats, codes = R.encode_infer(We, cb, audio)
        np.testing.assert_array_equal(codes.numpy(), g[f"codes_{tag}"])
        assert feats.shape == (audio.shape[0], 512, g[f"codes_{tag}"].shape[-1])
        emb = R.seanet_encode(We, audio).numpy()
        if f"emb_{tag}" in g.files:
            np.testing.assert_array_equal(emb, g[f"emb_{tag}"])
        else:
            np.testing.assert_array_equal(emb.reshape(-1)[::7], g[f"emb_{tag}_every7"])


def test_encoder_frame_count_matches_reference():
    """lvx_enc_frames (host-side SConv1d length chain, no GPU) = the reference's T = ceil(N / 320)"""
    from llmvox_amd import _lib
    lib = _lib.load()
    g = np.load(os.path.join(GOLDEN, "encoder_golden.npz"))
    for k in g.files:
        if k.startswith("codes_"):
            N = g["audio_" + k[len("codes_"):]].shape[1]
            assert lib.lvx_enc_frames(N) == g[k].shape[-1] == -(-N // 320)
    for N in (1, 2, 319, 320, 321, 641, 24000, 24001):
        assert lib.lvx_enc_frames(N) == -(-N // 320)
