"""GPU parity of the HIP hot path against the reference's golden vectors and the CPU oracle.

Bars (BASELINE.json north_star): speech-token ids bit-exact (fp32 parity mode), waveform
within 1e-4 (we hold max |diff| <= 2e-4 and RMS diff <= 1e-5 on PCM of RMS ~0.02).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def eng():
    from llmvox_amd.engine import build_engine
    e = build_engine(0, "fp32", "fp32", max_streams=8, max_positions=8192, max_codec_frames=1280)
    yield e
    e.close()


@pytest.fixture(scope="module")
def ar_golden():
    return np.load(os.path.join(GOLDEN, "ar_golden.npz"))


def _run_fused(eng, text_ids, n_steps, slot=0, B=1, stride=None):
    stride = stride or n_steps
    dev = eng.device
    plan = torch.full((B, stride), 384, dtype=torch.int32)
    for b in range(B):
        n = min(len(text_ids), stride)
        plan[b, :n] = torch.tensor(text_ids[:n], dtype=torch.int32)
    plan = plan.to(dev)
    slots = torch.arange(slot, slot + B, dtype=torch.int32, device=dev)
    rowstep = torch.zeros(B, dtype=torch.int32, device=dev)
    tok = torch.full((B, stride), -1, dtype=torch.int32, device=dev)
    marg = torch.zeros((B, stride), dtype=torch.float32, device=dev)
    for s in range(slot, slot + B):
        eng.reset_slot(s)
    eng.ar_steps(n_steps, slots, plan, rowstep, tok, marg)
    eng.check_errors()
    torch.cuda.synchronize()
    return tok.cpu().numpy(), marg.cpu().numpy()


def test_fused_step_ids_bitexact(eng, ar_golden):
    ids = ar_golden["ids"]
    tok, marg = _run_fused(eng, ar_golden["text_ids"].tolist(), len(ids))
    assert (tok[0] == ids).all(), f"first mismatch at {np.nonzero(tok[0] != ids)[0][:5]}"
    np.testing.assert_allclose(marg[0], ar_golden["margins"], atol=5e-5)


def test_fused_step_batched_streams(eng, ar_golden):
    """B=4 rows in 4 slots, same text: every row must reproduce the golden ids."""
    ids = ar_golden["ids"][:96]
    tok, _ = _run_fused(eng, ar_golden["text_ids"].tolist(), 96, slot=2, B=4)
    for b in range(4):
        assert (tok[b] == ids).all(), b


def test_dropin_model_matches_golden_logits(eng, ar_golden):
    """The .model drop-in (row forward) driven like streaming_server.py:323-346."""
    from llmvox_amd.handler import SpeechGPT, _SlotPool
    import torch.nn.functional as F
    from llmvox_amd import weights as LW
    _, cw, tt = LW.synthetic_all(1234)
    table = torch.from_numpy(tt).to(eng.device)
    cb = torch.from_numpy(cw[LW.CODEBOOK_KEY]).to(eng.device)
    model = SpeechGPT(eng, _SlotPool(eng.max_streams))
    text_ids = ar_golden["text_ids"].tolist()
    steps = ar_golden["logit_steps"].tolist()
    n = max(steps) + 1
    kv, prev, hist = None, None, None
    got = {}
    ids = []
    for i in range(n):
        tid = text_ids[i] if i < len(text_ids) else 384
        te = table[tid].view(1, 1, -1)
        se = torch.zeros(1, 1, 512, device=eng.device) if i == 0 else cb[prev].view(1, 1, -1)
        x = F.normalize(torch.cat([te, se], dim=2), p=2, dim=2, eps=1e-8)
        hist = x if hist is None else torch.cat([hist, x], dim=1)
        logits, _, kv = model(hist, kvcache=kv)
        prev = int(F.softmax(logits[:, -1, :], dim=-1).argmax(-1).item())
        ids.append(prev)
        if i in steps:
            got[i] = logits[0, -1].cpu().numpy()
    assert ids == ar_golden["ids"][:n].tolist()
    for k, i in enumerate(steps):
        np.testing.assert_allclose(got[i], ar_golden["logits"][k], atol=2e-5, rtol=0)


@pytest.mark.parametrize("L", [1, 2, 10, 30, 90])
def test_codec_decode_matches_golden(eng, L):
    c = np.load(os.path.join(GOLDEN, "codec_golden.npz"))
    codes = torch.from_numpy(c[f"codes_{L}"]).to(eng.device)
    pcm = eng.decode_codes(codes).cpu().numpy()
    ref = c[f"pcm_{L}"]
    assert pcm.shape == ref.shape
    d = pcm - ref
    assert np.abs(d).max() < 2e-4, np.abs(d).max()
    assert np.sqrt(np.mean(d.astype(np.float64) ** 2)) < 1e-5


def test_codec_decode_features_path(eng):
    """decode(features) through the reference layout [B,512,L] (pretrained.py:192-207)."""
    c = np.load(os.path.join(GOLDEN, "codec_golden.npz"))
    feats = torch.from_numpy(c["features_10"]).to(eng.device)
    pcm = eng.decode_features(feats, 0).cpu().numpy()
    assert np.abs(pcm - c["pcm_10"]).max() < 2e-4


def test_codec_long_chunk_rms(eng):
    c = np.load(os.path.join(GOLDEN, "codec_golden.npz"))
    codes = torch.from_numpy(c["codes_160"]).to(eng.device)
    pcm = eng.decode_codes(codes).cpu().numpy()[0]
    assert abs(np.sqrt(np.mean(pcm.astype(np.float64) ** 2)) - float(c["pcm_160_rms"])) < 1e-5
    assert np.abs(pcm[:512] - c["pcm_160_head"]).max() < 2e-4
    assert np.abs(pcm[-512:] - c["pcm_160_tail"]).max() < 2e-4


def test_codec_batched_equals_single(eng):
    """B streams in one call == B separate calls (streams are independent)."""
    g = torch.Generator().manual_seed(3)
    codes = torch.randint(0, 4096, (3, 40), generator=g).to(eng.device)
    batched = eng.decode_codes(codes).cpu()
    for b in range(3):
        single = eng.decode_codes(codes[b:b + 1]).cpu()
        assert torch.allclose(batched[b:b + 1], single, atol=1e-6, rtol=0)


@pytest.mark.parametrize("what", ["text_embed", "codes_to_features", "decode_codes"])
def test_out_of_range_ids_raise_index_error(eng, what):
    """The reference raises IndexError for an embedding / codebook id out of range (nn.Embedding,
    decoder/pretrained.py:209-239); the device path clamps the load, flags it, and the next
    check_errors raises LvxIndexError (an IndexError). The flag is cleared by the report."""
    from llmvox_amd._lib import LvxIndexError
    for bad in (-1, {"text_embed": 386}.get(what, 4096)):
        if what == "text_embed":
            eng.text_embed(torch.tensor([5, bad, 7], dtype=torch.int64, device=eng.device))
        elif what == "codes_to_features":
            eng.codes_to_features(torch.tensor([[1, 2, bad]], dtype=torch.int64, device=eng.device))
        else:
            eng.decode_codes(torch.tensor([[1, bad, 3]], dtype=torch.int32, device=eng.device))
        with pytest.raises(IndexError) as ei:
            eng.check_errors()
        assert isinstance(ei.value, LvxIndexError)
        eng.check_errors()  # cleared
    eng.decode_codes(torch.tensor([[0, 4095, 3]], dtype=torch.int32, device=eng.device))
    eng.check_errors()  # the envelope self-check holds and in-range codes raise nothing


def test_error_words_are_split_and_every_bit_is_reported(eng):
    """the codec keeps its own error word (it may run on a second stream beside the
    decode), a take of one word leaves the other alone, and check_errors names every set condition."""
    from llmvox_amd import _lib
    dev = eng.device
    eng.text_embed(torch.tensor([5, 400], dtype=torch.int64, device=dev))        # AR word, bit 4
    side = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(side):                                                # codec word, bit 4
        eng.decode_codes(torch.tensor([[1, 5000, 3]], dtype=torch.int32, device=dev))
    side.synchronize()
    bits = torch.zeros(1, dtype=torch.int32, device=dev)
    eng.take_errors(_lib.ERRW_CODEC, bits)                                       # the codec word only
    assert int(bits.item()) == 4 << 16
    with pytest.raises(_lib.LvxIndexError) as ei:                               # the AR bit is still set
        eng.check_errors()
    assert ei.value.bits == 0 or "text id" in str(ei.value)
    eng.check_errors()
    # both words at once: one exception naming both
    eng.text_embed(torch.tensor([-3], dtype=torch.int64, device=dev))
    eng.decode_codes(torch.tensor([[4096]], dtype=torch.int32, device=dev))
    with pytest.raises(_lib.LvxIndexError) as ei:
        eng.check_errors()
    assert "text id" in str(ei.value) and "codec: a code outside" in str(ei.value)
    eng.check_errors()
