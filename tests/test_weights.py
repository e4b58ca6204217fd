import numpy as np
import torch

from llmvox_amd import weights as LW


def test_synthetic_deterministic_and_shapes():
    a = LW.synthetic_gpt(1234)
    b = LW.synthetic_gpt(1234)
    for k, shp in LW.gpt_param_shapes().items():
        assert a[k].shape == shp and a[k].dtype == np.float32
        np.testing.assert_array_equal(a[k], b[k])
    c = LW.synthetic_codec(1234)
    assert set(c) == set(LW.codec_param_shapes())
    assert abs(float(c["backbone.convnext.0.gamma"].mean()) - 1 / 12) < 0.01
    t = LW.synthetic_text_embed(1234)
    assert t.shape == (386, 256)
    np.testing.assert_allclose(t[384], t[:384].mean(0), rtol=1e-6)
    np.testing.assert_allclose(t[385], t[:385].mean(0), rtol=1e-6)


def test_llmvox_checkpoint_loader_strips_orig_mod(tmp_path):
    gw = LW.synthetic_gpt(7)
    sd = {("_orig_mod." + k if i % 2 else k): torch.from_numpy(v) for i, (k, v) in enumerate(gw.items())}
    p = tmp_path / "ckpt.pt"
    torch.save({"model": sd, "model_args": {"n_layer": 4, "n_head": 8, "n_embd": 768, "block_size": 8192,
                                            "bias": False, "vocab_size": 4096}}, p)
    out = LW.load_llmvox_checkpoint(str(p))
    for k, v in gw.items():
        np.testing.assert_array_equal(out[k], v)


def test_wavtokenizer_checkpoint_loader_filters_prefixes(tmp_path):
    cw = LW.synthetic_codec(7)
    sd = {k: torch.from_numpy(v) for k, v in cw.items()}
    sd["discriminator.x"] = torch.zeros(3)
    p = tmp_path / "wt.ckpt"
    torch.save({"state_dict": sd}, p)
    out = LW.load_wavtokenizer_checkpoint(str(p))
    assert "discriminator.x" not in out and set(cw) <= set(out)


def test_text_embed_resize():
    base = np.random.default_rng(0).standard_normal((384, 256)).astype(np.float32)
    t = LW.load_text_embed_from_t5({"shared.weight": base})
    assert t.shape == (386, 256)
    np.testing.assert_allclose(t[384], base.mean(0), rtol=1e-5)


def test_reference_save_layout_loads_with_weights_only(tmp_path):
    """All three checkpoints in the reference's save layouts (tests/ckpt_files.py) load through the
    weights_only loaders, optimizer / config entries included, to the synthetic weights."""
    from tests.ckpt_files import write_all
    from llmvox_amd.handler import _load_t5_state
    paths = write_all(str(tmp_path), block_size=8192)
    gw, cw, tt = LW.synthetic_all(1234)
    g = LW.load_llmvox_checkpoint(paths["llmvox_checkpoint_path"])
    assert g.block_size == 8192 and set(g) == set(gw)
    for k in gw:
        np.testing.assert_array_equal(g[k], gw[k])
    c = LW.load_wavtokenizer_checkpoint(paths["wav_model_path"])
    assert set(c) == set(cw)  # the training-only modules are filtered out
    t = LW.load_text_embed_from_t5(_load_t5_state(paths["encoder_model_path"]))
    np.testing.assert_allclose(t, tt, rtol=0, atol=1e-6)


def test_block_size_is_validated(tmp_path):
    from tests.ckpt_files import write_llmvox_ckpt
    gw = LW.synthetic_gpt(3)
    p = tmp_path / "small.pt"
    write_llmvox_ckpt(p, gw, block_size=1024)
    g = LW.load_llmvox_checkpoint(str(p))
    assert g.block_size == 1024 and g["transformer.wpe.weight"].shape == (8192, 768)
    np.testing.assert_array_equal(g["transformer.wpe.weight"][:1024], gw["transformer.wpe.weight"][:1024])
    assert not g["transformer.wpe.weight"][1024:].any()
    big = dict(gw)
    big["transformer.wpe.weight"] = np.zeros((9000, 768), np.float32)
    torch.save({"model": {k: torch.from_numpy(v) for k, v in big.items()},
                "model_args": {"n_layer": 4, "n_head": 8, "n_embd": 768, "block_size": 9000, "bias": False,
                               "vocab_size": 4096}}, tmp_path / "big.pt")
    import pytest
    with pytest.raises(ValueError, match="block_size"):
        LW.load_llmvox_checkpoint(str(tmp_path / "big.pt"))
    torch.save({"model": {k: torch.from_numpy(v) for k, v in gw.items()},
                "model_args": {"n_layer": 4, "n_head": 8, "n_embd": 768, "block_size": 4096, "bias": False,
                               "vocab_size": 4096}}, tmp_path / "mismatch.pt")
    with pytest.raises(ValueError, match="wpe"):
        LW.load_llmvox_checkpoint(str(tmp_path / "mismatch.pt"))
