"""Weight sources for the hot path: seeded synthetic weights and checkpoint loaders.

Names are the reference state_dict keys so that the same dict can be loaded
into the reference modules (fixture generation), into the CPU oracle and into
the HIP library (by name, through the C-ABI ``lvx_set_weight``).

Synthetic weights follow the reference init scales, perturbed so that every
parameter carries information (a weight of exactly 1 or a bias of exactly 0
cannot catch a kernel that ignores it):

* GPT Linear ~ N(0, 0.02); attn/mlp ``c_proj`` ~ N(0, 0.02/sqrt(2*n_layer));
  ``wpe`` ~ N(0, 0.02)                              (src/model.py:171-176,193-199)
* GPT LayerNorm weight 1 + 0.05 N(0,1)             (src/model.py:33, bias=False)
* codec Conv1d/Linear weight ~ N(0, 0.02), bias 0.01 N(0,1)
                                                   (decoder/models.py:218-221)
* ConvNeXt gamma 1/12 (1 + 0.1 N)                  (decoder/modules.py:37-41)
* AdaLN scale 1 + 0.05 N, shift 0.02 N             (decoder/modules.py:76-79)
* GroupNorm / final LayerNorm weight 1 + 0.05 N, bias 0.02 N
* codebook ``embed`` ~ N(0, 1)                      (encoder/quantization/core_vq.py:137)
* text table [386, 256] ~ N(0, 1), rows 384/385 = mean of rows 0..383
                                                   (inference/model_handler.py:22-42)

The generator is numpy PCG64 seeded per tensor from crc32(name) ^ seed, so the
same weights come out on any host with this image.
"""
from __future__ import annotations

import zlib
from typing import Dict

import numpy as np

from . import config as C

Weights = Dict[str, np.ndarray]


def _rng(name: str, seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64((zlib.crc32(name.encode()) ^ (seed * 2654435761)) & 0xFFFFFFFF))


def _normal(name, shape, std, seed, mean=0.0):
    a = _rng(name, seed).standard_normal(size=shape, dtype=np.float32)
    return (a * np.float32(std) + np.float32(mean)).astype(np.float32)


def gpt_param_shapes(n_layer=C.N_LAYER, d=C.N_EMBD, vocab=C.VOCAB, block=C.BLOCK_SIZE):
    """state_dict keys/shapes of GPT(bias=False) (src/model.py:119-165)."""
    s = {"transformer.wpe.weight": (block, d)}
    for i in range(n_layer):
        p = f"transformer.h.{i}."
        s[p + "ln_1.weight"] = (d,)
        s[p + "attn.c_attn.weight"] = (3 * d, d)
        s[p + "attn.c_proj.weight"] = (d, d)
        s[p + "ln_2.weight"] = (d,)
        s[p + "mlp.c_fc.weight"] = (4 * d, d)
        s[p + "mlp.c_proj.weight"] = (d, 4 * d)
    s["transformer.ln_f.weight"] = (d,)
    s["lm_head.weight"] = (vocab, d)
    return s


def synthetic_gpt(seed: int = 1234) -> Weights:
    w = {}
    cproj_std = 0.02 / np.sqrt(2 * C.N_LAYER)
    for k, shp in gpt_param_shapes().items():
        if k.endswith("ln_1.weight") or k.endswith("ln_2.weight") or k.endswith("ln_f.weight"):
            w[k] = _normal(k, shp, 0.05, seed, mean=1.0)
        elif k.endswith("c_proj.weight"):
            w[k] = _normal(k, shp, cproj_std, seed)
        else:
            w[k] = _normal(k, shp, 0.02, seed)
    return w


CODEBOOK_KEY = "feature_extractor.encodec.quantizer.vq.layers.0._codebook.embed"
POS_NET_RESNET = (0, 1, 3, 4)
POS_NET_ATTN = 2
POS_NET_NORM = 5


def codec_param_shapes():
    """state_dict keys/shapes of the decode path of WavTokenizer
    (decoder/models.py:166-216, modules.py:24-41,72-79, heads.py:36-40)."""
    D, I, Cin = C.CODEC_DIM, C.CODEC_FF, C.CODEC_IN
    s = {
        "backbone.embed.weight": (D, Cin, 7),
        "backbone.embed.bias": (D,),
        "backbone.norm.scale.weight": (C.ADANORM_N, D),
        "backbone.norm.shift.weight": (C.ADANORM_N, D),
    }
    for i in POS_NET_RESNET:
        p = f"backbone.pos_net.{i}."
        for n in ("norm1", "norm2"):
            s[p + n + ".weight"] = (D,)
            s[p + n + ".bias"] = (D,)
        for n in ("conv1", "conv2"):
            s[p + n + ".weight"] = (D, D, 3)
            s[p + n + ".bias"] = (D,)
    p = f"backbone.pos_net.{POS_NET_ATTN}."
    s[p + "norm.weight"] = (D,)
    s[p + "norm.bias"] = (D,)
    for n in ("q", "k", "v", "proj_out"):
        s[p + n + ".weight"] = (D, D, 1)
        s[p + n + ".bias"] = (D,)
    s[f"backbone.pos_net.{POS_NET_NORM}.weight"] = (D,)
    s[f"backbone.pos_net.{POS_NET_NORM}.bias"] = (D,)
    for i in range(C.CODEC_LAYERS):
        p = f"backbone.convnext.{i}."
        s[p + "dwconv.weight"] = (D, 1, 7)
        s[p + "dwconv.bias"] = (D,)
        s[p + "norm.scale.weight"] = (C.ADANORM_N, D)
        s[p + "norm.shift.weight"] = (C.ADANORM_N, D)
        s[p + "pwconv1.weight"] = (I, D)
        s[p + "pwconv1.bias"] = (I,)
        s[p + "pwconv2.weight"] = (D, I)
        s[p + "pwconv2.bias"] = (D,)
        s[p + "gamma"] = (D,)
    s["backbone.final_layer_norm.weight"] = (D,)
    s["backbone.final_layer_norm.bias"] = (D,)
    s["head.out.weight"] = (C.N_FFT + 2, D)
    s["head.out.bias"] = (C.N_FFT + 2,)
    s[CODEBOOK_KEY] = (C.CODEBOOK_SIZE, C.CODEC_IN)
    return s


def synthetic_codec(seed: int = 1234) -> Weights:
    w = {}
    for k, shp in codec_param_shapes().items():
        if k == CODEBOOK_KEY:
            w[k] = _normal(k, shp, 1.0, seed)
        elif k.endswith("gamma"):
            w[k] = _normal(k, shp, 0.1 / C.CODEC_LAYERS, seed, mean=1.0 / C.CODEC_LAYERS)
        elif k.endswith("scale.weight"):
            w[k] = _normal(k, shp, 0.05, seed, mean=1.0)
        elif k.endswith("shift.weight"):
            w[k] = _normal(k, shp, 0.02, seed)
        elif len(shp) == 1 and (".norm" in k or "final_layer_norm" in k or f"pos_net.{POS_NET_NORM}." in k):
            if k.endswith(".weight"):
                w[k] = _normal(k, shp, 0.05, seed, mean=1.0)
            else:
                w[k] = _normal(k, shp, 0.02, seed)
        elif k.endswith(".bias"):
            w[k] = _normal(k, shp, 0.01, seed)
        else:
            w[k] = _normal(k, shp, 0.02, seed)
    return w


TEXT_EMBED_KEY = "encoder.embed_tokens.weight"


def synthetic_text_embed(seed: int = 1234) -> np.ndarray:
    """[386, 256]: 384 ByT5 rows + the two rows that smart_tokenizer_and_embedding_resize
    mean-initialises (inference/model_handler.py:31-42)."""
    t = _normal(TEXT_EMBED_KEY, (C.TEXT_VOCAB, C.TEXT_DIM), 1.0, seed)
    base = t[:384].mean(axis=0, keepdims=True)
    t[384] = base  # "[PAD]" added first: mean of the 384 rows before it
    t[385] = t[:385].mean(axis=0)  # "EOS" added second: mean of the 385 rows before it
    return t


def synthetic_all(seed: int = 1234):
    return synthetic_gpt(seed), synthetic_codec(seed), synthetic_text_embed(seed)


# ---------------------------------------------------------------------------
# WavTokenizer encoder (encode_infer, decoder/pretrained.py:185-190): the SEANet encoder
# EncodecFeatures builds (decoder/feature_extractors.py:66-69: n_filters 32, ratios [8, 5, 4, 2]
# reversed, one residual block per ratio, compress 2, ELU, weight_norm, reflect padding, 2-layer LSTM
# with skip, dimension 512; encoder/modules/seanet.py:94-140) and the 1-codebook quantizer.
# ---------------------------------------------------------------------------

ENC_PREFIX = "feature_extractor.encodec.encoder.model."
ENC_RATIOS = (2, 4, 5, 8)
ENC_LSTM = 13  # model index of the SLSTM


def encoder_convs():
    """[(name, cin, cout, kernel, stride, dilation, elu_before)] in execution order: name is the
    state_dict prefix of the SConv1d ('<prefix>.conv.conv.{weight_g,weight_v,bias}'). Residual blocks
    are the triples (block.1, block.3, shortcut) at model indices 1, 4, 7, 10
    (seanet.py:117-135, residual block seanet.py:36-64)."""
    out = [("0", 1, 32, 7, 1, 1, False)]
    mult, idx = 1, 1
    for ratio in ENC_RATIOS:
        dim = 32 * mult
        out += [(f"{idx}.block.1", dim, dim // 2, 3, 1, 1, True),
                (f"{idx}.block.3", dim // 2, dim, 1, 1, 1, True),
                (f"{idx}.shortcut", dim, dim, 1, 1, 1, False)]
        out.append((f"{idx + 2}", dim, 2 * dim, 2 * ratio, ratio, 1, True))
        mult *= 2
        idx += 3
    out.append(("15", 512, 512, 7, 1, 1, True))
    return out


def encoder_param_shapes():
    s = {}
    for name, cin, cout, k, _, _, _ in encoder_convs():
        p = ENC_PREFIX + name + ".conv.conv."
        s[p + "weight_v"] = (cout, cin, k)
        s[p + "weight_g"] = (cout, 1, 1)
        s[p + "bias"] = (cout,)
    p = ENC_PREFIX + f"{ENC_LSTM}.lstm."
    for layer in range(2):
        s[p + f"weight_ih_l{layer}"] = (4 * 512, 512)
        s[p + f"weight_hh_l{layer}"] = (4 * 512, 512)
        s[p + f"bias_ih_l{layer}"] = (4 * 512,)
        s[p + f"bias_hh_l{layer}"] = (4 * 512,)
    return s


def synthetic_encoder(seed: int = 1234) -> Weights:
    """weight_v ~ N(0, 1 / (cin k)) (unit gain), weight_g = |v| (1 + 0.1 N) per output channel (x 3
    for the last conv, so the embedding lives on the codebook's N(0, 1) scale and the quantiser's
    choice depends on x . e, not only on |e|), bias 0.01 N; LSTM weights and biases
    ~ N(0, 1/sqrt(3 x 512)) (the spread of PyTorch's U(-1/sqrt(512), 1/sqrt(512)) init). The codebook
    is the decoder's (CODEBOOK_KEY)."""
    w = {}
    for k, shp in encoder_param_shapes().items():
        if k.endswith("weight_v"):
            w[k] = _normal(k, shp, 1.0 / np.sqrt(shp[1] * shp[2]), seed)
        elif k.endswith("weight_g"):
            v = w[k[:-1] + "v"]
            nrm = np.sqrt((v.astype(np.float64) ** 2).sum(axis=(1, 2))).astype(np.float32).reshape(shp)
            gain = 3.0 if k.startswith(ENC_PREFIX + "15.") else 1.0
            w[k] = (gain * nrm * _normal(k, shp, 0.1, seed, mean=1.0)).astype(np.float32)
        elif ".lstm." in k:
            w[k] = _normal(k, shp, 1.0 / np.sqrt(3 * 512), seed)
        else:
            w[k] = _normal(k, shp, 0.01, seed)
    return w


def encoder_effective(we: Weights) -> Weights:
    """weight_norm resolved as the reference's forward pre-hook does (torch.nn.utils.weight_norm:
    w = torch._weight_norm(v, g, 0), on the CPU in fp32: the same bits as the reference), keyed
    '<prefix>.conv.conv.weight'; LSTM and bias entries unchanged."""
    import torch
    out = {}
    for k, v in we.items():
        if k.endswith("weight_g"):
            continue
        if k.endswith("weight_v"):
            g = torch.from_numpy(np.ascontiguousarray(we[k[:-1] + "g"]))
            out[k[:-2]] = torch._weight_norm(torch.from_numpy(np.ascontiguousarray(v)), g, 0).numpy()
        else:
            out[k] = v
    return out


# ---------------------------------------------------------------------------
# Checkpoint loaders.  Only loaders that execute nothing from the
# file: torch.load(weights_only=True).
# ---------------------------------------------------------------------------

class GPTWeights(dict):
    """GPT state dict (reference keys, fp32 numpy) + the checkpoint's ``block_size`` (the reference's
    GPT.forward asserts t <= block_size, src/model.py:205)."""
    block_size: int = C.BLOCK_SIZE


def load_llmvox_checkpoint(path: str) -> GPTWeights:
    """A checkpoint in the reference's save layout (src/utils.py:147-153: 'model', 'optimizer',
    'model_args', 'iter_num', 'config'), read as inference/model_handler.py:148-165 reads it:
    ``model_args`` fixes the architecture, ``_orig_mod.`` prefixes (torch.compile) are stripped,
    missing keys would keep their init under strict=False (here the hot-path keys are required).

    block_size: the library's position table holds 8192 rows (GPTConfig.block_size of the shipped
    model); a smaller block_size pads wpe with zero rows it can never reach (the returned
    ``block_size`` bounds positions, as the reference's assert does), a larger one is rejected."""
    import torch
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if "model" not in ck or "model_args" not in ck:
        raise KeyError("not an LLMVoX checkpoint: needs 'model' and 'model_args' (src/utils.py:147-153)")
    args = ck["model_args"]
    for k, v in (("n_layer", C.N_LAYER), ("n_head", C.N_HEAD), ("n_embd", C.N_EMBD), ("vocab_size", C.VOCAB)):
        if k in args and int(args[k]) != v:
            raise ValueError(f"checkpoint {k}={args[k]} but this build is specialised for {v}")
    if args.get("bias", False):
        raise ValueError("checkpoint has bias=True; the reference inference model uses bias=False")
    block = int(args.get("block_size", C.BLOCK_SIZE))
    if not 1 <= block <= C.BLOCK_SIZE:
        raise ValueError(f"checkpoint block_size={block}: this build holds at most {C.BLOCK_SIZE} positions")
    out = GPTWeights()
    out.block_size = block
    for k, v in ck["model"].items():
        if k.startswith("_orig_mod."):
            k = k[len("_orig_mod."):]
        out[k] = v.float().cpu().numpy()
    # strict=False in the reference: missing keys keep their init; we require the hot-path ones.
    missing = [k for k in gpt_param_shapes(block=block) if k not in out]
    if missing:
        raise KeyError(f"checkpoint lacks hot-path weights: {missing[:4]}...")
    wpe = out["transformer.wpe.weight"]
    if wpe.shape != (block, C.N_EMBD):
        raise ValueError(f"transformer.wpe.weight is {wpe.shape}, model_args block_size {block}")
    if block < C.BLOCK_SIZE:
        out["transformer.wpe.weight"] = np.concatenate(
            [wpe, np.zeros((C.BLOCK_SIZE - block, C.N_EMBD), np.float32)], 0)
    return out


def load_wavtokenizer_checkpoint(path: str) -> Weights:
    """Lightning ckpt: ckpt['state_dict'] filtered to backbone./head./feature_extractor.
    (WavTokenizer/decoder/pretrained.py:101-105). The encoder's entries (ENC_PREFIX, used by
    encode_infer) come along when the checkpoint holds them."""
    import torch
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck["state_dict"]
    out = {}
    for k, v in sd.items():
        if k.startswith(("backbone.", "head.", "feature_extractor.")):
            out[k] = v.float().cpu().numpy()
    need = [k for k in codec_param_shapes() if k not in out]
    if need:
        raise KeyError(f"codec checkpoint lacks decode-path weights: {need[:4]}...")
    return out


def load_text_embed_from_t5(state_dict: Dict[str, "np.ndarray"]) -> np.ndarray:
    """T5 ``encoder.embed_tokens.weight`` (or ``shared.weight``) resized to 386 rows with
    mean-initialised special rows (inference/model_handler.py:22-42,88-105)."""
    key = TEXT_EMBED_KEY if TEXT_EMBED_KEY in state_dict else "shared.weight"
    t = np.asarray(state_dict[key], dtype=np.float32)
    rows = [t[:384]] if t.shape[0] >= 384 else [t]
    base = np.concatenate(rows, 0)[:384]
    r384 = base.mean(0, keepdims=True)
    r385 = np.concatenate([base, r384], 0).mean(0, keepdims=True)
    return np.concatenate([base, r384, r385], 0).astype(np.float32)
