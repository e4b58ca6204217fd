"""CPU (PyTorch eager, fp32) restatement of the LLMVoX streaming-TTS hot path.

TEST INFRASTRUCTURE / CPU BASELINE ONLY — never imported by ``llmvox_amd``.

It restates, op for op, what the reference computes (file:line cite the
reference checkout), including its O(t) history / KV concatenation, so that

* ``tests/`` can check it against the golden fixtures the reference itself
  produced (``tests/golden/make_golden.py``), and then use it as the checker of
  the HIP path at sizes it finishes in seconds;
* ``bench.py`` can time it as the "reference CPU eager path" (cpu_baseline,
  kind "port").

Weights are the dicts of ``llmvox_amd.weights`` (reference state_dict keys).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

N_LAYER, N_HEAD, N_EMBD, BLOCK_SIZE = 4, 8, 768, 8192


def _t(w):
    return w if isinstance(w, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(w))


def to_torch(weights: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    return {k: _t(v).float() for k, v in weights.items()}


# ---------------------------------------------------------------------------
# a5-a10: GPT.forward with the reference's list-of-[K,V] cache (src/model.py:201-237)
# ---------------------------------------------------------------------------

def new_gelu(x):  # src/model.py:21-26 (tanh form)
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def gpt_forward(W, emb, kvcache=None, train_causal=False):
    """(emb [B,t,768], kvcache list|None) -> (logits [B,1,4096] or [B,t,4096], new kvcache).

    ``train_causal`` runs the teacher-forced full-sequence form (is_causal=True and
    lm_head on every position, src/model.py:92-93,225-230) — the second, independent
    oracle of the KV-cache decode."""
    b, t, _ = emb.shape
    assert t <= BLOCK_SIZE, f"Cannot forward sequence of length {t}, block size is only {BLOCK_SIZE}"
    x = emb + W["transformer.wpe.weight"][:t].unsqueeze(0)  # :206-212
    if not kvcache:
        kvcache = [None] * N_LAYER
    else:
        x = x[:, [-1], :]  # :216-217
    new_cache = []
    for i in range(N_LAYER):  # Block.forward :128-132
        p = f"transformer.h.{i}."
        h = F.layer_norm(x, (N_EMBD,), W[p + "ln_1.weight"], None, 1e-5)
        q, k, v = F.linear(h, W[p + "attn.c_attn.weight"]).split(N_EMBD, dim=2)  # :72
        if kvcache[i]:
            pk, pv = kvcache[i]
            k = torch.cat([pk, k], dim=1)  # :74-77
            v = torch.cat([pv, v], dim=1)
        new_cache.append([k, v])
        B, T, Cc = h.shape
        Tk = k.shape[1]
        kh = k.view(B, Tk, N_HEAD, Cc // N_HEAD).transpose(1, 2)
        qh = q.view(B, T, N_HEAD, Cc // N_HEAD).transpose(1, 2)
        vh = v.view(B, Tk, N_HEAD, Cc // N_HEAD).transpose(1, 2)
        y = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=None, dropout_p=0.0, is_causal=train_causal)
        y = y.transpose(1, 2).contiguous().view(B, T, Cc)
        x = x + F.linear(y, W[p + "attn.c_proj.weight"])  # :97
        h2 = F.layer_norm(x, (N_EMBD,), W[p + "ln_2.weight"], None, 1e-5)
        m = F.linear(new_gelu(F.linear(h2, W[p + "mlp.c_fc.weight"])), W[p + "mlp.c_proj.weight"])
        x = x + m
    x = F.layer_norm(x, (N_EMBD,), W["transformer.ln_f.weight"], None, 1e-5)  # :224
    if train_causal:
        return F.linear(x, W["lm_head.weight"]), new_cache
    return F.linear(x[:, [-1], :], W["lm_head.weight"]), new_cache  # :234


def build_input(text_row, speech_row):
    """a4: normalize(cat(text, speech), p=2, eps=1e-8) (streaming_server.py:332-334)."""
    v = torch.cat([text_row, speech_row], dim=2)
    return F.normalize(v, p=2, dim=2, eps=1e-8)


def greedy_token(logits):
    """a11: softmax -> argmax (first max) -> int (streaming_server.py:342-346)."""
    probs = F.softmax(logits[:, -1, :], dim=-1)
    return int(probs.argmax(dim=-1).item())


def ar_decode(W, text_table, codebook, text_ids: List[int], n_steps: int, pad_id: int = 384,
              record_logits: bool = False):
    """The per-token loop of audio_generator_sync restricted to one segment
    (streaming_server.py:323-354): step i feeds text id text_ids[i] (PAD once the
    text is exhausted) and the codebook row of the previous token (zeros at i=0).
    Returns ids, top1-top2 logit margins and (optionally) logits."""
    ids, margins, logits_all = [], [], []
    hist, kv, prev = None, None, None
    for i in range(n_steps):
        tid = text_ids[i] if i < len(text_ids) else pad_id
        te = text_table[tid].view(1, 1, -1)
        se = torch.zeros(1, 1, 512) if i == 0 else codebook[prev].view(1, 1, -1)
        x = build_input(te, se)
        hist = x if hist is None else torch.cat([hist, x], dim=1)  # :337-338
        logits, kv = gpt_forward(W, hist, kv)
        prev = greedy_token(logits)
        top2 = torch.topk(logits[0, -1], 2).values
        ids.append(prev)
        margins.append(float(top2[0] - top2[1]))
        if record_logits:
            logits_all.append(logits[0, -1].clone())
    return ids, margins, (torch.stack(logits_all) if record_logits else None)


def teacher_forced_logits(W, text_table, codebook, text_ids, tokens, pad_id=384):
    """Full-sequence causal pass over the inputs that the ids ``tokens`` induce
    (the training form, src/data.py:239-288 semantics)."""
    rows = []
    for i in range(len(tokens)):
        tid = text_ids[i] if i < len(text_ids) else pad_id
        te = text_table[tid].view(1, 1, -1)
        se = torch.zeros(1, 1, 512) if i == 0 else codebook[tokens[i - 1]].view(1, 1, -1)
        rows.append(build_input(te, se))
    emb = torch.cat(rows, dim=1)
    logits, _ = gpt_forward(W, emb, None, train_causal=True)
    return logits[0]


# ---------------------------------------------------------------------------
# a3, a13-a21: codec decode (WavTokenizer/decoder/*)
# ---------------------------------------------------------------------------

CODEBOOK_KEY = "feature_extractor.encodec.quantizer.vq.layers.0._codebook.embed"


def codes_to_features(Wc, codes):
    """pretrained.py:209-239 with n_q=1: codes (K, L) or (K, B, L) -> [B,512,L].
    A 2-D input is (K, L) with K codebooks (so only [1, L] is valid with n_q=1)."""
    if codes.dim() == 2:
        codes = codes.unsqueeze(1)
    K = codes.shape[0]
    idx = codes + torch.arange(0, 4096 * K, 4096).view(-1, 1, 1)
    feats = F.embedding(idx, Wc[CODEBOOK_KEY]).sum(dim=0)
    return feats.transpose(1, 2)


def _gn(x, w, b):
    return F.group_norm(x, 32, w, b, 1e-6)  # models.py:15-16


def _swish(x):
    return x * torch.sigmoid(x)  # models.py:10-12


def resnet_block(Wc, p, x):  # models.py:58-78 (temb None, dropout identity in eval)
    h = _swish(_gn(x, Wc[p + "norm1.weight"], Wc[p + "norm1.bias"]))
    h = F.conv1d(h, Wc[p + "conv1.weight"], Wc[p + "conv1.bias"], padding=1)
    h = _swish(_gn(h, Wc[p + "norm2.weight"], Wc[p + "norm2.bias"]))
    h = F.conv1d(h, Wc[p + "conv2.weight"], Wc[p + "conv2.bias"], padding=1)
    return x + h


def attn_block(Wc, p, x):  # models.py:107-127
    h = _gn(x, Wc[p + "norm.weight"], Wc[p + "norm.bias"])
    q = F.conv1d(h, Wc[p + "q.weight"], Wc[p + "q.bias"])
    k = F.conv1d(h, Wc[p + "k.weight"], Wc[p + "k.bias"])
    v = F.conv1d(h, Wc[p + "v.weight"], Wc[p + "v.bias"])
    b, c, L = q.shape
    w = torch.bmm(q.permute(0, 2, 1), k) * (int(c) ** (-0.5))
    w = F.softmax(w, dim=2).permute(0, 2, 1)
    h = torch.bmm(v, w)
    return x + F.conv1d(h, Wc[p + "proj_out.weight"], Wc[p + "proj_out.bias"])


def ada_ln(Wc, p, x, bw):  # modules.py:81-86, x [B,L,C]
    scale = Wc[p + "scale.weight"][bw]
    shift = Wc[p + "shift.weight"][bw]
    return F.layer_norm(x, (x.shape[-1],), eps=1e-6) * scale + shift


def convnext_block(Wc, p, x, bw):  # modules.py:43-60
    r = x
    x = F.conv1d(x, Wc[p + "dwconv.weight"], Wc[p + "dwconv.bias"], padding=3, groups=x.shape[1])
    x = ada_ln(Wc, p + "norm.", x.transpose(1, 2), bw)
    x = F.linear(x, Wc[p + "pwconv1.weight"], Wc[p + "pwconv1.bias"])
    x = F.gelu(x)
    x = F.linear(x, Wc[p + "pwconv2.weight"], Wc[p + "pwconv2.bias"])
    x = Wc[p + "gamma"] * x
    return r + x.transpose(1, 2)


def backbone(Wc, feats, bw=0):  # models.py:223-235
    x = F.conv1d(feats, Wc["backbone.embed.weight"], Wc["backbone.embed.bias"], padding=3)
    for i in (0, 1):
        x = resnet_block(Wc, f"backbone.pos_net.{i}.", x)
    x = attn_block(Wc, "backbone.pos_net.2.", x)
    for i in (3, 4):
        x = resnet_block(Wc, f"backbone.pos_net.{i}.", x)
    x = _gn(x, Wc["backbone.pos_net.5.weight"], Wc["backbone.pos_net.5.bias"])
    x = ada_ln(Wc, "backbone.norm.", x.transpose(1, 2), bw).transpose(1, 2)
    for i in range(12):
        x = convnext_block(Wc, f"backbone.convnext.{i}.", x, bw)
    return F.layer_norm(x.transpose(1, 2), (x.shape[1],), Wc["backbone.final_layer_norm.weight"],
                        Wc["backbone.final_layer_norm.bias"], 1e-6)


def istft_same(spec, n_fft=1280, hop=320):  # spectral_ops.py:33-75 (padding "same")
    win = torch.hann_window(n_fft)
    pad = (n_fft - hop) // 2
    B, N, T = spec.shape
    ifft = torch.fft.irfft(spec, n_fft, dim=1, norm="backward") * win[None, :, None]
    out_size = (T - 1) * hop + n_fft
    y = F.fold(ifft, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop))[:, 0, 0, pad:-pad]
    wsq = win.square().expand(1, T, -1).transpose(1, 2)
    env = F.fold(wsq, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop)).squeeze()[pad:-pad]
    assert (env > 1e-11).all()
    return y / env


def head(Wc, x):  # heads.py:42-67
    x = F.linear(x, Wc["head.out.weight"], Wc["head.out.bias"]).transpose(1, 2)
    mag, p = x.chunk(2, dim=1)
    mag = torch.clip(torch.exp(mag), max=1e2)
    S = mag * (torch.cos(p) + 1j * torch.sin(p))
    return istft_same(S)


def decode(Wc, feats, bw=0):  # pretrained.py:192-207
    return head(Wc, backbone(Wc, feats, bw))


def decode_codes(Wc, codes: torch.Tensor, bw=0):
    """codes [B, L] -> PCM [B, 320 L]; streams decoded independently, as the
    reference does per dump."""
    feats = F.embedding(codes, Wc[CODEBOOK_KEY]).transpose(1, 2)
    return decode(Wc, feats, bw)


# ---------------------------------------------------------------------------
# 8f.4: WavTokenizer.encode_infer (decoder/pretrained.py:185-190 -> feature_extractors.py:122-133):
# SEANet encoder (encoder/modules/seanet.py:94-143) + the 1-codebook quantizer's inference path
# (encoder/quantization/vq.py:115-140, core_vq.py:171-231, 245-276, 296-310). Weights: the effective
# dict of llmvox_amd.weights.encoder_effective (weight_norm resolved) + the codebook.
# ---------------------------------------------------------------------------

ENC_PREFIX = "feature_extractor.encodec.encoder.model."


def _enc_pad(x, k_eff, stride):
    """SConv1d's non-causal padding (encoder/modules/conv.py:54-61, 79-96, 195-211): reflect with
    padding_total = k_eff - stride split right-heavy-last, plus the extra right padding that makes the
    last window full; inputs no longer than the pad are zero-extended before reflecting."""
    L = x.shape[-1]
    pt = k_eff - stride
    n_frames = (L - k_eff + pt) / stride + 1
    extra = (math.ceil(n_frames) - 1) * stride + (k_eff - pt) - L
    pr = pt // 2
    pl = pt - pr
    right = pr + extra
    max_pad = max(pl, right)
    ex0 = max_pad - L + 1 if L <= max_pad else 0
    if ex0:
        x = F.pad(x, (0, ex0))
    y = F.pad(x, (pl, right), "reflect")
    return y[..., :y.shape[-1] - ex0]


def enc_conv(We, name, x, stride=1, dilation=1, elu=False):
    """[ELU ->] SConv1d (conv.py:195-211) on x [B, C, T]."""
    if elu:
        x = F.elu(x)  # nn.ELU(alpha=1.0)
    w = We[ENC_PREFIX + name + ".conv.conv.weight"]
    b = We[ENC_PREFIX + name + ".conv.conv.bias"]
    k_eff = (w.shape[-1] - 1) * dilation + 1
    return F.conv1d(_enc_pad(x, k_eff, stride), w, b, stride, 0, dilation)


def enc_lstm(We, x):
    """SLSTM (encoder/modules/lstm.py:31-39): 2-layer nn.LSTM over time, + the input (skip)."""
    lstm = torch.nn.LSTM(512, 512, 2)
    p = ENC_PREFIX + "13.lstm."
    with torch.no_grad():
        for n, t in lstm.named_parameters():
            t.copy_(We[p + n])
        y, _ = lstm(x.permute(2, 0, 1))
    return y.permute(1, 2, 0) + x


def seanet_encode(We, audio):
    """audio [B, N] -> embedding [B, 512, T] (seanet.py:94-143; ratios [2, 4, 5, 8])."""
    x = enc_conv(We, "0", audio.unsqueeze(1))
    idx = 1
    for ratio in (2, 4, 5, 8):
        h = enc_conv(We, f"{idx}.block.1", x, elu=True)      # ELU -> conv k3 (dim -> dim / 2)
        h = enc_conv(We, f"{idx}.block.3", h, elu=True)      # ELU -> conv k1 (dim / 2 -> dim)
        x = enc_conv(We, f"{idx}.shortcut", x) + h           # seanet.py:63-64
        x = enc_conv(We, f"{idx + 2}", x, stride=ratio, elu=True)
        idx += 3
    x = enc_lstm(We, x)
    return enc_conv(We, "15", x, elu=True)


def vq_encode(codebook, emb):
    """emb [B, 512, T] -> codes [B, T] (core_vq.py:175-183: argmax of -(|x|^2 - 2 x.e + |e|^2))."""
    x = emb.permute(0, 2, 1).reshape(-1, emb.shape[1])
    embed = codebook.t()
    dist = -(x.pow(2).sum(1, keepdim=True) - 2 * x @ embed + embed.pow(2).sum(0, keepdim=True))
    return dist.max(dim=-1).indices.view(emb.shape[0], emb.shape[2]), dist


def encode_infer(We, codebook, audio):
    """pretrained.py:185-190: (features [B, 512, T] = codebook rows of the codes, codes [1, B, T])."""
    emb = seanet_encode(We, audio)
    codes, _ = vq_encode(codebook, emb)
    feats = F.embedding(codes, codebook).transpose(1, 2)
    return feats, codes.unsqueeze(0)
