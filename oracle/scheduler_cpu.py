"""CPU oracle objects that plug into an ``audio_generator_sync``-style loop.

TEST INFRASTRUCTURE / CPU BASELINE ONLY.

``OracleHandler`` exposes the ``ModelHandler`` members that the reference
scheduler touches (inference/model_handler.py:45-63, used at
streaming_server.py:271-383): ``.device``, ``.tokenizer``, ``.llm_model``,
``.wavtokenizer.codes_to_features/.decode`` and ``.model`` — computed by the
fp32 CPU restatement in ``oracle.reference_cpu``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import reference_cpu as R


class _OracleGPT:
    def __init__(self, W):
        self.W = W

    def __call__(self, emb, targets=None, kvcache=None):
        logits, kv = R.gpt_forward(self.W, emb, kvcache)
        return logits, None, kv


class _OracleWavTokenizer:
    def __init__(self, Wc):
        self.Wc = Wc

    def codes_to_features(self, codes):
        return R.codes_to_features(self.Wc, codes)

    def decode(self, features, bandwidth_id=None):
        bw = 0 if bandwidth_id is None else int(bandwidth_id.view(-1)[0])
        return R.decode(self.Wc, features, bw)


class _OracleEmbed:
    def __init__(self, table):
        self.table = table

    def __call__(self, ids):
        return F.embedding(ids.cpu(), self.table)


def byt5_tokenizer():
    """The reference tokenizer: ByT5 + "[PAD]" (384) + "EOS" (385)
    (inference/model_handler.py:89-102)."""
    from transformers import ByT5Tokenizer
    t = ByT5Tokenizer()
    t.add_special_tokens(dict(pad_token="[PAD]"))
    t.add_special_tokens(dict(pad_token="EOS"))
    return t


class OracleHandler:
    def __init__(self, gpt_w, codec_w, text_table, tokenizer=None):
        self.device = torch.device("cpu")
        self.model = _OracleGPT(R.to_torch(gpt_w))
        self.wavtokenizer = _OracleWavTokenizer(R.to_torch(codec_w))
        self.llm_model = _OracleEmbed(torch.from_numpy(text_table))
        self.tokenizer = tokenizer or byt5_tokenizer()
