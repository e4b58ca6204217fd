"""Byte-level tokenizer equal to the reference's ByT5 tokenizer + its two added tokens.

Reference: inference/model_handler.py:89-102 builds ``AutoTokenizer(google/byt5-small)``
and adds "[PAD]" (id 384) then "EOS" (id 385); streaming_server.py:306 calls
``tokenizer(word)["input_ids"]``.  ByT5 ids: 0 <pad>, 1 </s>, 2 <unk>, 3 + byte value for
UTF-8 bytes, 259 + n for <extra_id_n> (n < 125), and "</s>" appended at the end.
Special tokens are matched in the text (longest match first); "<pad>", "</s>" and "<unk>"
also swallow the whitespace around them (their AddedToken has lstrip/rstrip=True). The
trailing </s> is not added again when the ids already end with </s>.
"""
from __future__ import annotations

import re
from typing import Dict, List

_STRIP_SPECIALS = {"<pad>": 0, "</s>": 1, "<unk>": 2}
_PLAIN_SPECIALS = {"[PAD]": 384, "EOS": 385}
_PLAIN_SPECIALS.update({f"<extra_id_{n}>": 259 + n for n in range(125)})


def _build_regex():
    alts = sorted(list(_STRIP_SPECIALS) + list(_PLAIN_SPECIALS), key=len, reverse=True)
    parts = []
    for a in alts:
        e = re.escape(a)
        parts.append(rf"\s*{e}\s*" if a in _STRIP_SPECIALS else e)
    return re.compile("|".join(parts))


_RX = _build_regex()


class ByteTokenizer:
    """``tokenizer(text)["input_ids"]`` -> ByT5 ids (with the trailing </s> = 1)."""

    pad_token_id = 384
    eos_text_id = 385
    vocab_size = 386

    def encode(self, text: str) -> List[int]:
        ids: List[int] = []
        pos = 0
        for m in _RX.finditer(text):
            if m.start() > pos:
                ids.extend(b + 3 for b in text[pos:m.start()].encode("utf-8"))
            tok = m.group(0).strip() if m.group(0).strip() in _STRIP_SPECIALS else m.group(0)
            ids.append(_STRIP_SPECIALS.get(tok, _PLAIN_SPECIALS.get(tok)))
            pos = m.end()
        if pos < len(text):
            ids.extend(b + 3 for b in text[pos:].encode("utf-8"))
        if not ids or ids[-1] != 1:  # ByT5 appends </s> only when the ids do not already end with it
            ids.append(1)
        return ids

    def __call__(self, text: str) -> Dict[str, List[int]]:
        return {"input_ids": self.encode(text)}

    def __len__(self):
        return self.vocab_size
