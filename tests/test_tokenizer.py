"""a1: the byte tokenizer == the reference's ByT5 tokenizer with "[PAD]" and "EOS" added."""
import json
import os
import random

import pytest

from llmvox_amd.tokenizer import ByteTokenizer

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_golden_cases():
    g = json.load(open(os.path.join(GOLDEN, "tokenizer_golden.json")))
    t = ByteTokenizer()
    for text, ids in g.items():
        assert t(text)["input_ids"] == ids, text


def test_config_sentence_has_66_ids():
    t = ByteTokenizer()
    words = "The quick brown fox jumps over the lazy dog near the river bank.".split(" ")
    n = sum(len(t(w)["input_ids"]) for w in words) + 1  # + EOS 385 at sentence end
    assert n == 66


def test_fuzz_against_transformers():
    tr = pytest.importorskip("transformers")
    ref = tr.ByT5Tokenizer()
    ref.add_special_tokens(dict(pad_token="[PAD]"))
    ref.add_special_tokens(dict(pad_token="EOS"))
    t = ByteTokenizer()
    rng = random.Random(0)
    alphabet = list("abcXYZ .,!?'-0123456789éü日") + ["EOS", "[PAD]", "</s>", "<pad>", "<unk>", " ", "  ",
                                                         "<extra_id_3>", "<extra_id_99>"]
    for _ in range(300):
        s = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 12)))
        assert t(s)["input_ids"] == ref(s)["input_ids"], repr(s)
