"""8f.4 upstream text producer (CPU): llm_streaming.StreamModel on a tiny random-init causal LM
built here (no network: the tokenizer and model are written to a temporary directory and loaded
back with local_files_only), and text_streamer_producer's routing (streaming_server.py:184-248)."""
from queue import Queue

import pytest


def _tiny_llm(path):
    """a word-level tokenizer with a chat template + a 2-layer Llama, saved like a HF checkpoint"""
    import torch
    from tokenizers import Tokenizer, models, pre_tokenizers, decoders
    from transformers import LlamaConfig, LlamaForCausalLM, PreTrainedTokenizerFast
    words = ("the quick brown fox jumps over lazy dog near river bank . hello how are you i am fine "
             "thank tell me about a story short answer yes no").split()
    specials = ["<unk>", "<pad>", "<|begin_of_text|>", "<|eot_id|>", "<|start_header_id|>", "<|end_header_id|>",
                "system", "user", "assistant"]
    vocab = {w: i for i, w in enumerate(specials + words)}
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    tk.decoder = decoders.WordPiece(prefix="##", cleanup=False)
    fast = PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="<unk>", pad_token="<pad>",
                                   bos_token="<|begin_of_text|>", eos_token="<|eot_id|>")
    fast.add_special_tokens({"additional_special_tokens": ["<|start_header_id|>", "<|end_header_id|>"]})
    fast.chat_template = ("{% for m in messages %}<|start_header_id|> {{ m['role'] }} <|end_header_id|> "
                          "{{ m['content'] }} <|eot_id|> {% endfor %}"
                          "{% if add_generation_prompt %}<|start_header_id|> assistant <|end_header_id|> {% endif %}")
    fast.save_pretrained(path)
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=len(vocab), hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256,
                      bos_token_id=vocab["<|begin_of_text|>"], eos_token_id=vocab["<|eot_id|>"],
                      pad_token_id=vocab["<pad>"])
    LlamaForCausalLM(cfg).save_pretrained(path)
    return path


def test_stream_model_streams_text_pieces(tmp_path):
    from llmvox_amd.llm_streaming import StreamModel
    path = _tiny_llm(str(tmp_path / "llm"))
    sm = StreamModel({"llm_checkpoint": path, "llm_device": "cpu", "llm_max_tokens": 12}).load()
    out = list(sm.predict({"system": "be brief", "prompt": "tell me about the fox"}))
    assert out and all(isinstance(p, str) and p.strip() for p in out)
    assert len(out) <= 12


class _Scripted:
    def __init__(self, pieces):
        self.pieces = pieces
        self.req = None

    def predict(self, request):
        self.req = dict(request)
        return iter(self.pieces)


def _drain(q):
    out = []
    while not q.empty():
        out.append(q.get())
    return out


def test_producer_routes_sentences_to_alternating_replicas():
    from llmvox_amd.llm_streaming import text_streamer_producer
    from llmvox_amd import config as C
    llm = _Scripted(["Sure", "-", " Mr.", " Fox", " jumps **high**.", "", " The", " dog & cat...", " sleep.",
                     " End<|eot_id|>"])
    q1, q2 = Queue(), Queue()
    routed = text_streamer_producer("tell me", llm, q1, q2)
    assert llm.req == {"system": C.SYSTEM_PROMPT, "prompt": "tell me"}
    # skip '' and '-', strip, clean_text (not the EOS piece), switch after a piece ending with '.'
    assert _drain(q1) == ["Sure", "Mr.", "The", "dog and cat pause ", "sleep."]
    assert _drain(q2) == ["Fox", "jumps high.", "End<|eot_id|>"]
    assert routed == ["Sure", "Mr.", "Fox", "jumps high.", "The", "dog and cat pause ", "sleep.", "End<|eot_id|>"]


def test_producer_appends_the_end_of_turn_token_when_the_llm_stops_at_max_tokens():
    from llmvox_amd.llm_streaming import text_streamer_producer
    q1, q2 = Queue(), Queue()
    routed = text_streamer_producer("x", _Scripted(["Hello", " there"]), q1, q2, {"eos_token": "<|eot_id|>"})
    assert routed == ["Hello", "there", "<|eot_id|>"]
    assert _drain(q1) == ["Hello", "there", "<|eot_id|>"] and q2.empty()


@pytest.mark.gpu
def test_stream_model_on_the_gpu(tmp_path):
    """the same tiny LM in bf16 on the ROCm device (SDPA attention), as ModelHandler's
    initialize_stream_model loads it"""
    from llmvox_amd.llm_streaming import StreamModel
    path = _tiny_llm(str(tmp_path / "llm"))
    sm = StreamModel({"llm_checkpoint": path, "llm_device": "cuda:0", "llm_max_tokens": 16}).load()
    assert next(sm.model.parameters()).device.type == "cuda"
    out = list(sm.predict({"system": "be brief", "prompt": "hello how are you"}))
    assert out and len(out) <= 16
