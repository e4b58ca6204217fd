"""Upstream text producer of the streaming service: the LLM text streamer
(inference/llm_streaming.py:13-105) and the producer thread that routes its output to the two TTS
replicas (streaming_server.py:184-248).

``StreamModel`` keeps the reference's interface — ``StreamModel(config)``, ``.load()``,
``.predict({"system", "prompt"})`` returning a generator of text pieces — on PyTorch-ROCm:
``AutoModelForCausalLM`` in bf16 on ``config["llm_device"]`` with ``attn_implementation="sdpa"``
(the reference asks for flash_attention_2, a CUDA package; SDPA dispatches to ROCm's fused
attention), a ``TextIteratorStreamer`` fed by ``generate`` on a worker thread, sampling, at most
``config["llm_max_tokens"]`` new tokens, special tokens kept so the end-of-turn token reaches the
router. Checkpoints are read from a local path (no network). The LLM is not part of the TTS hot
path; it is the text source the reference's /tts endpoint streams into it.

This module is a behavioural restatement of the reference's Hugging Face glue, not an algorithm:
the chat-template / streamer / generation calls and their arguments are the ones the reference
makes, because the routed words (and so the TTS byte stream) must be the reference's for the same
checkpoint and seed.
"""
from __future__ import annotations

from queue import Queue
from threading import Thread
from typing import Dict, Generator, Iterable

from . import config as C
from .streaming import route_text


def _get(config, key, default=None):
    if hasattr(config, "get"):
        v = config.get(key, default)
    else:
        v = getattr(config, key, default)
    return default if v is None else v


class StreamModel:
    """Streaming text generation (inference/llm_streaming.py:13-105)."""

    def __init__(self, config) -> None:
        self.config = config
        self.tokenizer = None
        self.model = None
        self.device = _get(config, "llm_device", "cuda:0")

    def load(self):
        import torch
        from transformers import AutoModelForCausalLM, AutoTokenizer
        path = _get(self.config, "llm_checkpoint")
        self.tokenizer = AutoTokenizer.from_pretrained(path, local_files_only=True)
        self.model = AutoModelForCausalLM.from_pretrained(
            path, torch_dtype=torch.bfloat16, attn_implementation="sdpa", use_cache=True,
            local_files_only=True).to(self.device)
        self.model.eval()
        return self

    def predict(self, request: Dict) -> Generator[str, None, None]:
        """request {"system", "prompt"} -> generator of the reply's text pieces (empty pieces dropped)"""
        import torch
        from transformers import GenerationConfig, TextIteratorStreamer
        system = request.pop("system")
        prompt = request.pop("prompt")
        messages = [{"role": "system", "content": system}, {"role": "user", "content": prompt}]
        inputs = self.tokenizer.apply_chat_template(messages, tokenize=True, add_generation_prompt=True,
                                                    return_tensors="pt", return_dict=True).to(self.device)
        streamer = TextIteratorStreamer(self.tokenizer, skip_prompt=True, skip_special_tokens=False)
        gen_cfg = GenerationConfig(pad_token_id=self.tokenizer.pad_token_id, do_sample=True)
        kwargs = {"input_ids": inputs["input_ids"], "generation_config": gen_cfg, "return_dict_in_generate": True,
                  "output_scores": True, "pad_token_id": self.tokenizer.eos_token_id,
                  "max_new_tokens": int(_get(self.config, "llm_max_tokens", 1000)), "streamer": streamer}

        def run():
            with torch.no_grad():
                self.model.generate(**kwargs)

        thread = Thread(target=run, daemon=True)
        thread.start()

        def inner():
            try:
                for text in streamer:
                    if text.strip():
                        yield text
            finally:
                thread.join()

        return inner()


def llm_words(pieces: Iterable[str], eos: str) -> Generator[str, None, None]:
    """The producer's view of the stream (streaming_server.py:224-235): each streamed piece is one
    'output' (the reference splits nothing further); after the stream ends, the end-of-turn token
    follows if the model stopped at max_new_tokens without emitting it (the reference's consumers
    would otherwise wait on their queues forever)."""
    seen = False
    for p in pieces:
        seen = seen or eos in p
        yield p
    if not seen:
        yield eos


def text_streamer_producer(request_text: str, stream_model, text_token_queue_1: Queue, text_token_queue_2: Queue,
                           config=None):
    """streaming_server.py:184-248 for chat_type 'voice' / 'text' (the intended text path: the
    request text is the prompt; SURVEY 8f.3 notes the reference's `"text" in request` is always
    False for a pydantic model). Routes the LLM's reply to the two replicas' queues, switching after
    every piece that ends a sentence. Returns the routed outputs (the reference logs them)."""
    system = _get(config, "system_prompt", C.SYSTEM_PROMPT)
    eos = _get(config, "eos_token", C.EOS_TOKEN)
    stream = stream_model.predict({"system": system, "prompt": request_text})
    return route_text(llm_words(stream, eos), [text_token_queue_1, text_token_queue_2], eos=eos)
