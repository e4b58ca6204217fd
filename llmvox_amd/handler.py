"""Drop-in ``ModelHandler`` for the reference's streaming scheduler.

Reference: inference/model_handler.py:45-166. ``streaming_server.audio_generator_sync``
(streaming_server.py:250-426) only touches these members, with these signatures:

  .device                                        torch.device
  .tokenizer(str)["input_ids"]                   -> list[int]          (:306)
  .llm_model(LongTensor[1, n])                   -> FloatTensor[1,n,256] (:315, :319)
  .wavtokenizer.codes_to_features(Long[1, L])    -> FloatTensor[1,512,L] (:329, :364, :382)
  .wavtokenizer.decode(F[1,512,L], bandwidth_id) -> FloatTensor[1,320L]  (:365, :383)
  .model(F[1,t,768], kvcache=None|handle)        -> (logits[1,1,4096], None, handle) (:341)

Every member runs on the HIP library (libllmvox_hip.so); nothing falls back to CPU.
"""
from __future__ import annotations

import threading
import weakref
from typing import Optional

import torch

from . import config as C
from .engine import Engine
from .tokenizer import ByteTokenizer
from . import weights as LW


def _check_ids(ids: torch.Tensor, n: int):
    """nn.Embedding's IndexError for ids outside [0, n), raised at the call as the reference does
    when the ids are on the host (the reference builds them there, streaming_server.py:313-314,
    328, 363). Device-resident ids are checked by the gather kernel instead (LVX_E_INDEX, raised as
    IndexError by the next Engine.check_errors) so the call stays asynchronous."""
    if ids.device.type == "cpu" and ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= n):
        raise IndexError("index out of range in self")


class _SlotLease:
    """One KV slot owned by one decode sequence; returned to the pool when the last
    handle of the sequence is garbage-collected (the reference drops its cache by
    rebinding ``kvcache = None``, streaming_server.py:412)."""

    def __init__(self, pool, slot):
        self.slot = slot
        self.length = 0
        self.generation = 0
        self._fin = weakref.finalize(self, pool._release, slot)


class KVHandle:
    """Opaque, truthy stand-in for the reference's list of [K, V] tensors. It holds the
    sequence length so the next call can check that exactly one row was appended."""

    __slots__ = ("lease", "length", "generation", "__weakref__")

    def __init__(self, lease: _SlotLease):
        self.lease = lease
        self.length = lease.length
        self.generation = lease.generation

    def __bool__(self):
        return True

    def __len__(self):  # the reference's cache is a list with one entry per layer
        return C.N_LAYER


class _SlotPool:
    def __init__(self, n):
        self.free = list(range(n - 1, -1, -1))
        self.lock = threading.Lock()

    def acquire(self, owner) -> _SlotLease:
        with self.lock:
            if not self.free:
                raise RuntimeError("all KV slots are in use (raise config max_streams)")
            s = self.free.pop()
        return _SlotLease(self, s)

    def _release(self, slot):
        with self.lock:
            self.free.append(slot)


class SpeechGPT:
    """``.model``: GPT.forward(emb, targets=None, kvcache=None) of src/model.py:201-237 at
    inference (is_train False). Only the last row of ``emb`` is computed; its position is
    t-1 and K/V of the earlier rows live in the library's slot for this sequence."""

    def __init__(self, engine: Engine, pool: _SlotPool, block_size: int = C.BLOCK_SIZE):
        self.engine = engine
        self.pool = pool
        self.config = C
        self.block_size = int(block_size)

    def __call__(self, emb: torch.Tensor, targets=None, kvcache=None):
        if targets is not None:
            raise NotImplementedError("training forward (targets) is outside the hot path")
        if emb.dim() != 3 or emb.shape[0] != 1 or emb.shape[2] != C.N_EMBD:
            raise ValueError(f"expected emb [1, t, {C.N_EMBD}], got {tuple(emb.shape)}")
        t = emb.shape[1]
        assert t <= self.block_size, f"Cannot forward sequence of length {t}, block size is only {self.block_size}"
        if not kvcache:
            if t != 1:
                raise NotImplementedError(
                    "a cache-less forward over t > 1 rows is a non-causal prefill (is_causal=False at "
                    "inference, src/model.py:92-93); the streaming path always starts at t = 1")
            lease = self.pool.acquire(self)
            lease.length = 0
        else:
            if not isinstance(kvcache, KVHandle):
                raise TypeError("kvcache must be a handle returned by this model")
            lease = kvcache.lease
            if kvcache.generation != lease.generation or kvcache.length != t - 1:
                raise ValueError(f"kvcache holds {kvcache.length} positions but emb has {t} rows; the caller "
                                 "must append exactly one row per step")
        row = emb[0, t - 1].to(self.engine.device, torch.float32).contiguous()
        logits = torch.empty(1, 1, C.VOCAB, device=self.engine.device, dtype=torch.float32)
        self.engine.forward_row(lease.slot, t - 1, row, logits)
        lease.length = t
        lease.generation += 1
        return logits, None, KVHandle(lease)

    def eval(self):
        return self


class TextEmbedding:
    """``.llm_model``: the T5 ``encoder.embed_tokens`` lookup (model_handler.py:105)."""

    def __init__(self, engine: Engine):
        self.engine = engine
        self.num_embeddings = C.TEXT_VOCAB
        self.embedding_dim = C.TEXT_DIM

    def __call__(self, ids: torch.Tensor) -> torch.Tensor:
        _check_ids(ids, C.TEXT_VOCAB)
        return self.engine.text_embed(ids)


class WavTokenizerDecoder:
    """``.wavtokenizer``: codes_to_features + decode of WavTokenizer
    (decoder/pretrained.py:192-239) for the yaml the reference ships (n_q = 1), and encode_infer
    (pretrained.py:185-190) on its own encoder context, built on first use."""

    def __init__(self, engine: Engine, encoder_weights=None, codebook=None, max_encode_samples: int = 24000 * 30):
        self.engine = engine
        self._enc_src = (encoder_weights, codebook, int(max_encode_samples))
        self._enc = None

    def encode_infer(self, audio_input: torch.Tensor, bandwidth_id=None, **kw):
        """audio [B, N] at 24 kHz -> (features [B, 512, T], codes [1, B, T]) as the reference returns them"""
        if self._enc is None:
            from .encoder import WavEncoder
            ew, cb, ms = self._enc_src
            if ew is None or not any(k.startswith(LW.ENC_PREFIX) for k in ew):
                raise KeyError("no WavTokenizer encoder weights (the checkpoint holds only the decode path)")
            self._enc = WavEncoder(self.engine.device_index, ew, cb, ms)
        return self._enc.encode(audio_input)

    def codes_to_features(self, codes: torch.Tensor) -> torch.Tensor:
        # pretrained.py:226-239: a 2-D input is (K, L), a 3-D input (K, B, L); K = n_q = 1.
        if codes.dim() == 2:
            codes = codes.unsqueeze(1)
        if codes.dim() != 3:
            raise ValueError("codes must be (K, L) or (K, B, L)")
        if codes.shape[0] != 1:
            raise IndexError("index out of range in self (n_q = 1: only one codebook)")
        _check_ids(codes, C.VOCAB)
        return self.engine.codes_to_features(codes[0])

    def decode(self, features_input: torch.Tensor, bandwidth_id: Optional[torch.Tensor] = None, **kw):
        if bandwidth_id is None:
            raise AssertionError("bandwidth_id is required (adanorm backbone, decoder/models.py:226-227)")
        bw = int(bandwidth_id.reshape(-1)[0]) if isinstance(bandwidth_id, torch.Tensor) else int(bandwidth_id)
        return self.engine.decode_features(features_input, bw)

    def to(self, *a, **k):
        return self

    def eval(self):
        return self


class ModelHandler:
    """``ModelHandler(config, device_id)`` (inference/model_handler.py:48-63).

    ``config`` is the reference's dict plus: weights "synthetic" | "checkpoint",
    weight_dtype "fp32" | "bf16", kv_dtype, codec_dtype (None | "fp8"), max_streams, max_positions, seed."""

    def __init__(self, config, device_id: Optional[int] = None):
        self.config = config
        if not torch.cuda.is_available():
            raise RuntimeError("llmvox_amd.ModelHandler needs a ROCm GPU; there is no CPU path")
        dev = 0 if device_id is None else int(device_id)
        get = config.get if hasattr(config, "get") else (lambda k, d=None: getattr(config, k, d))
        src = get("weights", "synthetic")
        if src == "synthetic":
            gw, cw, tt = LW.synthetic_all(int(get("seed", 1234)))
        else:  # the reference's three checkpoints (model_handler.py:80-106,140-166)
            gw = LW.load_llmvox_checkpoint(get("llmvox_checkpoint_path"))
            cw = LW.load_wavtokenizer_checkpoint(get("wav_model_path"))
            tt = LW.load_text_embed_from_t5(_load_t5_state(get("encoder_model_path")))
        block = int(getattr(gw, "block_size", C.BLOCK_SIZE))
        self.engine = Engine(dev, get("weight_dtype", "fp32"), get("kv_dtype", "fp32"),
                             int(get("max_streams", 8)), min(int(get("max_positions", C.BLOCK_SIZE)), block),
                             int(get("max_codec_frames", C.MAX_DUMP_SIZE)), get("codec_dtype", None))
        self.device = self.engine.device
        self.engine.load_weights(gw, cw, tt)
        ew = LW.synthetic_encoder(int(get("seed", 1234))) if src == "synthetic" else cw
        self.wavtokenizer = WavTokenizerDecoder(self.engine, ew, cw[LW.CODEBOOK_KEY],
                                                int(get("max_encode_samples", 24000 * 30)))
        self.tokenizer = ByteTokenizer()
        self.llm_model = TextEmbedding(self.engine)
        self.model = SpeechGPT(self.engine, _SlotPool(self.engine.max_streams), block)

    def initialize_stream_model(self):
        """the LLM text streamer (model_handler.py:108-118; llm_streaming.StreamModel on PyTorch-ROCm,
        config["llm_checkpoint"] a local path)"""
        from .llm_streaming import StreamModel
        return StreamModel(self.config).load()

    # the VLM / multimodal producers are out of scope
    def initialize_vlm_model(self):
        raise NotImplementedError("VLM producers are outside the TTS path (SURVEY §2)")

    initialize_stream_multimodal = initialize_vlm_model


def _load_t5_state(path):
    """T5 weights from a local directory (safetensors or pytorch_model.bin via weights_only)."""
    import os
    if path and os.path.isdir(path):
        st = os.path.join(path, "model.safetensors")
        if os.path.exists(st):
            from safetensors.numpy import load_file
            return load_file(st)
        binp = os.path.join(path, "pytorch_model.bin")
        sd = torch.load(binp, map_location="cpu", weights_only=True)
        return {k: v.float().numpy() for k, v in sd.items()}
    raise FileNotFoundError(f"T5 encoder weights not found at {path!r} (no network access)")
