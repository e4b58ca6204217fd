"""Thin Python owner of one ``lvx_ctx`` (one device): weights, KV slots, entry points.

Every compute method is asynchronous on the device's current torch stream and takes /
returns torch device tensors (torch is only the allocator and the stream provider here).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .weights import CODEBOOK_KEY, TEXT_EMBED_KEY


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Engine:
    def __init__(self, device_index: int = 0, weight_dtype: str = "fp32", kv_dtype: str = "fp32",
                 max_streams: int = 8, max_positions: int = 8192, max_codec_frames: int = 1280,
                 codec_dtype: Optional[str] = None):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("llmvox_amd needs a ROCm GPU (MI355X); there is no CPU path")
        self.device = torch.device(f"cuda:{device_index}")
        self.device_index = device_index
        cfg = _lib.LvxConfig(device_index, _lib.DTYPES[weight_dtype], _lib.DTYPES[kv_dtype], max_streams,
                             max_positions, max_codec_frames, _lib.DTYPES[codec_dtype] if codec_dtype else 0)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.lvx_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self._capture_stream = None
        self.weight_dtype = weight_dtype
        self.kv_dtype = kv_dtype
        self.codec_dtype = codec_dtype or weight_dtype
        self.max_streams = max_streams
        self.max_positions = max_positions
        self.max_codec_frames = max_codec_frames
        self.finalized = False

    # ---- weights ----------------------------------------------------------------
    def set_weight(self, name: str, arr):
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
        _lib.check(self.lib.lvx_set_weight(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size))

    def load_weights(self, gpt: Dict[str, np.ndarray], codec: Dict[str, np.ndarray], text_table: np.ndarray):
        for k, v in gpt.items():
            if k.endswith("attn.bias"):  # causal-mask buffer of the no-flash path, not a weight
                continue
            self.set_weight(k, v)
        for k, v in codec.items():
            if k == "head.istft.window":
                continue
            self.set_weight(k, v)
        self.set_weight(TEXT_EMBED_KEY, text_table)
        # exactly torch's periodic Hann window (decoder/spectral_ops.py:30-31)
        self.set_weight("head.istft.window", torch.hann_window(1280).numpy())
        with torch.cuda.device(self.device):
            _lib.check(self.lib.lvx_finalize(self.h))
        self.finalized = True

    # ---- helpers ----------------------------------------------------------------
    def stream_handle(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ---- drop-in members -------------------------------------------------------------
    def text_embed(self, ids: torch.Tensor) -> torch.Tensor:
        ids = ids.to(self.device, torch.int64).contiguous()
        out = torch.empty(*ids.shape, 256, device=self.device, dtype=torch.float32)
        _lib.check(self.lib.lvx_text_embed(self.h, _ptr(ids), ids.numel(), _ptr(out), self.stream_handle()))
        return out

    def codes_to_features(self, codes: torch.Tensor) -> torch.Tensor:
        """codes int [B, L] -> [B, 512, L]."""
        codes = codes.to(self.device, torch.int64).contiguous()
        B, L = codes.shape
        out = torch.empty(B, 512, L, device=self.device, dtype=torch.float32)
        _lib.check(self.lib.lvx_codes_to_features(self.h, _ptr(codes), B, L, _ptr(out), self.stream_handle()))
        return out

    def forward_row(self, slot: int, pos: int, row: torch.Tensor, logits: torch.Tensor):
        _lib.check(self.lib.lvx_ar_forward_row(self.h, slot, pos, _ptr(row), _ptr(logits), self.stream_handle()))

    def reset_slot(self, slot: int):
        _lib.check(self.lib.lvx_stream_reset(self.h, slot, self.stream_handle()))

    def set_slot(self, slot: int, pos: int, prev_token: int = 0):
        _lib.check(self.lib.lvx_stream_set(self.h, slot, pos, prev_token, self.stream_handle()))

    def slot_position(self, slot: int) -> int:
        v = ctypes.c_int()
        _lib.check(self.lib.lvx_stream_position(self.h, slot, ctypes.byref(v), self.stream_handle()))
        return v.value

    def ar_steps(self, n_steps: int, slots: torch.Tensor, text_plan: torch.Tensor, rowstep: torch.Tensor,
                 tok_plan: torch.Tensor, margin_plan: Optional[torch.Tensor] = None):
        B, stride = text_plan.shape
        self._capture_guard()
        _lib.check(self.lib.lvx_ar_steps(self.h, n_steps, B, _ptr(slots), _ptr(text_plan), stride, _ptr(rowstep),
                                         _ptr(tok_plan), _ptr(margin_plan), self.stream_handle()))

    def probe_kernel(self, which: int, slots: torch.Tensor, iters: int):
        self._capture_guard()
        _lib.check(self.lib.lvx_probe_kernel(self.h, which, slots.numel(), _ptr(slots), iters, self.stream_handle()))

    def select_probe(self, path: int, slots: torch.Tensor, logits: torch.Tensor, text_plan: torch.Tensor,
                     rowstep: torch.Tensor, tok_plan: torch.Tensor, margin_plan: Optional[torch.Tensor] = None):
        """Test hook: one production select path (0 argmax kernel, 1 deferred lm_head granules,
        2 batched deferred select) over the given logits [B, 4096], committed as a step commits."""
        B, stride = text_plan.shape
        logits = logits.to(self.device, torch.float32).contiguous()
        _lib.check(self.lib.lvx_select_probe(self.h, path, B, _ptr(slots), _ptr(logits), _ptr(text_plan), stride,
                                             _ptr(rowstep), _ptr(tok_plan), _ptr(margin_plan), self.stream_handle()))

    def last_logits(self, B: int) -> torch.Tensor:
        out = torch.empty(B, 4096, device=self.device, dtype=torch.float32)
        _lib.check(self.lib.lvx_ar_logits(self.h, B, _ptr(out), self.stream_handle()))
        return out

    def check_errors(self):
        """Synchronise the current stream and raise for the device error bits of both words (AR and
        codec); every set condition is named in the message."""
        code = self.lib.lvx_check_errors(self.h, self.stream_handle())
        if code:
            raise _lib.error_for(code)

    def take_errors(self, which: int, out: torch.Tensor):
        """Enqueue (no synchronisation) the atomic take of the AR (``_lib.ERRW_AR``) and / or codec
        (``_lib.ERRW_CODEC``) error bits into the device int32 ``out[0]``; ``_lib.check_bits`` on the
        host copy raises for them."""
        _lib.check(self.lib.lvx_error_take(self.h, int(which), _ptr(out), self.stream_handle()))

    def set_option(self, name: str, value: int):
        _lib.check(self.lib.lvx_set_option(self.h, name.encode(), int(value)))

    def set_capture_stream(self, stream: Optional["torch.cuda.Stream"]):
        """Capture the decode graphs on `stream` (None: on the caller's stream), lvx_set_capture_stream."""
        self._capture_stream = stream
        _lib.check(self.lib.lvx_set_capture_stream(self.h, ctypes.c_void_p(stream.cuda_stream if stream else None)))

    def _capture_guard(self):
        # Once an RCCL process group exists, its watchdog thread queries the events that synchronous
        # collectives record on the current stream, and HIP refuses that query while the stream is
        # capturing (lvx_api.cpp cached_graph): capture on a pooled stream of torch's that nothing else
        # records on. Not before: one more stream per process cost two ranks sharing a GPU 6.5x.
        # (a pooled stream may come round again as the caller's: never capture on the stream called on)
        if self._capture_stream is None:
            if not (dist.is_available() and dist.is_initialized() and "nccl" in str(dist.get_backend()).lower()):
                return
        elif self._capture_stream.cuda_stream != torch.cuda.current_stream(self.device).cuda_stream:
            return
        cur = torch.cuda.current_stream(self.device).cuda_stream
        s = torch.cuda.Stream(device=self.device)
        while s.cuda_stream == cur:
            s = torch.cuda.Stream(device=self.device)
        self.set_capture_stream(s)

    def set_graphs(self, enable: bool):
        _lib.check(self.lib.lvx_set_graphs(self.h, int(enable)))

    def decode_features(self, feats: torch.Tensor, bandwidth_id: int = 0) -> torch.Tensor:
        feats = feats.to(self.device, torch.float32).contiguous()
        B, C, L = feats.shape
        if C != 512:
            raise ValueError(f"features must be [B, 512, L], got {tuple(feats.shape)}")
        pcm = torch.empty(B, 320 * L, device=self.device, dtype=torch.float32)
        _lib.check(self.lib.lvx_codec_decode_features(self.h, _ptr(feats), B, L, int(bandwidth_id), _ptr(pcm),
                                                      self.stream_handle()))
        return pcm

    def decode_codes(self, codes: torch.Tensor, bandwidth_id: int = 0, out: Optional[torch.Tensor] = None):
        codes = codes.to(self.device, torch.int32).contiguous()
        B, L = codes.shape
        pcm = out if out is not None else torch.empty(B, 320 * L, device=self.device, dtype=torch.float32)
        _lib.check(self.lib.lvx_codec_decode_codes(self.h, _ptr(codes), B, L, int(bandwidth_id), _ptr(pcm),
                                                   self.stream_handle()))
        return pcm

    def close(self):
        if getattr(self, "h", None):
            self.lib.lvx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def build_engine(device_index=0, weight_dtype="fp32", kv_dtype="fp32", seed=1234, max_streams=8,
                 max_positions=8192, max_codec_frames=1280, weights=None, codec_dtype=None) -> Engine:
    """Engine loaded with ``weights`` = (gpt, codec, text_table) or the seeded synthetic set.
    codec_dtype "fp8": codec GEMM weights stored as e4m3fn with per-row scales (configs[4])."""
    from .weights import synthetic_all
    gw, cw, tt = weights if weights is not None else synthetic_all(seed)
    # a checkpoint trained with a smaller block_size has zero-padded wpe rows past it: positions
    # there must raise (the reference asserts t <= block_size, src/model.py:205), so the KV
    # capacity never exceeds it
    max_positions = min(int(max_positions), int(getattr(gw, "block_size", max_positions)))
    e = Engine(device_index, weight_dtype, kv_dtype, max_streams, max_positions, max_codec_frames, codec_dtype)
    e.load_weights(gw, cw, tt)
    return e


__all__ = ["Engine", "build_engine", "CODEBOOK_KEY"]
