"""WavTokenizer encoder on the HIP library: ``encode_infer`` of
WavTokenizer/decoder/pretrained.py:185-190 (SEANet encoder + the 1-codebook quantiser), fp32.

Owns one ``lvx_enc`` context (its own weights and scratch: the TTS path does not need them).
Audio in, (features [B, 512, T], codes [1, B, T]) out, on the device, asynchronous on torch's
current stream; T = ceil(N / 320).
"""
from __future__ import annotations

import ctypes
from typing import Dict

import numpy as np
import torch

from . import _lib
from . import weights as LW


class WavEncoder:
    def __init__(self, device_index: int, encoder_weights: Dict[str, np.ndarray], codebook: np.ndarray,
                 max_samples: int = 24000 * 30):
        """encoder_weights: reference state_dict entries (weight_g / weight_v pairs or resolved
        '.conv.conv.weight'), e.g. llmvox_amd.weights.synthetic_encoder() or a WavTokenizer checkpoint."""
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("llmvox_amd needs a ROCm GPU (MI355X); there is no CPU path")
        self.device = torch.device(f"cuda:{device_index}")
        self.max_samples = int(max_samples)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.lvx_enc_create(device_index, self.max_samples, ctypes.byref(h)))
        self.h = h
        eff = LW.encoder_effective(encoder_weights) if any(k.endswith("weight_g") for k in encoder_weights) \
            else encoder_weights
        for k, v in list(eff.items()) + [(LW.CODEBOOK_KEY, codebook)]:
            if not k.startswith(LW.ENC_PREFIX) and k != LW.CODEBOOK_KEY:
                continue
            a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
            _lib.check(self.lib.lvx_enc_set_weight(self.h, k.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size))
        with torch.cuda.device(self.device):
            _lib.check(self.lib.lvx_enc_finalize(self.h))

    def frames(self, n_samples: int) -> int:
        return int(self.lib.lvx_enc_frames(int(n_samples)))

    def encode(self, audio: torch.Tensor):
        """audio [B, N] (or [N]) -> (features [B, 512, T] fp32, codes [1, B, T] int64)."""
        if audio.dim() == 1:
            audio = audio.unsqueeze(0)
        if audio.dim() != 2:
            raise ValueError("audio must be [B, N] (mono)")
        a = audio.to(self.device, torch.float32).contiguous()
        B, N = a.shape
        T = self.frames(N)
        feats = torch.empty(B, 512, T, dtype=torch.float32, device=self.device)
        codes = torch.empty(B, T, dtype=torch.int32, device=self.device)
        s = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.lvx_encode(self.h, ctypes.c_void_p(a.data_ptr()), B, N, ctypes.c_void_p(feats.data_ptr()),
                                       ctypes.c_void_p(codes.data_ptr()), s))
        return feats, codes.long().unsqueeze(0)

    def embedding(self, B: int, T: int) -> torch.Tensor:
        """the pre-quantisation embedding [B, 512, T] of the last encode (test hook)"""
        out = torch.empty(B, T, 512, dtype=torch.float32, device=self.device)
        s = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.lvx_enc_embedding(self.h, ctypes.c_void_p(out.data_ptr()), B, T, s))
        return out.permute(0, 2, 1)

    def close(self):
        if getattr(self, "h", None):
            self.lib.lvx_enc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
