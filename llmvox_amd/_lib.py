"""ctypes binding of libllmvox_hip.so (include/llmvox.h).

The library is built in-tree (``__graft_entry__.build()`` / ``make -C llmvox_amd/csrc``)
and MUST be present: there is no CPU fallback anywhere in the product path.
``torch`` is imported first so that the process's single HIP runtime is torch's.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime that the library then shares)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LVX_LIB_PATH") or os.path.join(_HERE, "libllmvox_hip.so")  # override: A/B builds

LVX_OK = 0
LVX_E_ARG = -1
LVX_E_STATE = -2
LVX_E_HIP = -3
LVX_E_CAPACITY = -4
LVX_E_NAME = -5
LVX_E_INDEX = -6
LVX_DTYPE_F32 = 0
LVX_DTYPE_BF16 = 1
LVX_DTYPE_FP8 = 2  # kv_dtype only (OCP e4m3fn)

DTYPES = {"fp32": LVX_DTYPE_F32, "f32": LVX_DTYPE_F32, "float32": LVX_DTYPE_F32,
          "bf16": LVX_DTYPE_BF16, "bfloat16": LVX_DTYPE_BF16,
          "fp8": LVX_DTYPE_FP8, "e4m3": LVX_DTYPE_FP8}


class LvxConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("weight_dtype", ctypes.c_int), ("kv_dtype", ctypes.c_int),
                ("max_streams", ctypes.c_int), ("max_positions", ctypes.c_int),
                ("max_codec_frames", ctypes.c_int), ("codec_dtype", ctypes.c_int)]


class LvxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[lvx {code}] {msg}")
        self.code = code


class LvxStreamError(LvxError):
    """A device error that concerns particular streams; the scheduler names them in ``streams``
    (the service then ends only their requests)."""
    streams = ()


class LvxCapacityError(LvxStreamError, AssertionError):
    """Capacity overflow: the reference raises AssertionError here (src/model.py:205)."""


class LvxNumericError(LvxStreamError):
    """A non-finite / out-of-range partial in the B <= 2 fused MLP (error bit 32): the logits of the
    rows of that step are invalid."""


class LvxArgError(LvxError, ValueError):
    pass


class LvxIndexError(LvxError, IndexError):
    """An embedding id out of range: the reference's nn.Embedding raises IndexError."""


_P = ctypes.c_void_p
_I = ctypes.c_int
_SIGS = {
    "lvx_create": (_I, [ctypes.POINTER(LvxConfig), ctypes.POINTER(_P)]),
    "lvx_destroy": (None, [_P]),
    "lvx_last_error": (ctypes.c_char_p, []),
    "lvx_version": (_I, []),
    "lvx_set_weight": (_I, [_P, ctypes.c_char_p, _P, ctypes.c_int64]),
    "lvx_finalize": (_I, [_P]),
    "lvx_missing_weights": (_I, [_P, ctypes.POINTER(ctypes.c_char_p)]),
    "lvx_text_embed": (_I, [_P, _P, _I, _P, _P]),
    "lvx_codes_to_features": (_I, [_P, _P, _I, _I, _P, _P]),
    "lvx_stream_reset": (_I, [_P, _I, _P]),
    "lvx_ar_forward_row": (_I, [_P, _I, _I, _P, _P, _P]),
    "lvx_ar_step": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _P]),
    "lvx_ar_steps": (_I, [_P, _I, _I, _P, _P, _I, _P, _P, _P, _P]),
    "lvx_check_errors": (_I, [_P, _P]),
    "lvx_error_take": (_I, [_P, _I, _P, _P]),
    "lvx_error_status": (_I, [_I]),
    "lvx_ar_logits": (_I, [_P, _I, _P, _P]),
    "lvx_probe_kernel": (_I, [_P, _I, _I, _P, _I, _P]),
    "lvx_stream_set": (_I, [_P, _I, _I, _I, _P]),
    "lvx_select_probe": (_I, [_P, _I, _I, _P, _P, _P, _I, _P, _P, _P, _P]),
    "lvx_stream_position": (_I, [_P, _I, ctypes.POINTER(_I), _P]),
    "lvx_set_graphs": (_I, [_P, _I]),
    "lvx_set_capture_stream": (_I, [_P, _P]),
    "lvx_set_option": (_I, [_P, ctypes.c_char_p, _I]),
    "lvx_codec_decode_features": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "lvx_codec_decode_codes": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "lvx_enc_create": (_I, [_I, ctypes.c_longlong, ctypes.POINTER(_P)]),
    "lvx_enc_set_weight": (_I, [_P, ctypes.c_char_p, _P, ctypes.c_int64]),
    "lvx_enc_finalize": (_I, [_P]),
    "lvx_enc_destroy": (None, [_P]),
    "lvx_enc_frames": (_I, [_I]),
    "lvx_encode": (_I, [_P, _P, _I, _I, _P, _P, _P]),
    "lvx_enc_embedding": (_I, [_P, _P, _I, _I, _P]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


def load():
    """Load the library (raises if it was not built — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "or `make -C llmvox_amd/csrc` (hipcc, gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


ERRW_AR = 1     # LVX_ERRW_AR: the decode / drop-in gather error word
ERRW_CODEC = 2  # LVX_ERRW_CODEC: the codec's error word
BIT_NUMERIC = 32  # AR word: the fused MLP's fixed-point range check


def error_for(code: int, bits: int = 0):
    """The exception for a non-zero status (``bits``: the taken device error bits, if known)."""
    msg = _lib.lvx_last_error().decode(errors="replace") if _lib else "unknown"
    if code == LVX_E_CAPACITY:
        e = LvxCapacityError(code, msg)
    elif code == LVX_E_INDEX:
        e = LvxIndexError(code, msg)
    elif code in (LVX_E_ARG, LVX_E_NAME):
        e = LvxArgError(code, msg)
    elif code == LVX_E_STATE and bits & BIT_NUMERIC:
        e = LvxNumericError(code, msg)
    else:
        e = LvxError(code, msg)
    e.bits = bits
    return e


def check(code: int):
    if code != LVX_OK:
        raise error_for(code)


def check_bits(bits: int):
    """Raise for device error bits taken with lvx_error_take (every set condition in the message)."""
    if bits:
        raise error_for(load().lvx_error_status(int(bits)), int(bits))
