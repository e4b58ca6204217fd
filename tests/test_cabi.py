"""The C-ABI library loads and exports every symbol include/llmvox.h declares (no compute)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "llmvox.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(lvx_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    from llmvox_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "llmvox_amd", "csrc"), "-j8"], check=True)
    return _lib.load()


def test_every_declared_symbol_is_exported(lib):
    names = _declared()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n


def test_bindings_cover_the_header():
    from llmvox_amd import _lib
    assert sorted(_lib.EXPORTED_SYMBOLS) == _declared()


def test_version_and_error_string(lib):
    assert lib.lvx_version() >= 1
    assert isinstance(lib.lvx_last_error(), bytes)


def test_create_rejects_bad_config(lib):
    from llmvox_amd import _lib
    cfg = _lib.LvxConfig(0, 7, 0, 1, 16, 16)  # bad weight dtype: argument check before any HIP call
    h = ctypes.c_void_p()
    rc = lib.lvx_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc == _lib.LVX_E_ARG
    assert b"weight_dtype" in lib.lvx_last_error()


def test_no_compat_layers_in_sources():
    src = os.path.join(ROOT, "llmvox_amd", "csrc")
    for f in os.listdir(src):
        if f.endswith((".hip", ".cpp", ".h")):
            t = open(os.path.join(src, f)).read()
            assert "__HIP_PLATFORM_AMD__" not in t and "cuda" not in t.lower().replace("accum", ""), f


def test_error_status_names_every_set_bit(lib):
    """Device error bits (AR word | codec word << 16) map to one status, the most specific condition
    (index > state > capacity), with every set condition named in the message (an
    index error set together with another one was lost). A host-only call: no GPU needed."""
    from llmvox_amd import _lib
    assert lib.lvx_error_status(0) == _lib.LVX_OK
    assert lib.lvx_error_status(1) == _lib.LVX_E_CAPACITY
    assert lib.lvx_error_status(32 | 1) == _lib.LVX_E_STATE
    code = lib.lvx_error_status(1 | 32 | (4 << 16) | (8 << 16))
    assert code == _lib.LVX_E_INDEX
    msg = lib.lvx_last_error().decode()
    for part in ("codec: a code outside", "fused MLP", "ISTFT window envelope", "KV capacity"):
        assert part in msg, (part, msg)
    with pytest.raises(_lib.LvxIndexError) as ei:
        _lib.check_bits(1 | (4 << 16))
    assert ei.value.bits == 1 | (4 << 16) and "KV capacity" in str(ei.value)
    with pytest.raises(_lib.LvxNumericError):
        _lib.check_bits(32)
    with pytest.raises(_lib.LvxCapacityError):
        _lib.check_bits(2)
