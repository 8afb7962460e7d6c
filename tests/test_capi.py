"""CPU tests of the C-ABI boundary: libqamr.so loads, exports every symbol
include/qamr.h declares, the ctypes table binds exactly that set, and the
product path refuses to run without a device (no CPU fallback)."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, has_gpu

HEADER = os.path.join(ROOT, "include", "qamr.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"QR_API\s+(?:const\s+char\s*\*|int)\s*(qr_\w+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = header_symbols()
    for s in ("qr_code_create", "qr_decode_batch_device", "qr_decode_host", "qr_demap_create",
              "qr_demap_batch_device", "qr_demap_host", "qr_last_error"):
        assert s in syms


def test_library_exports_every_header_symbol():
    import qamr
    from qamr import _lib

    L = qamr.load()
    for s in header_symbols():
        assert hasattr(L, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\sT\s(qr_\w+)", out))
    assert set(header_symbols()) == exported
    assert set(_lib.SIGNATURES) == set(header_symbols())


def test_library_is_gfx950_code_object():
    from qamr import _lib

    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob  # the embedded offload bundle targets gfx950


def test_no_cpu_fallback():
    if has_gpu():
        pytest.skip("device present")
    import qamr

    with pytest.raises(qamr.QamrError):
        qamr.Decoder(np.array([0, 1], np.int64), np.array([0, 0], np.int64))
    with pytest.raises(qamr.QamrError):
        qamr.NoiseMapper(qamr.PAMAlphabet(2, 2.0), 1.0)


def test_dtype_and_size_errors_before_device():
    import qamr

    with pytest.raises(ValueError):  # Cython buffer dtype semantics (decoder.pyx:93)
        qamr.Decoder(np.array([0, 1], np.int32), np.array([0, 0], np.int32))
    with pytest.raises(ValueError):
        qamr.Decoder(np.array([0, 1, 2], np.int64), np.array([0, 0], np.int64)) if has_gpu() else \
            _size_mismatch()


def _size_mismatch():
    # qr_code_create validates sizes before touching the device
    import ctypes as C

    from qamr import _lib

    h = C.c_void_p()
    a = np.array([0, 1, 2], np.int64)
    b = np.array([0, 0], np.int64)
    _lib.check(_lib.load().qr_code_create(_lib.ptr(a), _lib.ptr(b), 3, 2, 0, C.byref(h)))


def test_status_mapping():
    from qamr import _lib

    with pytest.raises(ValueError):
        _lib.check(_lib.QR_EVALUE)
    with pytest.raises(MemoryError):
        _lib.check(_lib.QR_EMEMORY)
    with pytest.raises(_lib.QamrError):
        _lib.check(_lib.QR_EDEVICE)
