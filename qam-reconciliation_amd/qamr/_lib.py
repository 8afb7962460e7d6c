"""ctypes binding of libqamr.so (declared in include/qamr.h).

There is no CPU fallback: if the library or a HIP device is missing, every
compute entry point raises.  ``load()`` only needs the shared object (it works
on a CPU-only host, for symbol checks).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# QAMR_LIB overrides the library path (experiment builds, scripts/exp_build.sh).
LIB_PATH = os.environ.get("QAMR_LIB") or os.path.join(_HERE, "libqamr.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

QR_OK, QR_EVALUE, QR_EMEMORY, QR_EDEVICE, QR_EUNSUPPORTED = 0, 1, 2, 3, 4

_lib = None

vp = C.c_void_p
i32, i64, f64, u8 = C.c_int32, C.c_int64, C.c_double, C.c_uint8
P = C.POINTER

# name -> (argtypes); restype is int unless listed in _RESTYPE.
SIGNATURES = {
    "qr_last_error": [],
    "qr_version": [P(i32), P(i32)],
    "qr_device_count": [P(i32)],
    "qr_profile_enable": [i32],
    "qr_profile_reset": [],
    "qr_profile_select": [C.c_char_p],
    "qr_profile_query": [C.c_char_p, P(f64), P(i64)],
    "qr_tune_set": [C.c_char_p, i64],
    "qr_tune_get": [C.c_char_p, P(i64)],
    "qr_code_create": [vp, vp, i64, i64, i32, P(vp)],
    "qr_code_destroy": [vp],
    "qr_code_info": [vp, P(i64), P(i64), P(i64), P(i32), P(i32)],
    "qr_decode_workspace_size": [vp, i32, i32, P(C.c_size_t)],
    "qr_decode_batch_device": [vp, i32, i32, vp, vp, i32, vp, vp, vp, vp, C.c_size_t, vp],
    "qr_decode_repack_stats": [vp, i32, i32, vp, C.c_size_t, P(C.c_int32)],
    "qr_decode_host": [vp, i32, vp, vp, i32, vp, vp, vp],
    "qr_check_lappr_host": [vp, vp, vp, vp, vp],
    "qr_check_word_host": [vp, vp, vp, vp, vp],
    "qr_process_var_nodes_host": [vp, vp, i64, vp, vp, vp, vp],
    "qr_process_check_nodes_host": [vp, vp, i64, vp, vp, vp],
    "qr_demap_create": [i32, vp, vp, vp, f64, vp, i32, P(vp)],
    "qr_demap_destroy": [vp],
    "qr_demap_tables": [vp, vp, vp],
    "qr_demap_batch_device": [vp, i32, i32, i64, vp, vp, f64, vp, vp],
    "qr_demap_host": [vp, i64, vp, vp, vp],
    "qr_g_inv_search_host": [vp, i64, vp, vp, f64, vp],
    "qr_F_Y_host": [vp, i64, vp, vp],
    "qr_bob_map_device": [vp, i32, i32, i64, vp, vp, vp, vp, vp],
    "qr_map_noise_device": [vp, i32, i32, i64, vp, vp, vp, vp],
    "qr_syndrome_device": [vp, i32, i32, vp, vp, vp],
    "qr_symbols_to_bits_device": [i32, i32, i32, i64, vp, vp, vp],
    "qr_direct_lappr_device": [vp, f64, i32, i32, i64, vp, vp, vp],
    "qr_bare_llr_device": [i32, vp, i32, i32, i64, vp, vp, vp],
    "qr_count_errors_device": [i32, i32, i64, vp, vp, vp, vp, vp, vp, vp],
    "qr_to_frame_innermost_f64": [i32, i32, i64, vp, vp, vp],
    "qr_to_frame_major_f64": [i32, i32, i64, vp, vp, vp],
    "qr_to_frame_innermost_u8": [i32, i32, i64, vp, vp, vp],
    "qr_to_frame_innermost_i64": [i32, i32, i64, vp, vp, vp],
    "qr_stream_copy": [vp, vp, i64, vp],
    "qr_clock_probe": [vp, i32, i64, vp],
}
_RESTYPE = {"qr_last_error": C.c_char_p}


class QamrError(RuntimeError):
    pass


def build(verbose: bool = False) -> str:
    """Compile libqamr.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    jobs = min(3, os.cpu_count() or 1)
    subprocess.run(["make", "-s" if not verbose else "-w", f"-j{jobs}", "-C", CSRC], check=True)
    return LIB_PATH


def load():
    """Load the shared object (no device needed)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C {CSRC}` or __graft_entry__.build(). "
            "qamr has no CPU fallback.")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7.  If
    # libqamr were loaded first it would pull /opt/rocm's copy (same soname)
    # and torch would then load a second runtime that sees no GPU.  Importing
    # torch first makes libqamr bind to the runtime torch already loaded.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        if os.environ.get("QAMR_LIB") and not hasattr(L, name):
            continue  # an experiment build of an older interface (scripts/exp_*): only what it exports
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, C.c_int)
    _lib = L
    # QAMR_TUNE="knob=value,knob=value" presets the kernel-geometry knobs (qr_tune_set).
    for item in filter(None, os.environ.get("QAMR_TUNE", "").split(",")):
        k, v = item.split("=")
        check(L.qr_tune_set(k.strip().encode(), int(v)), "QAMR_TUNE")
    return L


def last_error() -> str:
    msg = load().qr_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = ""):
    if rc == QR_OK:
        return
    msg = last_error() or what
    if rc == QR_EVALUE:
        raise ValueError(msg)
    if rc == QR_EMEMORY:
        raise MemoryError(msg)
    raise QamrError(f"{what}: {msg}" if what else msg)


def device_count() -> int:
    n = i32(0)
    load().qr_device_count(C.byref(n))
    return int(n.value)


def require_gpu():
    if device_count() <= 0:
        raise QamrError("no HIP device visible: qamr runs only on the GPU (no CPU fallback)")


def ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


# ------------------------------------------------------------------ tuning
def tune_set(name: str, value: int):
    check(load().qr_tune_set(name.encode(), int(value)))


def tune_get(name: str) -> int:
    v = i64(0)
    check(load().qr_tune_get(name.encode(), C.byref(v)))
    return int(v.value)


# ------------------------------------------------------------------ profiling
def profile_enable(on: bool = True):
    check(load().qr_profile_enable(1 if on else 0))


def profile_reset():
    check(load().qr_profile_reset())


def profile_select(names=None):
    """Time only the launches named in ``names`` (iterable or comma-separated string);
    None = every launch."""
    if names is not None and not isinstance(names, str):
        names = ",".join(names)
    check(load().qr_profile_select((names or "").encode()))


def profile_query(name: str):
    ms, n = f64(0), i64(0)
    check(load().qr_profile_query(name.encode(), C.byref(ms), C.byref(n)))
    return float(ms.value), int(n.value)


def check_tensor(t, name: str, shape=None, dtype=None, device: int | None = None):
    """Validate a device tensor before its pointer crosses the C-ABI: the kernels
    index it as a dense row-major array of `shape` on GPU `device`, so a wrong
    dtype / shape / stride / device would be read or written out of bounds."""
    import torch

    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{name}: expected a torch tensor, got {type(t).__name__}")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor")
    if device is not None and t.device.index != device:
        raise ValueError(f"{name}: on cuda:{t.device.index}, expected cuda:{device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous (the kernels assume dense rows)")
    return t
