import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the libqamr kernels")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def has_gpu():
    try:
        import qamr
        return qamr.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    import qamr
    if qamr.device_count() <= 0:
        pytest.fail("GPU test selected but no HIP device is visible (qamr has no CPU fallback)")
    return 0


# LAPPR tolerance (north_star: "within 1e-6 on final LLRs"): relative 1e-6 of
# the reference value with an absolute floor for values near zero.
LLR_RTOL = 1e-6
LLR_ATOL = 1e-9


def assert_llr_close(got, ref, rtol=LLR_RTOL, atol=LLR_ATOL):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape
    nan_g, nan_r = np.isnan(got), np.isnan(ref)
    assert np.array_equal(nan_g, nan_r), f"NaN pattern differs ({nan_g.sum()} vs {nan_r.sum()})"
    inf_r = np.isinf(ref)
    assert np.array_equal(got[inf_r], ref[inf_r]), "inf entries differ"
    m = ~(nan_r | inf_r)
    err = np.abs(got[m] - ref[m])
    lim = rtol * np.abs(ref[m]) + atol
    bad = err > lim
    assert not bad.any(), f"{bad.sum()} LAPPRs out of tolerance; worst |d|={err.max():.3e}"


def assert_bit_exact(got, ref):
    """Identical doubles (signed zeros included); NaN matches NaN whatever its payload.
    The decoder's arithmetic (glibc_math.hpp, the only one) reproduces the
    reference's exp/log, so its outputs must equal the reference's bit for bit."""
    got = np.ascontiguousarray(got, np.float64)
    ref = np.ascontiguousarray(ref, np.float64)
    assert got.shape == ref.shape
    nan_g, nan_r = np.isnan(got), np.isnan(ref)
    assert np.array_equal(nan_g, nan_r), f"NaN pattern differs ({nan_g.sum()} vs {nan_r.sum()})"
    m = ~nan_r
    diff = got[m].view(np.int64) != ref[m].view(np.int64)
    if diff.any():
        k = np.flatnonzero(diff)[0]
        raise AssertionError(f"{diff.sum()} of {m.sum()} values differ; first: got {got[m][k]!r} ref {ref[m][k]!r} "
                             f"(|d| = {abs(got[m][k] - ref[m][k]):.3e})")


# Debug-build runs (tests/test_gpu_debug_build.py): with QAMR_DEBUG_ASSERTS=1 the process has
# loaded libqamr_debug.so (QAMR_LIB) and every test must leave its device index checks unfailed.
@pytest.fixture(autouse=True)
def _device_checks(request):
    if os.environ.get("QAMR_DEBUG_ASSERTS") != "1" or request.node.get_closest_marker("gpu") is None:
        yield
        return
    import ctypes

    from qamr import _lib

    L = _lib.load()
    assert hasattr(L, "qr_debug_asserts"), "QAMR_DEBUG_ASSERTS=1 but the debug library is not loaded"
    fn = L.qr_debug_asserts
    fn.argtypes = [ctypes.c_void_p]
    out = (ctypes.c_int64 * 4)()
    assert fn(out) == 0
    yield
    assert fn(out) == 0
    assert out[0] == 0, f"{out[0]} device index checks failed; first: site {out[1]} values {out[2]}, {out[3]}"
