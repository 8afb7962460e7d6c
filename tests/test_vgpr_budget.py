"""The register note of decoder.hip as a guard (CPU: reads the built gfx950 code object).

On MI355X the kernels that run on the variable stream BESIDE the degree-7 check sweep -- the
paced variable sweep k_var and the repack decision / row-move kernel k_repack_rows -- must
allocate 16 or 32 VGPRs, never 24: the check waves hold 4 x 120 of a SIMD's 512 VGPRs, and a
24-VGPR kernel beside them cost the headline 2.5-2.7 % (9 547 vs 9 790 frames/s, same box,
profiles/r05/ab/p_register_allocation.log; DESIGN.md "Register allocation beside the check
waves").  The allocation is read from the library's amdhsa metadata (.vgpr_count), so an edit
that moves one of these kernels to 24 fails here instead of silently costing the headline."""
import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
LIB = os.path.join(ROOT, "qam-reconciliation_amd", "qamr", "libqamr.so")


@pytest.fixture(scope="module")
def res():
    if not os.path.exists(LIB):
        pytest.skip("libqamr.so not built")
    import kernel_resources as K

    ks = K.kernels(LIB)
    dm = K.demangle([k.removesuffix(".kd") for k in ks])
    return {dm[k.removesuffix(".kd")]: v for k, v in ks.items()}


def _find(res, prefix):
    got = {k: v for k, v in res.items() if k.startswith(prefix)}
    assert got, f"no kernel {prefix!r} in the code object"
    return got


def test_check_sweep_leaves_32_vgprs(res):
    # the dominant launch at 4 waves/SIMD with at most 120 VGPRs: 32 of the 512 stay free
    for name, r in _find(res, "void qr::k_check<7, 1, ").items():
        assert r["vgpr"] <= 120, (name, r)
        assert r["scratch"] == 0, (name, r)


def test_variable_sweep_allocates_16(res):
    # two 16-VGPR variable waves per SIMD beside the check waves (32 measured -2.7 %)
    for name, r in _find(res, "void qr::k_var<false, ").items():
        assert r["vgpr"] == 16, (name, r)


def test_repack_rows_allocates_32_not_24(res):
    for name, r in _find(res, "qr::k_repack_rows(").items():
        assert r["vgpr"] in (16, 32), (name, r)
        assert r["vgpr"] != 24 and r["scratch"] == 0, (name, r)


def test_side_kernels_never_24(res):
    # everything else the variable stream launches during the loop: the small check-degree
    # classes (knob side) -- their own occupancy rules apply, but none may land on 24
    for prefix in ("void qr::k_check<6, 1, ", "void qr::k_var<"):
        for name, r in _find(res, prefix).items():
            assert r["vgpr"] != 24, (name, r)
