"""CPU test: the demapper's fast root search (Newton + replayed bisection,
qamr_math.hpp::g_inv_search_fast) is bit-identical to the reference search
(noisemapper.pyx:310-345 restated as qamr_math.hpp::g_inv_search), compiled
for the host with hipcc over random targets, orders, SNRs and sign configs."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def test_fast_search_bit_identical(tmp_path):
    src = os.path.join(ROOT, "tests", "native", "replay_check.cpp")
    exe = str(tmp_path / "replay_check")
    csrc = os.path.join(ROOT, "qam-reconciliation_amd", "csrc")
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc unavailable")
    subprocess.run([sys.executable, os.path.join(csrc, "gen_glibc_tables.py"), str(tmp_path / "glibc_tables.inc")],
                   check=True)
    cc = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-std=c++17",
                         "-I" + csrc, "-I" + str(tmp_path), "-o", exe, src], capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr[-2000:]
    run = subprocess.run([exe, "120000"], capture_output=True, text=True, timeout=300)
    print(run.stdout)
    assert run.returncode == 0, run.stdout
    assert "mismatches=0" in run.stdout
    # the fast path itself must be exercised: Newton certifies ~91 % of these draws (the rest
    # are the edge targets n = 0 / 1, 1e-12-deep tails and -2 dB spreads: brute force)
    import re
    m = re.search(r"draws=(\d+) mismatches=\d+ fallbacks=(\d+)", run.stdout)
    assert m and int(m.group(2)) < 0.15 * int(m.group(1)), run.stdout


def test_llr_exponent_division_bit_identical(tmp_path):
    """qamr_math.hpp::div_two_s2 (reciprocal + FMA correction) == IEEE x / (2 sigma^2)."""
    src = os.path.join(ROOT, "tests", "native", "division_check.cpp")
    exe = str(tmp_path / "division_check")
    csrc = os.path.join(ROOT, "qam-reconciliation_amd", "csrc")
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc unavailable")
    subprocess.run([sys.executable, os.path.join(csrc, "gen_glibc_tables.py"), str(tmp_path / "glibc_tables.inc")],
                   check=True)
    cc = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-std=c++17",
                         "-I" + csrc, "-I" + str(tmp_path), "-o", exe, src], capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr[-2000:]
    run = subprocess.run([exe, "20000000"], capture_output=True, text=True, timeout=300)
    print(run.stdout)
    assert run.returncode == 0, run.stdout
    assert "mismatches=0" in run.stdout
