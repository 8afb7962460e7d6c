"""Host check of the table-driven h(t) = log(1+exp(-t)) and box-plus of fastmath.hpp
against glibc (the reference's arithmetic, decoder.pyx:41-45): |error| <= ulp(1) for h,
NaN/inf behaviour of the reference.  Compiled for the host with hipcc."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def test_fastmath_h_and_box_plus(tmp_path):
    src = os.path.join(ROOT, "tests", "native", "fastmath_check.cpp")
    exe = str(tmp_path / "fastmath_check")
    csrc = os.path.join(ROOT, "qam-reconciliation_amd", "csrc")
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc unavailable")
    subprocess.run([sys.executable, os.path.join(csrc, "gen_glibc_tables.py"), str(tmp_path / "glibc_tables.inc")],
                   check=True)
    cc = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-std=c++17",
                         "-I" + csrc, "-I" + str(tmp_path), "-o", exe, src], capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr[-2000:]
    run = subprocess.run([exe, "2000000"], capture_output=True, text=True, timeout=300)
    print(run.stdout)
    assert run.returncode == 0, run.stdout
