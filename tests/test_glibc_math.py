"""Host check of glibc_math.hpp, the strict box-plus arithmetic: the restated glibc
exp/log (and h(t) = log(1.0 + exp(-t)), box-plus built on them) must return the same
bits as the host libm -- the reference's own arithmetic (decoder.pyx:41-45) -- on
~16M inputs dense on the decoder's domain.  Compiled for the host with hipcc; the
tables are regenerated from libm into tmp_path (gen_glibc_tables.py)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "qam-reconciliation_amd", "csrc")


def test_glibc_exp_log_restatement_bit_exact(tmp_path):
    subprocess.run([sys.executable, os.path.join(CSRC, "gen_glibc_tables.py"), str(tmp_path / "glibc_tables.inc")],
                   check=True)
    exe = str(tmp_path / "glibc_math_check")
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc unavailable")
    cc = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-ffp-contract=off", "-std=c++17", "-I" + CSRC,
                         "-I" + str(tmp_path), "-o", exe, os.path.join(ROOT, "tests", "native", "glibc_math_check.cpp")],
                        capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr[-2000:]
    run = subprocess.run([exe, "4000000"], capture_output=True, text=True, timeout=300)
    print(run.stdout)
    assert run.returncode == 0, run.stdout
