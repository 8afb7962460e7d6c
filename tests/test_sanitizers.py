"""SURVEY.md §5 sanitizers: the host-side code under AddressSanitizer + UndefinedBehavior-
Sanitizer (CPU only; GPU ASan is not available on the MI355X pool).

* oracle/qamr_oracle.c (the C restatement: CSR build, node rules, decode with inf/NaN/-0.0,
  NoiseMapper tables, demap, Bob side) driven by oracle/asan_main.c (`make -C oracle asan`);
* libqamr's host code: the Tanner-graph CSR builder and the NoiseMapper / fast-search table
  builders (csrc/host_build.hpp), glibc/fast-math tables, and the per-symbol demapper on the
  host (tests/native/host_asan_check.cpp, hipcc with -Xarch_host -fsanitize=...).

Both run with -fno-sanitize-recover=all: any report is a non-zero exit."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "qam-reconciliation_amd", "csrc")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def _run(exe):
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=ENV)
    out = r.stdout + r.stderr
    print(out[-3000:])
    assert r.returncode == 0, out[-3000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out


def test_oracle_under_asan_ubsan():
    if not shutil.which("gcc"):
        pytest.skip("gcc unavailable")
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], capture_output=True, text=True)
    assert b.returncode == 0, b.stderr[-2000:]
    _run(os.path.join(ROOT, "oracle", "_asan", "oracle_asan"))


def test_libqamr_host_code_under_asan_ubsan(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc unavailable")
    subprocess.run([sys.executable, os.path.join(CSRC, "gen_glibc_tables.py"), str(tmp_path / "glibc_tables.inc")],
                   check=True)
    exe = str(tmp_path / "host_asan_check")
    san = []
    for f in ("-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=all"):
        san += ["-Xarch_host", f]
    cc = subprocess.run([hipcc, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-ffp-contract=off",
                         "-fno-fast-math", "-fno-omit-frame-pointer", *san, "-I" + CSRC, "-I" + str(tmp_path),
                         "-I" + os.path.join(ROOT, "include"), "-o", exe,
                         os.path.join(ROOT, "tests", "native", "host_asan_check.cpp")],
                        capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr[-3000:]
    _run(exe)
