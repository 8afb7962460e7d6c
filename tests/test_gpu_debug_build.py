"""The device-asserting debug build (the reference compiles with bounds checks off,
decoder.pyx:181,240,289,332,399,411, so the port adds them).  `make -C qam-reconciliation_amd/csrc
DEBUG=1` (also part of the default build) makes qamr/libqamr_debug.so: libqamr with QR_DEBUG_ASSERT
index checks (decoder.hip QR_DCHECK) on the column repack's active-frame list, frame ids and row-group
slots (k_repack_rows, k_repack_output), the active-frame list writes (k_compact) and reads
(lane_frame), the narrow sweeps' lane -> (node, frame) mapping, and the frame-resident decode's LDS
posterior and message indices (k_resident).  This test runs the repack parity tests (the bench's
4-PAM 4.0 dB and 16-PAM 14.5 dB B = 4096 batches: repacks in both directions between the column
sets, transitions, narrow sweeps; a short max_iterations; the captured decode), the schedule and
tuning invariance test, and the frame-resident parity tests (configs[1] full batch, ragged batch
shapes) in a child process on that library; conftest's autouse fixture fails any test after which a device check failed."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
DEBUG_LIB = os.path.join(ROOT, "qam-reconciliation_amd", "qamr", "libqamr_debug.so")

CASES = [
    "tests/test_gpu_timed_schedule.py::test_column_repack_vs_oracle[2-4.0-4096-50]",
    "tests/test_gpu_timed_schedule.py::test_column_repack_vs_oracle[4-14.5-4096-50]",
    "tests/test_gpu_timed_schedule.py::test_column_repack_vs_oracle[4-14.5-1024-50]",
    "tests/test_gpu_timed_schedule.py::test_column_repack_vs_oracle[2-4.0-1024-22]",
    "tests/test_gpu_timed_schedule.py::test_repack_decode_is_asynchronous_and_capturable",
    "tests/test_gpu_timed_schedule.py::test_repack_stats_after_resident_decode",
    "tests/test_gpu_properties.py::test_schedule_and_tuning_invariance",
    "tests/test_gpu_parity_edges.py::test_configs1_full_batch_vs_oracle",
    "tests/test_gpu_parity_edges.py::test_resident_batch_shapes_vs_oracle",
]


def test_debug_build_device_checks(gpu):
    assert os.path.exists(DEBUG_LIB), "libqamr_debug.so missing: run __graft_entry__.build() (make -C csrc)"
    env = dict(os.environ, QAMR_LIB=DEBUG_LIB, QAMR_DEBUG_ASSERTS="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *CASES], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "12 passed" in r.stdout, tail  # the 9 cases above (the batch-shape test has 4 parameters)
