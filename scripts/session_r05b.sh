#!/bin/bash
# Round-5 GPU session b: tests (device-steered repack), smoke, the driver's bench command, and a
# same-box A/B of the headline: the round-4 library (qamr/exp/libqamr_r04.so, built from commit
# b3b3aa8), this build, this build without the repack.  One gpu_steps.sh chain: a crash, abort
# or timeout of any step ends the session there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R04=qam-reconciliation_amd/qamr/exp/libqamr_r04.so
bash scripts/gpu_steps.sh \
  "t_sched|600|python -u -m pytest tests/test_gpu_timed_schedule.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "t_all|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke|300|python __graft_entry__.py smoke" \
  "bench|600|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "res_ab|300|for r in 1 2; do for s in 0 1 2 3; do QAMR_TUNE=res_stagger=\$s python scripts/small_ab.py --knobs resident=1 --reps 50 || exit 3; done; done" \
  "ab_3db|700|LIBS='$R04 default default@repack=0' ROUNDS=2 STEPS=10 bash scripts/lib_ab.sh"
