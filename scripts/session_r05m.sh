#!/bin/bash
# Round-5 GPU session m: the current build against the same build with the 579bc0a repack row moves
# (k1v2): headline with and without repack, the converging points, and the timed-schedule tests
# on k1v2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "ab_head|900|LIBS='default $E/libqamr_k1v2.so default@repack=0 $E/libqamr_k1v2.so@repack=0' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh" \
  "ab_4db|600|LIBS='$E/libqamr_r04.so default $E/libqamr_k1v2.so' ROUNDS=2 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_145|600|LIBS='$E/libqamr_r04.so default $E/libqamr_k1v2.so' ROUNDS=2 STEPS=10 BENCH_ARGS='--workload dvbs2_16pam --snr 14.5 --no-roofline' bash scripts/lib_ab.sh" \
  "t_k1v2|600|QAMR_LIB=$E/libqamr_k1v2.so python -u -m pytest tests/test_gpu_timed_schedule.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
