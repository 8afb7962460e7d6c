#!/bin/bash
# Round-5 GPU session i: what the repack decision launches cost the dense iterations: headline and
# 4.0 dB A/B of the round-4 library, the current build with and without repack, and a diagnostic
# build with two empty launches per variable sweep (repack off); decoder tests of the current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "t_dec|600|python -u -m pytest tests/test_gpu_timed_schedule.py tests/test_gpu_decoder.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "ab_head|600|LIBS='$E/libqamr_r04.so default default@repack=0 $E/libqamr_nop2.so@repack=0' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh" \
  "ab_4db|600|LIBS='$E/libqamr_r04.so default default@repack=0 $E/libqamr_nop2.so@repack=0' ROUNDS=2 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh"
