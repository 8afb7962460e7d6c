#!/bin/bash
# Round-5 GPU session ab: the repack commit folded into the row-move kernel (its last workgroup):
# the timed-schedule and parity tests, then A/B against the previous build (r05d) at the
# converging points and the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "t_sched|600|python -u -m pytest tests/test_gpu_timed_schedule.py tests/test_gpu_decoder.py tests/test_gpu_properties.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "ab_4db|600|LIBS='$E/libqamr_r05d.so default' ROUNDS=3 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_145|600|LIBS='$E/libqamr_r05d.so default' ROUNDS=3 STEPS=10 BENCH_ARGS='--workload dvbs2_16pam --snr 14.5 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_head|600|LIBS='$E/libqamr_r05d.so default' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh"
