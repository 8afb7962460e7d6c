#!/bin/bash
# Round-5 GPU session c: the timed-schedule tests, then same-box A/Bs of the converging operating
# points (4-PAM 4.0 dB, 16-PAM 14.5 dB): the round-4 library (host-decided repack), this build
# (device-decided repack), this build without the repack; then the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R04=qam-reconciliation_amd/qamr/exp/libqamr_r04.so
bash scripts/gpu_steps.sh \
  "t_sched|600|python -u -m pytest tests/test_gpu_timed_schedule.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "ab_xcd|600|LIBS='default default@xcd_remap=1' ROUNDS=3 STEPS=10 bash scripts/lib_ab.sh" \
  "ab_4db|600|LIBS='$R04 default default@repack=0' ROUNDS=2 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_145|600|LIBS='$R04 default default@repack=0' ROUNDS=2 STEPS=10 BENCH_ARGS='--workload dvbs2_16pam --snr 14.5 --no-roofline' bash scripts/lib_ab.sh" \
  "bench|600|python bench.py --gpus 1 --steps 20 --warmup 5"
