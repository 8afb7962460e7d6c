#!/bin/bash
# Round-5 GPU session d: the device-decided repack's threshold (knob repack_pct) at the two
# converging operating points, same box, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "pct_4db|600|LIBS='default@repack_pct=75 default@repack_pct=50 default@repack_pct=35 default@repack_pct=25 default@repack_pct=15' ROUNDS=2 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh" \
  "pct_145|600|LIBS='default@repack_pct=75 default@repack_pct=50 default@repack_pct=35 default@repack_pct=25 default@repack_pct=15' ROUNDS=2 STEPS=10 BENCH_ARGS='--workload dvbs2_16pam --snr 14.5 --no-roofline' bash scripts/lib_ab.sh"
