#!/bin/bash
# Round-5 GPU session q: the candidate final build (repack kernel at 32 VGPRs, variable sweep at 16):
# the whole GPU suite, then same-box A/B against the round-4 library and 579bc0a at the headline,
# the converging points and configs[1].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "t_all|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "ab_head|900|LIBS='$E/libqamr_r04.so $E/libqamr_579bc0a.so default' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh" \
  "ab_4db|900|LIBS='$E/libqamr_r04.so default' ROUNDS=2 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_145|900|LIBS='$E/libqamr_r04.so default' ROUNDS=2 STEPS=10 BENCH_ARGS='--workload dvbs2_16pam --snr 14.5 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_c1|900|LIBS='$E/libqamr_r04.so $E/libqamr_r05a.so default' ROUNDS=2 STEPS=300 BENCH_ARGS='--workload reg1008_4pam --batch 1024 --no-roofline' bash scripts/lib_ab.sh"
