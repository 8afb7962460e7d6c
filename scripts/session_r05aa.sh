#!/bin/bash
# Round-5 GPU session aa: the variable sweep at 32 allocated VGPRs (one wave per SIMD beside the
# check waves) against the final build's 16 (two).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "ab_var32|600|LIBS='default $E/libqamr_var32.so' ROUNDS=3 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh"
