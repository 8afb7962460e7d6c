#!/bin/bash
# Round-5 GPU session j: headline A/B bisection of the round-5 commits against the round-4 library
# (same box, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
L="$E/libqamr_r04.so $E/libqamr_79801bc.so $E/libqamr_c615674.so $E/libqamr_6c7fc31.so $E/libqamr_567e613.so $E/libqamr_579bc0a.so $E/libqamr_r05a.so default"
bash scripts/gpu_steps.sh \
  "ab_bisect|900|LIBS='$L' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh"
