#!/bin/bash
# Round-5 GPU session k: headline A/B of 579bc0a vs 3a5de12 (r05a) in alternating order, with the
# repack threshold and the repack switched off on each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
L="$E/libqamr_r05a.so $E/libqamr_579bc0a.so $E/libqamr_579bc0a.so@repack_pct=50 $E/libqamr_r05a.so@repack_pct=75 $E/libqamr_r05a.so@repack=0 $E/libqamr_579bc0a.so@repack=0"
bash scripts/gpu_steps.sh \
  "ab_k|900|LIBS='$L' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh"
