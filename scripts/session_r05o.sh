#!/bin/bash
# Round-5 GPU session o: does code placement move the headline?  The current build with 0 / 3.5 /
# 7 / 10.5 / 14 KB of never-launched code in front of the decoder kernels, against 579bc0a and r04.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
L="$E/libqamr_579bc0a.so default $E/libqamr_pad128.so $E/libqamr_pad256.so $E/libqamr_pad384.so $E/libqamr_pad512.so $E/libqamr_nar0.so@repack=0 $E/libqamr_r05a.so@repack=0"
bash scripts/gpu_steps.sh \
  "ab_pad|900|LIBS='$L' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh"
