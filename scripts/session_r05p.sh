#!/bin/bash
# Round-5 GPU session p: which change slows the dense iterations?  nar0 (no narrow sweeps) with the
# round-5 repack row-move kernel, with the 579bc0a one (n0v2), with it forced to 32 VGPRs (n0v32);
# the narrow sweeps with the repack off (check only, variable only, both), against 579bc0a.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
L="$E/libqamr_579bc0a.so $E/libqamr_nar0.so $E/libqamr_n0v2.so $E/libqamr_n0v32.so $E/libqamr_nar1.so@repack=0 $E/libqamr_nar2.so@repack=0 default@repack=0"
bash scripts/gpu_steps.sh \
  "ab_p|900|LIBS='$L' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh"
