#!/bin/bash
# Round-5 GPU session n: headline and 4.0 dB A/B of the narrow-sweep variants (nar0: none, nar1:
# check only, default: check + variable) against 579bc0a and the round-4 library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
L="$E/libqamr_r04.so $E/libqamr_579bc0a.so default $E/libqamr_nar0.so $E/libqamr_nar1.so"
bash scripts/gpu_steps.sh \
  "ab_head|900|LIBS='$L' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh" \
  "ab_4db|900|LIBS='$L' ROUNDS=2 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh"
