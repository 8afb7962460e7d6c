#!/bin/bash
# Round-5 GPU session t: the demapper's exp table replicated 8x (bank slots per copy): the demap
# tests on that build, demap-only timing against the final build, and the 16-PAM workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "t_demap|600|QAMR_LIB=$E/libqamr_dm8.so python -u -m pytest tests/test_gpu_demap.py tests/test_gpu_parity_edges.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "dm_ab|600|for r in 1 2; do QAMR_LIB=$E/libqamr_dm8.so python scripts/demap_ab.py --variants 1 --reps 3 && python scripts/demap_ab.py --variants 1 --reps 3 || exit 3; done" \
  "ab_16|600|LIBS='default $E/libqamr_dm8.so' ROUNDS=2 STEPS=4 BENCH_ARGS='--workload dvbs2_16pam --no-roofline' bash scripts/lib_ab.sh" \
  "ab_145|600|LIBS='default $E/libqamr_dm8.so' ROUNDS=2 STEPS=10 BENCH_ARGS='--workload dvbs2_16pam --snr 14.5 --no-roofline' bash scripts/lib_ab.sh"
