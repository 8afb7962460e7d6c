#!/bin/bash
# Round-5 GPU session y: frame-resident decode with its variables' LDS message indices in
# registers (regular variable degree <= 3): the resident tests on both variants (check indices
# pinned: resA, not pinned: resB), then configs[1] A/B against the committed build (r05c).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
T="tests/test_gpu_parity_edges.py -k 'fused_iteration or resident_batch' tests/test_gpu_decoder.py"
bash scripts/gpu_steps.sh \
  "t_resA|600|QAMR_LIB=$E/libqamr_resA.so python -u -m pytest $T -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "t_resB|600|QAMR_LIB=$E/libqamr_resB.so python -u -m pytest $T -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "ab_c1|600|LIBS='$E/libqamr_r05c.so $E/libqamr_resA.so $E/libqamr_resB.so' ROUNDS=3 STEPS=300 BENCH_ARGS='--workload reg1008_4pam --batch 1024 --no-roofline' bash scripts/lib_ab.sh"
