#!/bin/bash
# Round-5 GPU session l: same-box headline kernel traces of 579bc0a and 3a5de12 (r05a).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "tr_579|300|QAMR_LIB=$E/libqamr_579bc0a.so QAMR_NO_CLOCK_PASS=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r05l_579/trace -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-secondary --no-roofline" \
  "tr_r05a|300|QAMR_LIB=$E/libqamr_r05a.so QAMR_NO_CLOCK_PASS=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r05l_r05a/trace -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-secondary --no-roofline"
