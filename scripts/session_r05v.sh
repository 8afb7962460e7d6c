#!/bin/bash
# Round-5 GPU session v: counters of the check launch beside a 24-VGPR repack kernel (nar0, the
# build before the register fix, narrow sweeps compiled out) and beside the 32-VGPR one (final
# build): waves, wave-cycles, VALU issue, per launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp QAMR_NO_CLOCK_PASS=1
E=qam-reconciliation_amd/qamr/exp
P="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
A="--steps 2 --warmup 1 --cpu-seconds 0 --no-roofline --no-secondary"
bash scripts/gpu_steps.sh \
  "pmc_v24|300|QAMR_LIB=$E/libqamr_nar0.so rocprofv3 --pmc $P --output-format csv -d gpurun_out/prof_r05v/v24 -o run -- python3 bench.py $A" \
  "pmc_v32|300|rocprofv3 --pmc $P --output-format csv -d gpurun_out/prof_r05v/v32 -o run -- python3 bench.py $A" \
  "tr_v24|300|QAMR_LIB=$E/libqamr_nar0.so rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r05v/tv24 -o run -- python3 bench.py $A" \
  "tr_v32|300|rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r05v/tv32 -o run -- python3 bench.py $A"
