#!/bin/bash
# configs[1] (reg-(3,6) N=1008, B = 1024) under the frame-resident decode: kernel trace + PMC
# passes of k_resident<6> (VALU issue, waits, LDS); summary -> gpurun_out/prof_${PTAG:-r04}_resident/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS="--workload reg1008_4pam --batch 1024 --steps 5 --warmup 1 --cpu-seconds 0 --no-roofline --no-secondary"
TAG=${PTAG:-r04}_resident TRACE_ARGS="$ARGS" PMC_ARGS="$ARGS" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
bash scripts/profile_session.sh || exit 1
python3 scripts/summarize_profile.py gpurun_out/prof_${PTAG:-r04}_resident --kernel 'k_resident<6>' --kernel-key resident_d6 \
    --workload reg1008_4pam --batch 1024 > /dev/null || exit 1
echo done
