#!/bin/bash
# Round-5 evidence: kernel trace + PMC passes of the default bench (4-PAM headline) and of the
# 16-PAM workload (its demapper), kernel traces of configs[1] and of the 4-PAM 4.0 dB converging
# point; summaries -> gpurun_out/prof_r05*/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --cpu-seconds 0 --no-roofline --no-secondary"
TAG=${PTAG:-r05} TRACE_ARGS="--steps 3 --warmup 1 --cpu-seconds 0 --no-secondary" PMC_ARGS="$ARGS" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
bash scripts/profile_session.sh || exit 1
python3 scripts/summarize_profile.py gpurun_out/prof_${PTAG:-r05} --kernel 'k_check<7, 1, true>' --kernel-key check_d7 > /dev/null || exit 1
TAG=${PTAG:-r05}_16pam TRACE_ARGS="--workload dvbs2_16pam --steps 2 --warmup 1 --cpu-seconds 0 --no-secondary" \
PMC_ARGS="--workload dvbs2_16pam $ARGS" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
bash scripts/profile_session.sh || exit 1
python3 scripts/summarize_profile.py gpurun_out/prof_${PTAG:-r05}_16pam --kernel 'k_demap_wave<4>' --kernel-key demap \
    --workload dvbs2_16pam > /dev/null || exit 1
TAG=${PTAG:-r05}_configs1 TRACE_ARGS="--workload reg1008_4pam --batch 1024 --steps 5 --warmup 1 --cpu-seconds 0 --no-secondary" \
SKIP_PMC=1 bash scripts/profile_session.sh || exit 1
TAG=${PTAG:-r05}_4db TRACE_ARGS="--snr 4.0 --steps 2 --warmup 1 --cpu-seconds 0 --no-secondary" \
SKIP_PMC=1 bash scripts/profile_session.sh || exit 1
echo done
