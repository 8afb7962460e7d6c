# Round-1 strict-arithmetic evidence: kernel trace of the default bench command, then PMC passes.
TAG=strict2s PMC_ARGS="--steps 1 --warmup 0 --cpu-seconds 0 --no-roofline --no-alt" \
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
bash scripts/profile_session.sh && python3 scripts/summarize_profile.py gpurun_out/prof_strict2s --kernel 'k_check<7, 1, true, 0>' --kernel-key check_d7 > /dev/null && cat gpurun_out/prof_strict2s/summary.md gpurun_out/prof_strict2s/pmc_traffic.json && tail -1 gpurun_out/prof_strict2s/trace.log
