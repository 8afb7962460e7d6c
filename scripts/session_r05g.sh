#!/bin/bash
# Round-5 GPU session g: same-box kernel traces of the 4-PAM 4.0 dB decode with the round-4 library
# and the current build; configs[1] A/B of the frame-resident kernel variants (LAPPRs held in
# registers, check indices pinned or not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "trace_r04|300|QAMR_LIB=$E/libqamr_r04.so QAMR_NO_CLOCK_PASS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05g_r04/trace -o run -- python3 bench.py --snr 4.0 --steps 2 --warmup 1 --cpu-seconds 0 --no-secondary --no-roofline" \
  "trace_cur|300|QAMR_NO_CLOCK_PASS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05g_cur/trace -o run -- python3 bench.py --snr 4.0 --steps 2 --warmup 1 --cpu-seconds 0 --no-secondary --no-roofline" \
  "ab_res|600|LIBS='$E/libqamr_res_p1l0.so $E/libqamr_res_p1l1.so $E/libqamr_res_p0l1.so' ROUNDS=3 STEPS=300 BENCH_ARGS='--workload reg1008_4pam --batch 1024 --no-roofline' bash scripts/lib_ab.sh"
