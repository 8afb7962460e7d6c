#!/bin/bash
# Round-5 GPU session f: narrow sweeps of repacked ranges folded into the check / variable
# launches (device-selected): the timed-schedule and decoder tests, A/B of the converging points
# and of the headline against the previous build and the round-4 library, a 4.0 dB trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R04=qam-reconciliation_amd/qamr/exp/libqamr_r04.so
R05A=qam-reconciliation_amd/qamr/exp/libqamr_r05a.so
bash scripts/gpu_steps.sh \
  "t_sched|600|python -u -m pytest tests/test_gpu_timed_schedule.py tests/test_gpu_decoder.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "ab_4db|600|LIBS='$R04 $R05A default' ROUNDS=2 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_145|600|LIBS='$R04 $R05A default' ROUNDS=2 STEPS=10 BENCH_ARGS='--workload dvbs2_16pam --snr 14.5 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_head|600|LIBS='$R05A default' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh" \
  "trace_4db|300|QAMR_NO_CLOCK_PASS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05f_4db/trace -o run -- python3 bench.py --snr 4.0 --steps 2 --warmup 1 --cpu-seconds 0 --no-secondary"
