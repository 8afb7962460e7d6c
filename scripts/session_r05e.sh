#!/bin/bash
# Round-5 GPU session e: repack kernel v3 (no posterior moves, short rows grouped): the
# timed-schedule tests, A/B of the converging points against the round-4 library, a 4.0 dB trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R04=qam-reconciliation_amd/qamr/exp/libqamr_r04.so
bash scripts/gpu_steps.sh \
  "t_sched|600|python -u -m pytest tests/test_gpu_timed_schedule.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "ab_4db|600|LIBS='$R04 default default@repack_pct=35' ROUNDS=2 STEPS=10 BENCH_ARGS='--snr 4.0 --no-roofline' bash scripts/lib_ab.sh" \
  "ab_145|600|LIBS='$R04 default default@repack_pct=35' ROUNDS=2 STEPS=10 BENCH_ARGS='--workload dvbs2_16pam --snr 14.5 --no-roofline' bash scripts/lib_ab.sh" \
  "trace_4db|300|QAMR_NO_CLOCK_PASS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05e_4db/trace -o run -- python3 bench.py --snr 4.0 --steps 2 --warmup 1 --cpu-seconds 0 --no-secondary"
