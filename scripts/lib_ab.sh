#!/bin/bash
# A/B of library builds on the default bench (no secondary configs), interleaved:
#   LIBS="qam-reconciliation_amd/qamr/exp/libqamr_r03.so default" ROUNDS=2 bash scripts/lib_ab.sh
# a LIBS entry lib.so@k=v,k=v runs that library with QAMR_TUNE=k=v,k=v
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for L in ${LIBS}; do
    LIB=${L%%@*}; TUNE=""; [[ $L == *@* ]] && TUNE=${L#*@}
    [ "$LIB" = default ] && LIB=""
    QAMR_LIB=$LIB QAMR_TUNE=$TUNE timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --cpu-seconds 0 --no-secondary ${BENCH_ARGS:-} > gpurun_out/lib_ab_run.json 2>&1 || { tail -5 gpurun_out/lib_ab_run.json; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/lib_ab_run.json').read().strip().splitlines()[-1]);r=d.get('roofline') or {};v=r.get('valu') or {};print('round $r', '$L', d['value'], d['ms_per_step'], r.get('avg_launch_us'), v.get('clock_ghz'), v.get('frac'), flush=True)"
  done
done
