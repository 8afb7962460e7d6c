#!/bin/bash
# A/B the decode step over library variants: LIBS="a.so b.so" [TUNES="k=v,..;..."] bash scripts/exp_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LIBS:-""}; do
  IFS=';' read -r -a TS <<< "${TUNES:-}"
  [ ${#TS[@]} -eq 0 ] && TS=("")
  for T in "${TS[@]}"; do
    QAMR_LIB=$L QAMR_TUNE=$T timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/exp.log 2>&1 || { tail -5 gpurun_out/exp.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/exp.log').read().strip().splitlines()[-1]);print('${L:-default}', '$T', d['value'], (d.get('roofline') or {}).get('avg_launch_us'), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
  done
done
