#!/bin/bash
# Frames/s and fused-launch time vs batch size (row stride = batch * 8 B):
# BATCHES="3584 4096 4608" bash scripts/batch_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for B in ${BATCHES:-3584 4096 4608 5120 8192}; do
  timeout -k 10 300 python bench.py --batch $B --steps ${STEPS:-2} --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/sweep_$B.log 2>&1 || { tail -5 gpurun_out/sweep_$B.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sweep_$B.log').read().strip().splitlines()[-1]);r=d['roofline'];print('B=$B', d['value'], 'fused us', r['avg_launch_us'], 'us/frame', round(r['avg_launch_us']/($B/2),4), 'frac', r['frac'])"
done
