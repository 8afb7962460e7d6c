#!/bin/bash
# Round-5 final bench session: smoke and the driver's bench command on the final build (the PMC
# row the bench prices with is profiles/pmc_traffic.json, from session r).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "smoke|300|python __graft_entry__.py smoke" \
  "bench_final|900|python bench.py --gpus 1 --steps 20 --warmup 5"
