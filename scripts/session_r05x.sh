#!/bin/bash
# Round-5 GPU session x: the whole GPU suite and the driver's bench command once more on the
# committed final tree (a second box for the bench record).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "t_all|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench_final2|900|python bench.py --gpus 1 --steps 20 --warmup 5"
