#!/bin/bash
# Round-5 GPU session z: the final build (frame-resident decode with register-held LAPPRs and
# message indices): the whole GPU suite, smoke, the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "t_all|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke|300|python __graft_entry__.py smoke" \
  "bench_final3|900|python bench.py --gpus 1 --steps 20 --warmup 5"
