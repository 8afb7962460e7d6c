#!/bin/bash
# Round-5 first GPU session: the timed-schedule tests (device-steered repack), the full GPU
# suite, smoke, the driver's bench command, and A/Bs of the frame-resident decode's variable
# phase and of the demapper's exp (previous builds in qamr/exp/).  One gpu_steps.sh call: a
# crash, abort or timeout of any step ends the session there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OLD=qam-reconciliation_amd/qamr/exp/libqamr_resold.so
DOLD=qam-reconciliation_amd/qamr/exp/libqamr_demapold.so
exec_steps() { bash scripts/gpu_steps.sh "$@"; }
exec_steps \
  "t_sched|600|python -u -m pytest tests/test_gpu_timed_schedule.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "t_all|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke|300|python __graft_entry__.py smoke" \
  "bench|600|python bench.py --gpus 1 --steps 20 --warmup 5" \
  "res_ab|300|for r in 1 2; do QAMR_LIB=$OLD python scripts/small_ab.py --knobs resident=1 --reps 50 && python scripts/small_ab.py --knobs resident=1 --reps 50 || exit 3; done" \
  "demap_ab|400|for r in 1 2; do QAMR_LIB=$DOLD python scripts/demap_ab.py --variants 1 --reps 3 && python scripts/demap_ab.py --variants 1 --reps 3 || exit 3; done"
