#!/bin/bash
# One GPU-box session: gpu tests, smoke, short bench.  Each GPU step has its own
# time limit; a crash/timeout/abort of any step ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>; continue on plain test failures (rc 1) only
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] >>> $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] <<< $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,smoke,bench}
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:--x} -p no:cacheprovider
[[ $STEPS == *smoke* ]] && run smoke 300 python __graft_entry__.py smoke
[[ $STEPS == *tune* ]] && run tune 900 python scripts/tune.py ${TUNE_ARGS:-}
[[ $STEPS == *demap* ]] && run demap_bench 600 python scripts/demap_bench.py
[[ $STEPS == *bench* ]] && run bench 900 python bench.py ${BENCH_ARGS:-}
exit 0
