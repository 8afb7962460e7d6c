#!/bin/bash
# Run GPU steps in order, each under its own time limit, logs in gpurun_out/<name>.log:
#   bash scripts/gpu_steps.sh "name|seconds|command" ...
# A plain test failure (rc 1) continues; a crash, abort, timeout or any other rc ends the
# session there (no retries: after a GPU fault nothing more runs in this call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "[$(date +%T)] >>> $name: $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] <<< $name rc=$rc"; tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
done
exit 0
