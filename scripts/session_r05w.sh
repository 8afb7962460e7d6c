#!/bin/bash
# Round-5 GPU session w: re-tune of the two-stream knobs on the final build (headline): variable
# sweep pacing and the short-tail check grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L="default default@var_pace=24 default@var_pace=32 default@var_pace=40 default@check_tail=2 default@check_tail=8 default@var_boost=2"
bash scripts/gpu_steps.sh \
  "ab_knobs|900|LIBS='$L' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh"
