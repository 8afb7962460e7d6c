#!/bin/bash
# Round-5 GPU session ac: the check sweep's geometry on the final build (checks per thread, frame
# tile), headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L="default default@check_per=12 default@check_per=20 default@check_per=24 default@check_ft=64 default@var_per=4 default@var_per=16"
bash scripts/gpu_steps.sh \
  "ab_geom|900|LIBS='$L' ROUNDS=2 STEPS=6 BENCH_ARGS='--no-roofline' bash scripts/lib_ab.sh"
