#!/bin/bash
# Round-5 GPU session zz: kernel trace of configs[1] on the final build (k_resident with
# register-held message indices).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PTAG=r05final2 bash -c 'TAG=${PTAG}_configs1 TRACE_ARGS="--workload reg1008_4pam --batch 1024 --steps 5 --warmup 1 --cpu-seconds 0 --no-secondary" SKIP_PMC=1 bash scripts/profile_session.sh'
