#!/bin/bash
# Round-5 final profile session: scripts/prof_r05.sh (PTAG=r05final) on the final build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PTAG=r05final bash scripts/prof_r05.sh
