#!/bin/bash
# Round-5 GPU session u: where the 16-PAM demapper's time goes: diagnostic builds without the root
# search (dsplit1) and without the LLR sums (dsplit2), timing only (their LAPPRs are wrong).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
E=qam-reconciliation_amd/qamr/exp
bash scripts/gpu_steps.sh \
  "dsplit|600|for L in default $E/libqamr_dsplit1.so $E/libqamr_dsplit2.so; do if [ \$L = default ]; then python scripts/demap_ab.py --variants 1 --reps 3 --cases 4:14.5,2:3.0 || exit 3; else QAMR_LIB=\$L python scripts/demap_ab.py --variants 1 --reps 3 --cases 4:14.5,2:3.0 || exit 3; fi; done"
