#!/bin/bash
# Kernel trace of one converging operating point (configs[2] code at 4.0 dB by default):
#   WORKLOAD=dvbs2_4pam SNR=4.0 bash scripts/prof_op.sh  -> gpurun_out/prof_op_<workload>_<snr>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${WORKLOAD:-dvbs2_4pam}; S=${SNR:-4.0}
OUT=gpurun_out/prof_op_${W}_${S}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 scripts/knob_ab.py --workload "$W" --snr "$S" --steps 1 --rounds 1 --knobs "split=3" > "$OUT/log.txt" 2>&1
