#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel for several kernel-geometry presets.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sweep; mkdir -p $OUT
i=0
for cfg in ${CFGS:-"split=1,nt=1,check_ft=256" "split=1,nt=1,check_ft=64" "split=1,nt=0,check_ft=64" "split=2,nt=1,check_ft=256" "split=2,nt=1,check_ft=64"}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    echo "[$(date +%T)] $cfg $ctr"
    QAMR_TUNE=$cfg timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/c$i -o run -- python3 scripts/decode_once.py > $OUT/c$i.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; tail -5 $OUT/c$i.log; exit $rc; fi
    echo "$cfg $ctr" > $OUT/c$i/cfg.txt
  done
done
