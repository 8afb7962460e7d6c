#!/bin/bash
# FETCH_SIZE of the fused sweep for several (library, tune) variants:
#   VARIANTS="lib.so|k=v,k=v;lib2.so|..." bash scripts/pmc_fused.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_fused; mkdir -p $OUT
IFS=';' read -r -a VS <<< "$VARIANTS"
i=0
for v in "${VS[@]}"; do
  i=$((i+1)); L=${v%%|*}; T=${v#*|}
  QAMR_LIB=$L QAMR_TUNE=$T timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/v$i -o run -- python3 scripts/decode_once.py > $OUT/v$i.log 2>&1 || { echo "STOP $v"; tail -5 $OUT/v$i.log; exit 1; }
  python3 - "$OUT/v$i" "$v" <<'PY'
import csv, glob, sys
d, v = sys.argv[1], sys.argv[2]
f = [float(r["Counter_Value"]) for p in glob.glob(d + "/**/run_counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(p)) if r["Kernel_Name"].startswith("void qr::k_fused<7, 1, true, 0")]
print(v, "fused launches", len(f), "FETCH GB/launch (x2)", round(2 * sum(f) / len(f) * 1024 / 1e9, 3) if f else None)
PY
done
