#!/bin/bash
# SQ counters of the dominant check kernel for several library builds (one rocprofv3
# --pmc pass per counter group and build; decode_once.py = one short batched decode).
#   LIBS="a.so b.so" [KERNEL='k_check<7, 1, true>'] bash scripts/pmc_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
K=${KERNEL:-"k_check<7, 1, true>"}
G1=${G1:-"SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"}
G2=${G2:-"SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU"}
G3=${G3:-"SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU SQ_CYCLES SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"}
n=0; mkdir -p gpurun_out/pmcab
for L in ${LIBS}; do
  n=$((n+1)); g=0
  for grp in "$G1" "$G2" "$G3"; do
    g=$((g+1)); d=gpurun_out/pmcab/l${n}_g${g}
    QAMR_LIB=$L timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $d -o run -- python3 scripts/decode_once.py --iters ${ITERS:-5} > $d.log 2>&1 || { echo "FAIL $L $g"; tail -5 $d.log; exit 1; }
  done
  K="$K" N=$n L=$L python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/pmcab/l{os.environ['N']}_g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void qr::" + os.environ["K"]):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(os.environ["L"], {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(agg.items())})
PY
done
