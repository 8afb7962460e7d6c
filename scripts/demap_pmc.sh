#!/bin/bash
# PMC passes over both demap kernels (k_demap_hyp and k_demap, via scripts/demap_ab.py,
# which runs demap_hyp = 1 then 0 on the same batch), one rocprofv3 run per group.
#   CASES=4:13.0 bash scripts/demap_pmc.sh  ->  gpurun_out/dpmc/summary.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/dpmc
mkdir -p $OUT
CASES=${CASES:-4:13.0}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "[$(date +%T)] pmc$i: $grp"
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 scripts/demap_ab.py --cases $CASES --reps 1 > $OUT/p$i.log 2>&1 || { echo "pmc$i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/dpmc/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_demap' in r['Kernel_Name']:
            agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
out = {k: {c: sorted(v) for c, v in d.items()} for k, d in agg.items()}
json.dump(out, open('gpurun_out/dpmc/summary.json', 'w'), indent=1)
for k, d in out.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {v}")
PY
