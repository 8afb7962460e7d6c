#!/bin/bash
# One rocprofv3 PMC pass over a command, summarised per kernel (median over dispatches):
#   NAME=x GROUP="SQ_... SQ_..." FILTER=k_check bash scripts/pmc_kernel.sh python3 bench.py ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${NAME:-x}
mkdir -p $OUT
timeout -s KILL ${SECS:-300} rocprofv3 --pmc $GROUP --output-format csv -d $OUT -o run -- "$@" > $OUT/run.log 2>&1 || { echo "rocprofv3 failed rc=$?"; tail -5 $OUT/run.log; exit 1; }
python3 - "$OUT" "${FILTER:-k_}" <<'PY'
import csv, glob, collections, json, sys
out, flt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if flt in r['Kernel_Name']:
            agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
res = {k: {c: sorted(v)[len(v) // 2] for c, v in d.items()} for k, d in agg.items()}
res_n = {k: len(next(iter(d.values()))) for k, d in agg.items()}
json.dump({"median_per_dispatch": res, "dispatches": res_n}, open(out + '/summary.json', 'w'), indent=1)
for k, d in res.items():
    print(k, res_n[k], {c: f"{v:.4g}" for c, v in sorted(d.items())})
PY
