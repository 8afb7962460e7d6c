set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dprof
timeout -k 10 300 python scripts/demap_bench.py > gpurun_out/dprof/bench.log 2>&1 || exit $?
cat gpurun_out/dprof/bench.log
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS --output-format csv -d gpurun_out/dprof/pmc1 -o run -- python3 scripts/demap_bench.py > gpurun_out/dprof/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/dprof/pmc2 -o run -- python3 scripts/demap_bench.py > gpurun_out/dprof/pmc2.log 2>&1 || exit $?
python3 - <<'PY'
import csv,glob,collections
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/dprof/pmc*/run_counter_collection.csv')+glob.glob('gpurun_out/dprof/pmc*/*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'k_demap' in r['Kernel_Name']:
            agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in agg.items():
    print(k, {c: [f"{x:.4g}" for x in vals] for c,vals in v.items()})
PY
