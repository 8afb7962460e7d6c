SKIP_TRACE=1 TAG=fusedpmc PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" BENCH=scripts/decode_once.py PMC_ARGS="--iters 5" bash scripts/profile_session.sh > /dev/null 2>&1 || exit 1
python3 - <<PY
import csv,glob,collections
agg=collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/prof_fusedpmc/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void qr::k_fused_eps<7, 1"):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c,v in agg.items(): print(c, "%.4g" % (sum(v)/len(v)), len(v))
PY
