# SQ/LDS counters of the fused sweep (decode_once.py), one rocprofv3 pass per group.
#   MATH=0|1|2 (decoder arithmetic knob) picks the k_fused<7, 1, true, MATH> instantiation.
M=${MATH:-0}
QAMR_TUNE="math=$M" SKIP_TRACE=1 TAG=fusedpmc$M PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" BENCH=scripts/decode_once.py PMC_ARGS="--iters 5" bash scripts/profile_session.sh > /dev/null 2>&1 || exit 1
M=$M python3 - <<'PY'
import csv,glob,collections,os
m=os.environ["M"]
agg=collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/prof_fusedpmc{m}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith(f"void qr::k_fused<7, 1, true, {m}"):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("math", m)
for c,v in agg.items(): print(c, "%.4g" % (sum(v)/len(v)), len(v))
PY
