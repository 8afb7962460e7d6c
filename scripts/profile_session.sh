#!/bin/bash
# rocprofv3 session: kernel-trace + stats of the default bench command, then
# one PMC pass per counter group (separate runs, as MI355X_MICROARCH.md says).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export QAMR_NO_CLOCK_PASS=1  # bench.py: no child clock pass under the profiler
OUT=gpurun_out/prof_${TAG:-r1}
mkdir -p "$OUT"
BENCH=${BENCH:-"bench.py"}
PMC_ARGS=${PMC_ARGS:-"--steps 1 --warmup 0 --cpu-seconds 0 --no-roofline"}
step() {  # step <name> <secs> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] >>> $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] <<< $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
if [[ ${SKIP_TRACE:-0} != 1 ]]; then
step trace 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH ${TRACE_ARGS:-}
fi
[[ ${SKIP_PMC:-0} == 1 ]] && exit 0
if [ -n "${PMC_GROUPS:-}" ]; then IFS=';' read -r -a GRPS <<< "$PMC_GROUPS"; else
GRPS=("FETCH_SIZE" "WRITE_SIZE"
      "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
      "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU"); fi
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  step pmc$i 900 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- python3 $BENCH $PMC_ARGS
done
exit 0
