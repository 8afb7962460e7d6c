#!/bin/bash
# Copy the summaries of a scripts/profile_session.sh output directory into profiles/ (tracked):
#   bash scripts/keep_profile.sh gpurun_out/prof_TAG profiles/r06/NAME
# kernel trace stats (+ the per-dispatch trace when KEEP_TRACE=1), the per-pass PMC counters,
# summary.md / pmc_traffic.json of scripts/summarize_profile.py.
set -eu
src=$1; dst=$2
mkdir -p "$dst"
[ -f "$src/trace/run_kernel_stats.csv" ] && cp "$src/trace/run_kernel_stats.csv" "$dst/kernel_stats.csv"
[ "${KEEP_TRACE:-0}" = 1 ] && [ -f "$src/trace/run_kernel_trace.csv" ] && cp "$src/trace/run_kernel_trace.csv" "$dst/kernel_trace.csv"
for d in "$src"/pmc*/; do
  [ -f "$d/run_counter_collection.csv" ] && cp "$d/run_counter_collection.csv" "$dst/$(basename "$d")_counters.csv"
done
for f in summary.md pmc_traffic.json; do [ -f "$src/$f" ] && cp "$src/$f" "$dst/$f"; done
ls "$dst"
