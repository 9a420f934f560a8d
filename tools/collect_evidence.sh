#!/bin/bash
# Copy an evidence pass (tools/gpu_round.sh, merged back under gpurun_out/<TAG>) into the tracked
# profiles/<ROUND>/final/ layout: bench lines, rocprofv3 kernel stats, PMC passes, test and smoke
# logs, and the counter summary bound to the kernel build id.  usage: tools/collect_evidence.sh TAG [ROUND]
set -e
cd "$(dirname "$0")/.."
TAG=$1; ROUND=${2:-r4}
SRC=gpurun_out/$TAG; DST=profiles/$ROUND/final
mkdir -p "$DST"
for f in "$SRC"/bench_*.json "$SRC/pytest_gpu.log" "$SRC/smoke.log"; do [ -f "$f" ] && cp "$f" "$DST/"; done
for d in "$SRC"/prof_*/; do
  k=$(basename "$d"); k=${k#prof_}
  cp "$d/run_kernel_stats.csv" "$DST/${k}_kernel_stats.csv"
  mkdir -p "$DST/pmc_$k"
  for p in fetch write sq; do [ -f "$SRC/${p}_$k/run_counter_collection.csv" ] && cp "$SRC/${p}_$k/run_counter_collection.csv" "$DST/pmc_$k/$p.csv"; done
done
[ -f "$SRC/pmc_traffic.json" ] && cp "$SRC/pmc_traffic.json" "profiles/$ROUND/pmc_traffic.json"
echo "collected $SRC -> $DST"
