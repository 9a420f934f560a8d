#!/bin/bash
# GPU quick pass (tests + smoke + bench lines for CFGS), then for each config in PROF: the SQ issue
# counters, FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes, and kernel stats.
# Output: gpurun_out/$TAG (tools/pmc_summary.py reads fetch_/write_/sq_ dirs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cfgprof}
mkdir -p "$OUT"
TAG=${TAG:-cfgprof} CFGS="${CFGS:-A}" bash tools/gpu_quick.sh || exit $?
for cfg in ${PROF:-A}; do
  b="python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu"
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq_$cfg" -o run -- $b > "$OUT/sq_$cfg.json" 2> "$OUT/sq_$cfg.err" \
  && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$cfg" -o run -- $b > "$OUT/fetch_$cfg.json" 2> "$OUT/fetch_$cfg.err" \
  && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$cfg" -o run -- $b > "$OUT/write_$cfg.json" 2> "$OUT/write_$cfg.err" \
  || exit $?
done
TAG=${TAG:-cfgprof} CFGS="${PROF:-A}" bash tools/gpu_stats.sh
