#!/bin/bash
# SQ counters of the two-lanes-per-check kernel against the default (A, 30 iterations).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sqsplit}
mkdir -p "$OUT"
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$OUT/def" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/def.json" 2> "$OUT/def.err" \
&& FPLDPC_KERNEL=flood_split timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$OUT/split" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/split.json" 2> "$OUT/split.err"
rc=$?; echo "exit $rc"; exit $rc
