#!/bin/bash
# Per-wave time split of the packed loop under the three FPLDPC_WAIT_TRACE stamp modes (1: other
# barriers, 2: the per-step LLR copy, 3: everything after the per-step barrier), per config.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-waitsplit}; mkdir -p $OUT
for c in ${CFGS:-A W}; do
  for m in 1 2 3; do
    FPLDPC_WG_TRACE=$OUT/wait_${c}_m$m.bin FPLDPC_LIB_PATH=build/wait/w$m.so timeout -k 10 120 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu > $OUT/wait_${c}_m$m.json 2> $OUT/wait_${c}_m$m.err || exit 1
    python tools/wait_trace.py $OUT/wait_${c}_m$m.bin.waves --json $OUT/wait_${c}_m$m.summary.json > $OUT/wait_${c}_m$m.txt || exit 1
    echo "$c mode $m: $(head -1 $OUT/wait_${c}_m$m.txt)"
  done
done
rm -f $OUT/*.bin $OUT/*.bin.waves
echo exit 0
