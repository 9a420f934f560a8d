#!/bin/bash
# Round-6 call: R's wave-role permutations / wave priorities (tools/build_r_variants.py builds) A/B
# against the in-tree build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q6}; mkdir -p $OUT
TAG=${TAG:-r6q6}/abR REPS=${REPS:-2} VARIANTS="${RVARIANTS:-base||}" CASES="R:--config R" bash tools/ab_env.sh > $OUT/abR.txt 2>&1 || { tail -5 $OUT/abR.txt; exit 1; }
tail -8 $OUT/abR.txt

if [ -n "$WAITLIB" ]; then
  FPLDPC_WG_TRACE=$OUT/wait_R.bin FPLDPC_LIB_PATH=$WAITLIB timeout -k 10 300 python bench.py --config R --steps 2 --warmup 2 --no-cpu > $OUT/wait_R.json 2>&1 || exit 1
  python tools/wait_trace.py $OUT/wait_R.bin.waves --json $OUT/wait_R.summary.json > $OUT/wait_R.txt; cat $OUT/wait_R.txt
fi
echo exit 0
