#!/bin/bash
# Round-6 call: R's wave-role permutations / wave priorities (tools/build_r_variants.py builds) A/B
# against the in-tree build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q6}; mkdir -p $OUT
TAG=${TAG:-r6q6}/abR REPS=${REPS:-2} VARIANTS="${RVARIANTS:-base||}" CASES="R:--config R" bash tools/ab_env.sh > $OUT/abR.txt 2>&1 || { tail -5 $OUT/abR.txt; exit 1; }
tail -8 $OUT/abR.txt
echo exit 0
