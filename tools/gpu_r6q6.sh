#!/bin/bash
# Round-6 call: R's wave-role permutations (FPLDPC_R_ROLES builds) A/B against the in-tree build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q6}; mkdir -p $OUT
TAG=$TAG/abR REPS=${REPS:-2} VARIANTS="base|| r012|build/ab/r012.so| r201|build/ab/r201.so| r120|build/ab/r120.so| r102|build/ab/r102.so| r021|build/ab/r021.so|" CASES="R:--config R" bash tools/ab_env.sh > $OUT/abR.txt 2>&1 || { tail -5 $OUT/abR.txt; exit 1; }
tail -8 $OUT/abR.txt
echo exit 0
