#!/bin/bash
# W: opaque refill / store loop starts for the table policy (91 VGPRs: 5 workgroups / CU fit), with
# the grid at the occupancy query's 5 / CU or capped at 4, and built for 5 waves; A/B vs the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3p}
mkdir -p "$OUT"
timeout -k 10 900 python tools/ab.py "$OUT/ab" 3 'W=--config W' 'W2=--config W --ebn0 2.0' -- 'new=' \
  'op=FPLDPC_LIB_PATH=build/ab/tabop.so' 'op4=FPLDPC_LIB_PATH=build/ab/tabop.so|FPLDPC_GRID_PER_CU=4' \
  'op5=FPLDPC_LIB_PATH=build/ab/tabop5.so'
