#!/bin/bash
# W: 4 vs 5 workgroups per CU with and without the opaque loop starts; R layouts; ET traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3h}
mkdir -p "$OUT"
timeout -k 10 300 python tools/et_order.py --config A --ebn0 4.5 --trace "$OUT/trace" > "$OUT/et_order_A.txt" 2>&1 || exit $?
timeout -k 10 300 python tools/et_order.py --config W --ebn0 2.0 --trace "$OUT/trace" > "$OUT/et_order_W.txt" 2>&1 || exit $?
for f in "$OUT"/trace/*.bin; do echo "== $f"; python tools/wg_trace.py "$f"; done > "$OUT/traces.txt" 2>&1
cat "$OUT/traces.txt"
timeout -k 10 900 python tools/ab.py "$OUT/ab" 2 'W=--config W' 'W2=--config W --ebn0 2.0' -- 'new=' 'r2=FPLDPC_LIB_PATH=build/ab/r2.so' 'g4=FPLDPC_GRID_PER_CU=4' && timeout -k 10 600 python tools/ab.py "$OUT/abr" 2 'R=--config R' -- 'new=' 'r2=FPLDPC_LIB_PATH=build/ab/r2.so' 'walk=FPLDPC_KERNEL=flood_array2<P=47,CPL=2>'
