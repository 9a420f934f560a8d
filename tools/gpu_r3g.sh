#!/bin/bash
# Loop bounds made opaque (A 163 -> 142 VGPRs, W 109 -> 96, R walked offsets spill-free): parity,
# then A/B against round 2 on every config, W at 4 vs 5 workgroups per CU, R layouts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3g}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 1000 python tools/ab.py "$OUT/ab" 2 'A=--config A' 'W=--config W' 'R=--config R' 'A45=--ebn0 4.5' 'W2=--config W --ebn0 2.0' -- 'new=' 'r2=FPLDPC_LIB_PATH=build/ab/r2.so' 'g4=FPLDPC_GRID_PER_CU=4' 'walk=FPLDPC_KERNEL=flood_array2<P=47,CPL=2>'
timeout -k 10 300 python tools/et_order.py --config A --ebn0 4.5 > "$OUT/et_order_A.txt" 2>&1 || exit $?
timeout -k 10 300 python tools/et_order.py --config W --ebn0 2.0 > "$OUT/et_order_W.txt" 2>&1 || exit $?
cat "$OUT/et_order_A.txt" "$OUT/et_order_W.txt" | grep -v "^{"
