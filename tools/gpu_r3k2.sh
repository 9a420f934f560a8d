#!/bin/bash
# Masked magnitudes kept across the middle-out phases (FPLDPC_MAG_KEEP = 8 / 12 per side, A only), 4 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3k2}
mkdir -p "$OUT"
FPLDPC_LIB_PATH=build/ab/km12.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > "$OUT/parity_km12.log" 2>&1 \
&& timeout -k 10 900 python tools/ab.py "$OUT/ab" ${REPS:-4} 'A=--config A' 'A45=--ebn0 4.5' -- 'def=' 'head=FPLDPC_LIB_PATH=build/ab/head.so' \
  'km8=FPLDPC_LIB_PATH=build/ab/km8.so' 'km12=FPLDPC_LIB_PATH=build/ab/km12.so'
rc=$?
echo "exit $rc"; exit $rc
