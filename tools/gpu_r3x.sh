#!/bin/bash
# Stored slot offsets as bytes (A: 140 -> 128 VGPRs, 4 workgroups per CU) vs 16-bit halves, 4 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3x}
mkdir -p "$OUT"
timeout -k 10 900 python tools/ab.py "$OUT/ab" 4 'A=--config A' 'A45=--ebn0 4.5' -- 'def=' \
  'byte=FPLDPC_LIB_PATH=build/ab/byte.so'
rc=$?
[ $rc -eq 0 ] && FPLDPC_LIB_PATH=build/ab/byte.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -x -q --timeout 200 --timeout-method thread > "$OUT/parity_byte.log" 2>&1
rc=$?
echo "exit $rc"; exit $rc
