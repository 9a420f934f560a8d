#!/bin/bash
# W: the degree-sorted table kernel (passes 0-2 fold 7 slots): parity (parity, KAT, compat, other
# codes), then an A/B against the HEAD build on the bench's full-output step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3o}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_compat.py tests/test_gpu_codes.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 900 python tools/ab.py "$OUT/ab" 3 'W=--config W' 'W2=--config W --ebn0 2.0' 'A=--config A' -- 'new=' 'head=FPLDPC_LIB_PATH=build/ab/head.so'
