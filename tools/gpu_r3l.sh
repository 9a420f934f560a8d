#!/bin/bash
# BER from the hard-decision ballots + per-workgroup totals: parity (incl. both BER paths), then A/B
# against the previous build on the bench's full-output step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3l}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_compat.py tests/test_gpu_perftest.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 900 python tools/ab.py "$OUT/ab" 3 'A=--config A' 'W=--config W' 'R=--config R' 'A45=--ebn0 4.5' -- 'new=' 'prev=FPLDPC_LIB_PATH=build/ab/prev.so'
