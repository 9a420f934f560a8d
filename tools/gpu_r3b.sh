#!/bin/bash
# Syndrome-first pass: parity suite, then A/B of the threshold on the 30-iteration and
# early-termination points.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_compat.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 1000 python tools/ab.py "$OUT/ab" 2 'A=--config A' 'A45=--ebn0 4.5' 'W=--config W' 'W2=--config W --ebn0 2.0' 'R=--config R' -- 'off=FPLDPC_PRE_T=0' 't8=FPLDPC_PRE_T=8' 't24=FPLDPC_PRE_T=24' 't64=FPLDPC_PRE_T=64'
