#!/bin/bash
# Wave-priority experiment (build/ab/prio.so, FPLDPC_PRIO 0/1/2) on the 30-iteration and
# early-termination points, against the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3j}
mkdir -p "$OUT"
FPLDPC_LIB_PATH=build/ab/prio.so FPLDPC_PRIO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 1000 python tools/ab.py "$OUT/ab" 2 'A=--config A' 'A45=--ebn0 4.5' 'W=--config W' 'W2=--config W --ebn0 2.0' 'R=--config R' -- 'def=' 'p0=FPLDPC_LIB_PATH=build/ab/prio.so' 'lrpt=FPLDPC_LIB_PATH=build/ab/prio.so|FPLDPC_PRIO=1' 'att=FPLDPC_LIB_PATH=build/ab/prio.so|FPLDPC_PRIO=2'
