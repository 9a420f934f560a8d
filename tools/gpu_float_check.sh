#!/bin/bash
# Float decoder check: the float GPU tests, then tools/gpu_float_ab.sh over RUNS (bench + FETCH/WRITE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-float_check}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
TAG=${TAG:-float_check} bash tools/gpu_float_ab.sh
