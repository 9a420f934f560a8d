#!/bin/bash
# Float decoder with log_1to2: parity (tests/test_gpu_float.py, -s for the measured agreement),
# the fixed-point parity suite on the default build, then the float bench lines (A/W/R, with the
# CPU baseline) and an A/B of the old (device libm) log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3d}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py -s -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_float.log" 2>&1 || { echo "float pytest failed"; tail -30 "$OUT/pytest_float.log"; exit 1; }
grep -E "differ|passed|failed" "$OUT/pytest_float.log"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_fixed.log" 2>&1 || { echo "fixed pytest failed"; tail -30 "$OUT/pytest_fixed.log"; exit 1; }
tail -1 "$OUT/pytest_fixed.log"
timeout -k 10 300 python bench.py --decoder float --steps 5 --warmup 2 > "$OUT/bench_A_float.json" 2> "$OUT/bench_A_float.err" || exit $?
timeout -k 10 600 python tools/ab.py "$OUT/ab" 2 'Af=--decoder float --steps 5 --warmup 2' 'Wf=--decoder float --config W --steps 5 --warmup 2' 'A=--config A' -- 'fast=' 'oldlog=FPLDPC_LIB_PATH=build/ab/oldlog.so' 'r2=FPLDPC_LIB_PATH=build/ab/r2.so'
