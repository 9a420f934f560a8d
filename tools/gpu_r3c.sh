#!/bin/bash
# Same-box A/B: round-2 library, this round without / with the syndrome-first pass, and wave
# priority by attained iterations, on the 30-iteration and early-termination points.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3c}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
FPLDPC_PRIO_SHIFT=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_prio.log" 2>&1 || { echo "pytest (prio) failed"; tail -30 "$OUT/pytest_gpu_prio.log"; exit 1; }
tail -1 "$OUT/pytest_gpu_prio.log"
timeout -k 10 120 tools/ubench/f64_rate > "$OUT/f64_rate.txt" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sqf_A" -o run -- python3 bench.py --decoder float --steps 3 --warmup 1 --no-cpu > "$OUT/sqf_A.json" 2> "$OUT/sqf_A.err" || exit $?
timeout -k 10 1100 python tools/ab.py "$OUT/ab" 2 'A=--config A' 'A45=--ebn0 4.5' 'W=--config W' 'W2=--config W --ebn0 2.0' -- 'r2=FPLDPC_LIB_PATH=build/ab/r2.so' 'nopre=FPLDPC_LIB_PATH=build/ab/nopre.so' 'pre24=' 'p2=FPLDPC_PRIO_SHIFT=2' 'p3=FPLDPC_PRIO_SHIFT=3' 'p3off=FPLDPC_PRIO_SHIFT=3,FPLDPC_PRE_T=0'
