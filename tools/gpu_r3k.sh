#!/bin/bash
# R: the pipelined LDS-offset gather against the unpipelined one; and the N = 4 / 8 bench path
# rehearsed with gloo ranks sharing the box's GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3k}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 python tools/ab.py "$OUT/ab" 3 'R=--config R' -- 'pipe=' 'nopipe=FPLDPC_LIB_PATH=build/ab/r3k_nopipe.so' || exit $?
timeout -k 10 300 python bench.py --gpus 4 --backend gloo --steps 5 --warmup 2 > "$OUT/bench_g4.json" 2> "$OUT/bench_g4.err" || exit $?
timeout -k 10 300 python bench.py --gpus 8 --backend gloo --batch 2048 --steps 3 --warmup 1 > "$OUT/bench_g8.json" 2> "$OUT/bench_g8.err" || exit $?
cat "$OUT/bench_g4.json" "$OUT/bench_g8.json" | cut -c1-400
