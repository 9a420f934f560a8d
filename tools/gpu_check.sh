#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit; steps chain with && so the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-check}
mkdir -p "$OUT"
rocm-smi --showproductname > "$OUT/smi.txt" 2>&1 || true
nproc > "$OUT/nproc.txt"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& timeout -k 10 300 python bench.py --config W --no-cpu > "$OUT/bench_W.json" 2> "$OUT/bench_W.err" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?
echo "exit $rc"
exit $rc
