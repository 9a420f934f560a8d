#!/bin/bash
# Round-3 first pass: the whole GPU suite (new: per-frame drop-in, PerfTest, bench self-launch,
# rank-failure injection), the counter list of this box, and one bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3a}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc $rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_A.json" 2> "$OUT/bench_A.err" || exit $?
echo "done"
