#!/bin/bash
# Quick GPU pass: the GPU parity suite (optional K=pytest -k expression), smoke, and bench lines for
# the configs in CFGS.  Every GPU step has its own time limit; steps chain with && (first failure ends).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p "$OUT"
lscpu > "$OUT/lscpu.txt" 2>&1 || true
run_tests() {
  [ -n "$NOTEST" ] && return 0
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${K:+-k "$K"} > "$OUT/pytest_gpu.log" 2>&1
  local rc=$?; tail -3 "$OUT/pytest_gpu.log"; return $rc
}
run_tests \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& for cfg in ${CFGS:-A}; do
     timeout -k 10 300 python bench.py --config $cfg ${BENCH_ARGS} > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || exit $?
     python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['kernel'], d['parity_vs_cpu_oracle'])" "$OUT/bench_$cfg.json" $cfg
   done
rc=$?
echo "exit $rc"
exit $rc
