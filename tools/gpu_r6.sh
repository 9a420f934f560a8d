#!/bin/bash
# Round-6 measurement pass (one gpurun call): the GPU suite (+ the parameter-sweep report), smoke,
# bench lines, the per-frame drop-in latency (tools/frame_latency.py) and the early-termination tail
# traces of the FPLDPC_TAIL_TRACE build (tools/tail_trace.py).  STEPS selects a subset
# ("tests smoke bench frames tail").  Every GPU step has its own time limit; steps chain with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6}
STEPS=${STEPS:-tests smoke bench frames tail}
mkdir -p "$OUT"
has() { [[ " $STEPS " == *" $1 "* ]]; }
step_tests() {
  has tests || return 0
  FPLDPC_PARAM_REPORT="$OUT/param_sweep.jsonl" timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 \
    --timeout-method thread ${K:+-k "$K"} > "$OUT/pytest_gpu.log" 2>&1
  local rc=$?; tail -3 "$OUT/pytest_gpu.log"; return $rc
}
step_smoke() {
  has smoke || return 0
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
}
step_bench() {
  has bench || return 0
  for cfg in ${CFGS:-A W R}; do
    timeout -k 10 300 python bench.py --config $cfg ${BENCH_ARGS} > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || return $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['kernel'], d['parity_vs_cpu_oracle'])" "$OUT/bench_$cfg.json" $cfg
  done
}
step_frames() {
  has frames || return 0
  timeout -k 10 600 python tools/frame_latency.py ${FRAME_ARGS} > "$OUT/frame_latency.jsonl" 2> "$OUT/frame_latency.err"
  local rc=$?; cat "$OUT/frame_latency.jsonl"; return $rc
}
step_tail() {
  has tail || return 0
  for w in "A_4.5dB --ebn0 4.5" "W_2dB --config W --ebn0 2.0" "A_0dB"; do
    set -- $w; name=$1; shift
    FPLDPC_WG_TRACE="$OUT/tail_$name.bin" FPLDPC_LIB_PATH=build/tail/libfpldpc.so timeout -k 10 300 \
      python bench.py "$@" --steps 3 --warmup 3 --no-cpu > "$OUT/tail_$name.json" 2> "$OUT/tail_$name.err" || return $?
    python tools/tail_trace.py "$OUT/tail_$name.bin" --json "$OUT/tail_$name.summary.json" > "$OUT/tail_$name.txt" || return $?
    head -12 "$OUT/tail_$name.txt"
  done
}
step_tests && step_smoke && step_bench && step_frames && step_tail
rc=$?
echo "exit $rc"
exit $rc
