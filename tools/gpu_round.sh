#!/bin/bash
# Evidence pass for profiles/<round>: PHASE=prof -- rocprofv3 kernel stats and the FETCH_SIZE /
# WRITE_SIZE / SQ --pmc passes of every bench workload (tools/pmc_summary.py -> pmc_traffic.json,
# bound to the kernel build id); PHASE=bench -- the GPU parity suite, smoke and the bench lines
# (which read that summary for their roofline).  PHASE=all runs both.  Every GPU step has its own
# time limit and the steps chain with &&: the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}
ROUND=${ROUND:-r4}
PHASE=${PHASE:-all}
mkdir -p "$OUT"
rocm-smi --showproductname > "$OUT/smi.txt" 2>&1 || true
b() {  # b NAME ARGS... : one bench line
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
}
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
SQF="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
prof() {  # prof KEY ARGS... : kernel stats + FETCH / WRITE / SQ passes of one workload
  local key=$1; shift
  local sq="$SQ"; [[ $key == *_float* ]] && sq="$SQF"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$key" -o run --output-format csv -- python3 bench.py "$@" --no-cpu > "$OUT/prof_$key.json" 2> "$OUT/prof_$key.err" \
  && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$key" -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu > "$OUT/fetch_$key.json" 2> "$OUT/fetch_$key.err" \
  && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$key" -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu > "$OUT/write_$key.json" 2> "$OUT/write_$key.err" \
  && timeout -s KILL 300 rocprofv3 --pmc $sq --kernel-trace --output-format csv -d "$OUT/sq_$key" -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu > "$OUT/sq_$key.json" 2> "$OUT/sq_$key.err" \
  && echo "profiled $key"
}
has_key() { [ -z "$PROF_KEYS" ] || [[ " $PROF_KEYS " == *" $1 "* ]]; }
pk() { local key=$1; has_key $key || return 0; prof "$@"; }
run_prof() {  # PROF_KEYS="A W ..." profiles a subset (several calls into one TAG); NO_SUMMARY=1 leaves the summary to the caller
  pk A --config A && pk W --config W && pk R --config R \
  && pk A_4.5dB --config A --ebn0 4.5 && pk W_2dB --config W --ebn0 2.0 && pk A_b8192 --config A --batch 8192 \
  && pk A_float --config A --decoder float --steps 5 --warmup 2 && pk R_float --config R --decoder float --steps 2 --warmup 1 \
  && pk W_float --config W --decoder float --steps 5 --warmup 2 \
  && { [ -n "$NO_SUMMARY" ] || { python tools/pmc_summary.py "$OUT" profiles/$ROUND/pmc_traffic.json > /dev/null && cp profiles/$ROUND/pmc_traffic.json "$OUT/"; }; }
}
run_bench() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  && tail -1 "$OUT/pytest_gpu.log" \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  && b A --inflight-steps 50 && b W --config W --inflight-steps 50 && b R --config R --inflight-steps 50 \
  && b A_4.5dB --ebn0 4.5 --inflight-steps 50 && b W_2dB --config W --ebn0 2.0 --inflight-steps 50 \
  && b A_b8192 --batch 8192 --no-cpu \
  && b A_b8192_gloo2 --gpus 2 --backend gloo --batch 8192 --steps 5 --warmup 2 --cpu-frames 512 \
  && b R_gloo2 --gpus 2 --backend gloo --config R --steps 3 --warmup 1 --cpu-frames 64 \
  && b A_float --decoder float --steps 5 --warmup 2 && b W_float --config W --decoder float --steps 5 --warmup 2 \
  && b R_float --config R --decoder float --steps 2 --warmup 1
}
case $PHASE in
  prof) run_prof ;;
  bench) run_bench ;;
  *) run_prof && run_bench ;;
esac
rc=$?
echo "exit $rc"
exit $rc
