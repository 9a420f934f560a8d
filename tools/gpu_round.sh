#!/bin/bash
# Full GPU pass for the committed evidence under profiles/<round>: parity tests, smoke, bench lines
# for every config (+ early-termination points and the float decoder), rocprofv3 kernel stats, and
# the FETCH_SIZE / WRITE_SIZE / SQ passes for tools/pmc_summary.py (the float decoder: FP64 issue
# counters).  Every GPU step has its own time limit and the steps chain with &&: the first failure
# ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}
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
  local sq="$SQ"; [[ $key == *_float ]] && sq="$SQF"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$key" -o run --output-format csv -- python3 bench.py "$@" --no-cpu > "$OUT/prof_$key.json" 2> "$OUT/prof_$key.err" \
  && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$key" -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu > "$OUT/fetch_$key.json" 2> "$OUT/fetch_$key.err" \
  && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$key" -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu > "$OUT/write_$key.json" 2> "$OUT/write_$key.err" \
  && timeout -s KILL 300 rocprofv3 --pmc $sq --kernel-trace --output-format csv -d "$OUT/sq_$key" -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu > "$OUT/sq_$key.json" 2> "$OUT/sq_$key.err"
}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& prof A --config A && prof W --config W && prof R --config R && prof A_float --config A --decoder float --steps 5 --warmup 2 \
&& python tools/pmc_summary.py "$OUT" profiles/${ROUND:-r3}/pmc_traffic.json > /dev/null && cp profiles/${ROUND:-r3}/pmc_traffic.json "$OUT/" \
&& b A --inflight-steps 50 && b W --config W --inflight-steps 50 && b R --config R --inflight-steps 50 \
&& b A_4.5dB --ebn0 4.5 --no-cpu --inflight-steps 50 && b W_2dB --config W --ebn0 2.0 --no-cpu --inflight-steps 50 \
&& b A_float --decoder float --steps 5 --warmup 2 && b W_float --config W --decoder float --steps 5 --warmup 2 \
&& b R_float --config R --decoder float --steps 2 --warmup 1 --no-cpu
rc=$?
echo "exit $rc"
exit $rc
