#!/bin/bash
# Full GPU pass for the committed evidence under profiles/<round>: parity tests, smoke, bench lines
# for every config (+ early-termination points and the float decoder), rocprofv3 kernel stats, and
# the FETCH_SIZE / WRITE_SIZE passes for tools/pmc_summary.py.  Every GPU step has its own time
# limit and the steps chain with &&: the first failure ends the call.
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
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& b A && b W --config W && b R --config R \
&& b A_4.5dB --ebn0 4.5 --no-cpu && b W_2dB --config W --ebn0 2.0 --no-cpu \
&& b A_float --decoder float --steps 5 --no-cpu \
&& for cfg in A W R; do
     timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu > "$OUT/prof_$cfg.json" 2> "$OUT/prof_$cfg.err" || exit $?
     timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$cfg" -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > "$OUT/fetch_$cfg.json" 2> "$OUT/fetch_$cfg.err" || exit $?
     timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$cfg" -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > "$OUT/write_$cfg.json" 2> "$OUT/write_$cfg.err" || exit $?
     timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq_$cfg" -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > "$OUT/sq_$cfg.json" 2> "$OUT/sq_$cfg.err" || exit $?
   done
rc=$?
echo "exit $rc"
exit $rc
