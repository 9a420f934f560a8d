#!/bin/bash
# Round-6 call: the GPU suite on the build with W's split tail, smoke, bench lines, and R's wait
# attribution (FPLDPC_WAIT_TRACE stamps of every packed-loop barrier + SQ counters of the same build).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q5}; mkdir -p $OUT
FPLDPC_ALLOW_STALE_PROFILE=1 FPLDPC_PARAM_REPORT=$OUT/param_sweep.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
for w in "A --config A" "W --config W" "R --config R" "W_2dB --config W --ebn0 2.0" "A_4.5dB --config A --ebn0 4.5"; do
  set -- $w; name=$1; shift
  timeout -k 10 300 python bench.py "$@" --inflight-steps 30 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['kernel'].split()[0], d['parity_vs_cpu_oracle'], (d.get('two_in_flight') or {}).get('value'))" $OUT/bench_$name.json $name
done
SQ="SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
FPLDPC_WG_TRACE=$OUT/wait_R.bin FPLDPC_LIB_PATH=build/wait/libfpldpc.so timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $OUT/pmc_R_wait -o run -- python3 bench.py --config R --steps 3 --warmup 1 --no-cpu > $OUT/pmc_R_wait.json 2> $OUT/pmc_R_wait.err || exit 1
python tools/wait_trace.py $OUT/wait_R.bin.waves --json $OUT/wait_R.summary.json > $OUT/wait_R.txt; head -1 $OUT/wait_R.txt
echo exit 0
