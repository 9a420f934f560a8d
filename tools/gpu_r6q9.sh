#!/bin/bash
# Round-6 call: the GPU suite with R's new wave roles, then A's balanced-progress priority A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q9}; mkdir -p $OUT
FPLDPC_ALLOW_STALE_PROFILE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit $rc
TAG=${TAG:-r6q9}/abA REPS=2 VARIANTS="base|build/ab/base.so| abal1|build/ab/abal1.so| abal2|build/ab/abal2.so|" CASES="A:--config A;A45:--config A --ebn0 4.5" bash tools/ab_env.sh > $OUT/abA.txt 2>&1 || { tail -5 $OUT/abA.txt; exit 1; }
tail -7 $OUT/abA.txt
timeout -k 10 300 python bench.py --config R > $OUT/bench_R.json 2> $OUT/bench_R.err || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('R', d['value'], d['ms_per_step'], d['parity_vs_cpu_oracle'])" $OUT/bench_R.json
echo exit 0
