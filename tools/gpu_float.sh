#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r2_float
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_float.py tests/test_gpu_perftest.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for cfg in A W R; do
  timeout -k 10 300 python bench.py --config $cfg --decoder float --steps 5 --warmup 2 --no-cpu > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), d['parity_vs_cpu_oracle'])" $OUT/bench_$cfg.json $cfg
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_A -o run --output-format csv -- python3 bench.py --decoder float --steps 5 --warmup 2 --no-cpu > $OUT/prof_A.json 2> $OUT/prof_A.err \
&& timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch_A -o run -- python3 bench.py --decoder float --steps 2 --warmup 1 --no-cpu > $OUT/fetch_A.json 2> $OUT/fetch_A.err \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write_A -o run -- python3 bench.py --decoder float --steps 2 --warmup 1 --no-cpu > $OUT/write_A.json 2> $OUT/write_A.err
echo "exit $?"
