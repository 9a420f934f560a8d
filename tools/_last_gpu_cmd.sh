set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/final6; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && tail -1 $OUT/pytest_gpu.log \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -3 $OUT/smoke.log \
&& timeout -k 10 300 python bench.py > $OUT/bench_A.json 2> $OUT/bench_A.err \
&& python3 -c "import json; d=json.load(open('$OUT/bench_A.json')); print('A', d['value'], d['roofline']['frac'], (d['valu_issue'] or {}).get('frac'), d['cpu_baseline'], d['parity_vs_cpu_oracle'])"
