set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/bench5; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench_A.json 2> $OUT/bench_A.err && \
timeout -k 10 300 python bench.py --config W --no-cpu > $OUT/bench_W.json 2> $OUT/bench_W.err && \
timeout -k 10 300 python bench.py --config R --no-cpu > $OUT/bench_R.json 2> $OUT/bench_R.err && \
for c in A W R; do python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['roofline']['frac'], d['valu_issue'], d['cpu_baseline'])"; done
