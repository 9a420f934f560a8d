set -o pipefail
mkdir -p gpurun_out/r1p
timeout -k 10 300 python tools/debug/w_scale.py > gpurun_out/r1p/w_scale.txt 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/r1p/pytest_gpu.log 2>&1; rc=$?
for c in A W; do timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/r1p/bench_$c.json 2>> gpurun_out/r1p/bench.err; done
exit $rc
