set -o pipefail
mkdir -p gpurun_out/r1l
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r1l/pytest_gpu.log 2>&1; rc=$?
timeout -k 10 300 python bench.py --config R --no-cpu --steps 5 > gpurun_out/r1l/bench_R.json 2> gpurun_out/r1l/bench_R.err
FPLDPC_CLOCK_PROBE=1 timeout -k 10 300 python bench.py --config R --no-cpu --steps 2 --warmup 1 > /dev/null 2> gpurun_out/r1l/clock_R.txt
exit $rc
