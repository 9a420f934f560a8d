set -o pipefail
mkdir -p gpurun_out/r1c
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r1c/pytest_gpu.log 2>&1; rc=$?
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r1c/bench_A.json 2> gpurun_out/r1c/bench_A.err
exit $rc
