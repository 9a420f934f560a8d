set -o pipefail
mkdir -p gpurun_out/r1d
timeout -k 10 900 python -m pytest tests -m gpu -x -q -rA > gpurun_out/r1d/pytest_gpu.log 2>&1
