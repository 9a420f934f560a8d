set -o pipefail
mkdir -p gpurun_out/gen3
timeout -k 10 600 python -m pytest tests/test_gpu_perftest.py -q -rf -x -s > gpurun_out/gen3/pytest.log 2>&1
