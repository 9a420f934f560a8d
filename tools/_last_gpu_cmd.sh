TAG=r1b bash tools/gpu_pmc.sh && timeout -k 10 900 python -m pytest tests/test_gpu_kat.py -x -q -s > gpurun_out/r1b/pytest_kat.log 2>&1
