set -o pipefail
mkdir -p gpurun_out/fl4
timeout -k 10 300 python -m pytest tests/test_gpu_perftest.py -q -rf -k "float" > gpurun_out/fl4/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --config A --decoder float --steps 5 --warmup 1 > gpurun_out/fl4/bench_A.json 2> gpurun_out/fl4/bench_A.err && \
timeout -k 10 300 python bench.py --config W --decoder float --steps 5 --warmup 1 > gpurun_out/fl4/bench_W.json 2> gpurun_out/fl4/bench_W.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fl4/prof -o run --output-format csv -- python3 bench.py --config A --decoder float --steps 3 --warmup 1 --no-cpu > gpurun_out/fl4/prof.json 2> gpurun_out/fl4/prof.err
