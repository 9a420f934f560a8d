set -o pipefail
TAG=r1k bash tools/gpu_check.sh && TAG=r1k bash tools/gpu_pmc.sh && BENCH_ARGS="--config R --steps 3 --warmup 1 --no-cpu" timeout -k 10 600 python bench.py --config R --no-cpu --steps 5 > gpurun_out/r1k/bench_R.json 2> gpurun_out/r1k/bench_R.err
