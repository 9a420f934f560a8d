set -o pipefail
cd "${GRAFT_REPO_ROOT}"
TAG=r1_sqA BENCH_ARGS="--steps 2 --warmup 1 --no-cpu" bash tools/gpu_sq.sh \
&& TAG=r1_sqW BENCH_ARGS="--config W --steps 2 --warmup 1 --no-cpu" bash tools/gpu_sq.sh \
&& TAG=r1_sqR BENCH_ARGS="--config R --steps 2 --warmup 1 --no-cpu" bash tools/gpu_sq.sh
