set -o pipefail
mkdir -p gpurun_out/gen4
timeout -k 10 300 python tools/bench_gen.py > gpurun_out/gen4/bench_gen.jsonl 2> gpurun_out/gen4/bench_gen.err
