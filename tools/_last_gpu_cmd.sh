set -o pipefail
mkdir -p gpurun_out/opt3
for rep in 1 2; do
  FPLDPC_LIB_PATH="$PWD/exp/libs/libfpldpc_a0.so" timeout -k 10 300 python bench.py --no-cpu --steps 30 > gpurun_out/opt3/A_a0.$rep.json 2>> gpurun_out/opt3/b.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu --steps 30 > gpurun_out/opt3/A_default.$rep.json 2>> gpurun_out/opt3/b.err || exit 1
done
timeout -k 10 300 python bench.py --config W --no-cpu --steps 30 > gpurun_out/opt3/W.json 2>> gpurun_out/opt3/b.err
