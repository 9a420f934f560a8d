set -o pipefail
mkdir -p gpurun_out/r1e
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r1e/pytest_gpu.log 2>&1; rc=$?
for k in "flood_array2<P=47,W=3" "flood_array2<P=47,W=4" "flood_array<P=47"; do
  FPLDPC_KERNEL="$k" timeout -k 10 300 python bench.py --no-cpu >> gpurun_out/r1e/bench_variants.jsonl 2>> gpurun_out/r1e/bench.err || break
done
exit $rc
