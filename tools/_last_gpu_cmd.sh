set -o pipefail
mkdir -p gpurun_out/r1j
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r1j/pytest_gpu.log 2>&1; rc=$?
for k in "flood_array2<P=47,W=3" "flood_array2<P=47,W=2"; do
  FPLDPC_KERNEL="$k" timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r1j/tmp.json 2>> gpurun_out/r1j/bench.err || exit 1
  cat gpurun_out/r1j/tmp.json >> gpurun_out/r1j/bench_variants.jsonl
done
exit $rc
