set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/stamps2; mkdir -p $OUT
for v in stamps stamps_abl3 stamps_abl2; do
  FPLDPC_LIB_PATH=build/ab/$v.so FPLDPC_WG_TRACE=$OUT/$v.bin timeout -k 10 120 python bench.py --no-cpu --steps 2 --warmup 1 > $OUT/$v.json 2> $OUT/$v.err || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('$OUT/$v.json')); print(d['value'], d['roofline']['avg_launch_ms'])")"
  python3 tools/wg_trace.py $OUT/$v.bin | head -5
done
