set -o pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/tr_final; mkdir -p $OUT
for v in new= nofinal=build/ab/nofinal.so never=build/ab/never.so; do
  n=${v%%=*}; p=${v#*=}
  FPLDPC_LIB_PATH=$p FPLDPC_WG_TRACE=$OUT/$n.bin timeout -k 10 120 python bench.py --steps 1 --warmup 2 --no-cpu > $OUT/$n.json 2>$OUT/$n.err || exit 1
  python3 tools/wg_trace.py $OUT/$n.bin > $OUT/$n.txt 2>&1
  FPLDPC_LIB_PATH=$p timeout -k 10 120 python bench.py --no-cpu > $OUT/${n}_b.json 2>>$OUT/$n.err || exit 1
done
for n in new nofinal never; do echo "== $n"; python3 -c "import json; d=json.load(open('$OUT/${n}_b.json')); print(d['value'])"; head -12 $OUT/$n.txt; done
