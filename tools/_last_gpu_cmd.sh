set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/activity; mkdir -p $OUT
for v in "rand" "zero --llr-fill 0" "neg --llr-fill -16" "rand2"; do
  set -- $v; name=$1; shift
  FPLDPC_CLOCK_PROBE=1 timeout -k 10 120 python bench.py --no-cpu --steps 6 --warmup 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  echo "$name $(python3 -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['roofline']['avg_launch_ms'], d['ber']['avg_iters'], d['parity_vs_cpu_oracle'])") $(grep clock $OUT/$name.err | tail -1)"
done
