#!/bin/bash
# Float decoder A/B on config A: builds (FPLDPC_LIB_PATH) x grid caps (FPLDPC_FLOAT_WG_PER_CU), each
# with a bench line and FETCH_SIZE / WRITE_SIZE passes.  Usage: RUNS="base:0 fk=build/ab/fk.so:0 ..." tools/gpu_float_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-float_ab}
mkdir -p "$OUT"
for r in ${RUNS:-base:0}; do
  spec=${r%%:*}; cap=${r##*:}; name=${spec%%=*}; lib=""; [ "$spec" != "$name" ] && lib=${spec#*=}
  tag=${name}_wg$cap
  export FPLDPC_LIB_PATH=$lib FPLDPC_FLOAT_WG_PER_CU=$cap
  timeout -k 10 300 python bench.py --decoder float --steps 4 --warmup 1 --no-cpu > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" \
  && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$tag" -o run -- python3 bench.py --decoder float --steps 2 --warmup 1 --no-cpu > /dev/null 2> "$OUT/fetch_$tag.err" \
  && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$tag" -o run -- python3 bench.py --decoder float --steps 2 --warmup 1 --no-cpu > /dev/null 2> "$OUT/write_$tag.err" \
  || exit $?
  python3 - "$OUT" "$tag" <<'PY'
import csv, json, sys
out, tag = sys.argv[1], sys.argv[2]
d = json.load(open(f"{out}/bench_{tag}.json"))
def kib(kind, c):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f"{out}/{kind}_{tag}/run_counter_collection.csv"))
         if r["Counter_Name"] == c and "bp_float" in r["Kernel_Name"]]
    return sum(v) / len(v) * 1024 / 1e9
f, w = kib("fetch", "FETCH_SIZE"), kib("write", "WRITE_SIZE")
print(f"{tag}: {d['value']:.1f} Mb/s, launch {d['roofline'].get('avg_launch_ms')} ms, FETCH x2 {2*f:.2f} GB + WRITE {w:.2f} GB = {2*f+w:.2f} GB/launch, parity {d['parity_vs_cpu_oracle']}")
PY
done
echo "exit 0"
