#!/bin/bash
# rocprofv3 kernel stats of bench.py for the configs in CFGS (after an optional quick pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-stats}
mkdir -p "$OUT"
for cfg in ${CFGS:-A}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu ${BENCH_ARGS} > "$OUT/prof_$cfg.json" 2> "$OUT/prof_$cfg.err" || exit $?
  python3 - "$OUT/prof_$cfg/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.2f} us")
PY
done
echo "exit 0"
