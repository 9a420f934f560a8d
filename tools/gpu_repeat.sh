#!/bin/bash
# Repeatability of the headline: the driver's default bench command 5 times on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-repeat}
mkdir -p "$OUT"
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --no-cpu > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit 1
done
python - "$OUT" <<'P'
import json, sys, statistics as st
v = [json.loads(open(f"{sys.argv[1]}/bench_{i}.json").read().strip().splitlines()[-1])["value"] for i in range(1, 6)]
print("A headline, 5 runs of python bench.py --no-cpu:", v, "median", st.median(v), "spread %.2f %%" % (100 * (max(v) - min(v)) / st.median(v)))
P
