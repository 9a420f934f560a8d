#!/bin/bash
# A/B of alternative builds (FPLDPC_LIB_PATH) on the bench configs, alternating, optionally after
# the GPU parity suite.  Usage: TAG=x LIBS="base=build/ab/a.so g8=" CONFIGS="A W" PYTEST=1 tools/gpu_ab.sh
# (an empty path means the in-tree build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
if [ -n "$PYTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
for rep in 1 2; do
  for cfg in ${CONFIGS:-A W R}; do
    for lv in ${LIBS:-new=}; do
      name=${lv%%=*}; path=${lv#*=}
      FPLDPC_LIB_PATH=$path timeout -k 10 300 python bench.py --config $cfg --no-cpu ${BENCH_ARGS} > "$OUT/${name}_${cfg}_$rep.json" 2> "$OUT/${name}_${cfg}_$rep.err" || exit $?
    done
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_[AWR]_[12].json"))):
    try:
        d = json.load(open(f))
        print(os.path.basename(f), d["value"], d["config"]["kernel"].split(" ")[0], d["roofline"]["avg_launch_ms"], d["parity_vs_cpu_oracle"])
    except Exception as e:
        print(os.path.basename(f), "error", e)
PY
