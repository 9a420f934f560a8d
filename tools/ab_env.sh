#!/bin/bash
# A/B of builds and environment settings on bench workloads, interleaved, REPS repetitions.
#   VARIANTS="base|build/ab/base.so| st0||FPLDPC_SPLIT_TAIL=0"   name|library (empty: in-tree)|env (comma-separated)
#   CASES="A:--config A  A45:--config A --ebn0 4.5"                name:bench arguments
# Prints one line per run and a mean per case / variant.  Every run has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abenv}
mkdir -p "$OUT"
IFS=' ' read -r -a VS <<< "${VARIANTS}"
mapfile -t CS < <(echo "${CASES:-A:--config A}" | tr ';' '\n')
for rep in $(seq 1 ${REPS:-2}); do
  for c in "${CS[@]}"; do
    cname=${c%%:*}; cargs=${c#*:}
    for v in "${VS[@]}"; do
      IFS='|' read -r vname vlib venv <<< "$v"
      envs=()
      [ -n "$vlib" ] && envs+=("FPLDPC_LIB_PATH=$vlib")
      [ -n "$venv" ] && IFS=',' read -r -a more <<< "$venv" && envs+=("${more[@]}")
      env "${envs[@]}" timeout -k 10 300 python bench.py $cargs --no-cpu ${BENCH_ARGS} > "$OUT/${vname}_${cname}_$rep.json" 2> "$OUT/${vname}_${cname}_$rep.err" || exit $?
    done
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_[0-9].json"))):
    b = os.path.basename(f)[:-5]
    v, c, r = b.rsplit("_", 2) if b.count("_") >= 2 else (b, "", "")
    try:
        d = json.load(open(f))
        acc[(c, v)].append((d["value"], d["roofline"]["avg_launch_ms"], d["parity_vs_cpu_oracle"]))
        print(b, d["value"], d["roofline"]["avg_launch_ms"], d["parity_vs_cpu_oracle"])
    except Exception as e:
        print(b, "error", e)
print("summary (mean value per case / variant):")
for (c, v), xs in sorted(acc.items()):
    print(f"  {c:8s} {v:14s} {sum(x[0] for x in xs) / len(xs):10.1f} Mb/s  {sum(x[1] for x in xs) / len(xs):.4f} ms  parity {all(x[2] for x in xs)}")
PY
