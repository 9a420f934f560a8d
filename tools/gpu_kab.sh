#!/bin/bash
# A/B of kernel variants (FPLDPC_KERNEL) on one config, alternating, 2 reps.
# Usage: CFG=A KERNELS="flood_array2<P=47,W=3>;flood_array2<P=47,W=4,walk>" tools/gpu_kab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-kab}
mkdir -p "$OUT"
IFS=';' read -ra KS <<< "$KERNELS"
for rep in 1 2; do
  for k in "${KS[@]}"; do
    FPLDPC_KERNEL="$k" timeout -k 10 300 python bench.py --config ${CFG:-A} --no-cpu ${BENCH_ARGS} > "$OUT/x.json" 2> "$OUT/x.err" || { tail -5 "$OUT/x.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/x.json')); print(d['value'], d['roofline']['avg_launch_ms'], d['config']['kernel'], d['parity_vs_cpu_oracle'])"
  done
done
