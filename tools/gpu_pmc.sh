#!/bin/bash
# HBM traffic of the decode kernel: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes
# (MI355X_MICROARCH.md "rocprofv3 PMC slots": they do not fit one pass), kernel trace alongside.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
for cfg in ${CFGS:-A W}; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_$cfg" -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > "$OUT/fetch_$cfg.json" 2> "$OUT/fetch_$cfg.err" \
  && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_$cfg" -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu > "$OUT/write_$cfg.json" 2> "$OUT/write_$cfg.err" \
  || exit $?
done
echo "pmc done"
