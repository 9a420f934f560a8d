#!/bin/bash
# R with the checks beyond 1024 two lanes per check (flood_array2<P=47,CPL=2,ldsoffs,mix>): parity
# (every variant; the R reference fixtures forced onto it), then A/B against the default, 3 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3m}
mkdir -p "$OUT"
M='flood_array2<P=47,CPL=2,ldsoffs,mix>'
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "every_variant" > "$OUT/parity_mix.log" 2>&1 \
&& FPLDPC_KERNEL="$M" timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kat.py -k "frames_r" >> "$OUT/parity_mix.log" 2>&1 \
&& timeout -k 10 900 python tools/ab.py "$OUT/ab" ${REPS:-3} 'R=--config R' -- 'def=' "mix=FPLDPC_KERNEL=$M"
rc=$?; tail -3 "$OUT/parity_mix.log"; echo "exit $rc"; exit $rc
