#!/bin/bash
# Two lanes per check (flood_split<P=47>): parity (every variant + the 4096-frame early-termination
# batch forced onto it), then A/B against the default kernel, 3 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3z}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "every_variant" > "$OUT/parity_split.log" 2>&1 \
&& FPLDPC_KERNEL=flood_split timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_parity.py::test_full_batch_early_termination[A-4.5]" >> "$OUT/parity_split.log" 2>&1 \
&& timeout -k 10 900 python tools/ab.py "$OUT/ab" ${REPS:-3} 'A=--config A' 'A45=--ebn0 4.5' -- 'def=' \
  'split=FPLDPC_KERNEL=flood_split' 'split_g2=FPLDPC_KERNEL=flood_split|FPLDPC_GRID_PER_CU=2'
rc=$?
echo "exit $rc"; exit $rc
