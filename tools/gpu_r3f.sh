#!/bin/bash
# R with the slot offsets in an LDS table: parity (every variant, reference fixtures, KATs), then
# an A/B against the walked-offset layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3f}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_compat.py -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 python tools/ab.py "$OUT/ab" 2 'R=--config R' 'R8=--config R --ebn0 8' -- 'tab=' 'walk=FPLDPC_KERNEL=flood_array2<P=47,CPL=2>'
