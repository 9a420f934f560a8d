#!/bin/bash
# W: the table kernel in a 512-thread workgroup (2 checks per lane, 80 VGPRs, 3 workgroups / CU),
# also capped at 2 / CU and with opaque loop starts, against the default 256-thread kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3q}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity.py::test_every_variant_parity[W]" "tests/test_gpu_parity.py::test_full_batch_early_termination" -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
K='FPLDPC_KERNEL=flood_tab2<DC=8,CPL=2,lo=1,NT=512>'
timeout -k 10 900 python tools/ab.py "$OUT/ab" 3 'W=--config W' 'W2=--config W --ebn0 2.0' -- 'new=' \
  "n512=$K" "n512g2=$K|FPLDPC_GRID_PER_CU=2" "n512op=$K|FPLDPC_LIB_PATH=build/ab/tabop.so"
