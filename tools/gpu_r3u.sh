#!/bin/bash
# SDWA slot addresses (one 32-bit add with a word select per slot instead of v_add_u16 / shift + add)
# and the lock-step experiment built on them: parity of every A and R variant on the SDWA build,
# then A/B: default vs SDWA (A, R) and the lock-step kernel (A, A at 4.5 dB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3u}
mkdir -p "$OUT"
FPLDPC_LIB_PATH=build/ab/sdwa.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_every_variant_parity" -q -rf --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
K='FPLDPC_KERNEL=flood_lock<P=47,S=3>'
timeout -k 10 900 python tools/ab.py "$OUT/ab" 3 'A=--config A' 'A45=--ebn0 4.5' 'R=--config R' -- 'def=' \
  'sdwa=FPLDPC_LIB_PATH=build/ab/sdwa.so' "lock=FPLDPC_LIB_PATH=build/ab/sdwa.so|$K"
