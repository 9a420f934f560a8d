#!/bin/bash
# Lock-step experiment: three frame pairs per 768-thread workgroup (flood_lock<P=47,S=3>), parity
# (every A variant incl. the int16-range fallback frames), then an A/B against the default kernel
# at 30 iterations and with early termination at 4.5 dB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3u}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_every_variant_parity[A]" -q -rf --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
K='FPLDPC_KERNEL=flood_lock<P=47,S=3>'
timeout -k 10 600 python tools/ab.py "$OUT/ab" 3 'A=--config A' 'A45=--ebn0 4.5' 'A4=--ebn0 4.0' -- 'def=' "lock=$K"
