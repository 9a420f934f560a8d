#!/bin/bash
# End-game pulling (FPLDPC_ENDGAME=T: the last T frames go to each CU's oldest workgroup only):
# parity with it on, then A/B over T, 3 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3e}
mkdir -p "$OUT"
FPLDPC_ENDGAME=512 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > "$OUT/parity_eg.log" 2>&1 \
&& timeout -k 10 900 python tools/ab.py "$OUT/ab" ${REPS:-3} 'A=--config A' 'A45=--ebn0 4.5' 'W=--config W' 'W2=--config W --ebn0 2.0' -- 'def=' \
  'eg256=FPLDPC_ENDGAME=256' 'eg512=FPLDPC_ENDGAME=512' 'eg1024=FPLDPC_ENDGAME=1024' 'eg2048=FPLDPC_ENDGAME=2048'
rc=$?
echo "exit $rc"; exit $rc
