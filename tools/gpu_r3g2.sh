#!/bin/bash
# W / W at 2 dB against workgroups per CU and the 512-thread table kernel; A at 4.5 dB at 2 per CU.  3 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3g2}
mkdir -p "$OUT"
timeout -k 10 900 python tools/ab.py "$OUT/abw" ${REPS:-3} 'W=--config W' 'W2=--config W --ebn0 2.0' -- 'def=' \
  'g3=FPLDPC_GRID_PER_CU=3' 'g2=FPLDPC_GRID_PER_CU=2' 'nt512=FPLDPC_KERNEL=flood_tab2<DC=8,CPL=2,lo=1,NT=512>' \
&& timeout -k 10 600 python tools/ab.py "$OUT/aba" ${REPS:-3} 'A=--config A' 'A45=--ebn0 4.5' -- 'def=' 'g2=FPLDPC_GRID_PER_CU=2'
rc=$?
echo "exit $rc"; exit $rc
