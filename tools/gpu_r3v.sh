#!/bin/bash
# SDWA slot addresses vs the default (v_add_u16 / shift + add), 4 repetitions: A, A at 4.5 dB, R.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3v}
mkdir -p "$OUT"
timeout -k 10 900 python tools/ab.py "$OUT/ab" 4 'A=--config A' 'A45=--ebn0 4.5' 'R=--config R' -- 'def=' \
  'sdwa=FPLDPC_LIB_PATH=build/ab/sdwa.so'
