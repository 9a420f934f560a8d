#!/bin/bash
# The driver's bench command (--steps 20 --warmup 5) with and without the minimum warm-up time,
# against the default 30 / 50 steps: how much of the short run's deficit is the clock settling.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s}
mkdir -p "$OUT"
timeout -k 10 900 python tools/ab.py "$OUT/ab" 4 'd0=--steps 20 --warmup 5 --min-warmup-s 0 --no-cpu' \
  'd25=--steps 20 --warmup 5 --no-cpu' 'def=--no-cpu' -- 'new='
