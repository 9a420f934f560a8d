#!/bin/bash
# rocprofv3 kernel stats of the early-termination points (A at 4.5 dB, W at 2 dB; one batch at a
# time, then two batches in flight), for profiles/<round>/et/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-etstats}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/A45" -o run --output-format csv -- python3 bench.py --ebn0 4.5 --no-cpu > "$OUT/A45.json" 2> "$OUT/A45.err" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/W2" -o run --output-format csv -- python3 bench.py --config W --ebn0 2.0 --no-cpu > "$OUT/W2.json" 2> "$OUT/W2.err" \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/A45_if" -o run --output-format csv -- python3 bench.py --ebn0 4.5 --no-cpu --steps 5 --warmup 1 --inflight-steps 50 > "$OUT/A45_if.json" 2> "$OUT/A45_if.err"
rc=$?; echo "exit $rc"; exit $rc
