#!/bin/bash
# Check-step throughput decomposition (tools/ubench/step_mix.hip): one build per FPLDPC_ABLATE value,
# each run under its own time limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-stepmix}
mkdir -p "$OUT"
for ab in ${ABLS:-0 1 16 32 64 112 113}; do
  echo "== $ab" >> "$OUT/step_mix.txt"; timeout -k 10 60 ./tools/ubench/step_mix_$ab >> "$OUT/step_mix.txt" 2>&1 || exit $?
done
cat "$OUT/step_mix.txt"
