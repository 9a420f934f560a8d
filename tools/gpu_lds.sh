#!/bin/bash
# LDS bank conflicts and activity of the decode kernels (A, W, R): one rocprofv3 --pmc pass each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lds}
mkdir -p "$OUT"
for k in A W R; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/lds_$k" -o run -- python3 bench.py --config $k --steps 3 --warmup 1 --no-cpu > "$OUT/lds_$k.json" 2> "$OUT/lds_$k.err" || exit 1
done
echo done
