#!/bin/bash
# SQ / LDS counter passes on the bench kernel (one rocprofv3 --pmc pass per counter group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sq}
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex flood --output-format csv -d "$OUT/sq$i" -o run -- python3 bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu} > "$OUT/sq$i.json" 2> "$OUT/sq$i.err" || exit $?
done
echo sq done
