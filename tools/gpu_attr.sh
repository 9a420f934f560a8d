#!/bin/bash
# Issue-stall attribution of the bench kernels: three rocprofv3 --pmc passes
# per config (each within the per-block counter limits), the flood kernel only.  CONFIGS="A W R"
# by default; summaries by tools/pmc_attr.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-attr}
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS_ATOMIC SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE"
for cfg in ${CONFIGS:-A W R}; do
  i=0
  for grp in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex flood --output-format csv -d "$OUT/${cfg}_p$i" -o run \
      -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu ${EXTRA_ARGS} > "$OUT/${cfg}_p$i.json" 2> "$OUT/${cfg}_p$i.err" || exit $?
  done
  echo "attr $cfg done"
done
