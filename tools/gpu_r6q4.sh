#!/bin/bash
# Round-6 call: the W split form under W-unit code-generation options (A/B), its parity, and the
# issue-stall counters of R beside the FPLDPC_WAIT_TRACE build's barrier stamps (same build).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q4}; mkdir -p $OUT
FPLDPC_ALLOW_STALE_PROFILE=1 FPLDPC_LIB_PATH=build/ab/wsplit.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "split_tail or full_batch or every_variant or int16_range" > $OUT/pytest_wsplit.log 2>&1; rc=$?; tail -2 $OUT/pytest_wsplit.log; [ $rc = 0 ] || exit $rc
TAG=$TAG/abW REPS=2 VARIANTS="base|build/ab/base.so| wsplit|build/ab/wsplit.so| wsnotrk|build/ab/ws_notrk.so| wsilp|build/ab/ws_ilp.so| wsnpr|build/ab/ws_npr.so| wstrknpr|build/ab/ws_trk_npr.so|" CASES="W:--config W;W2:--config W --ebn0 2.0" bash tools/ab_env.sh > $OUT/abW.txt 2>&1 || { tail -5 $OUT/abW.txt; exit 1; }
tail -13 $OUT/abW.txt
SQ="SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
for v in "wait build/wait/libfpldpc.so" "base build/ab/base.so"; do
  set -- $v
  FPLDPC_WG_TRACE=$OUT/wait_R_$1.bin FPLDPC_LIB_PATH=$2 timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $OUT/pmc_R_$1 -o run -- python3 bench.py --config R --steps 3 --warmup 1 --no-cpu > $OUT/pmc_R_$1.json 2> $OUT/pmc_R_$1.err || exit 1
  echo "pmc R $1 done"
done
python tools/wait_trace.py $OUT/wait_R_wait.bin.waves --json $OUT/wait_R.summary.json > $OUT/wait_R.txt; head -1 $OUT/wait_R.txt
echo exit 0
