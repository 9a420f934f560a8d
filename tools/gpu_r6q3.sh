#!/bin/bash
# Round-6 call: parity of the end game and of the W split form (FPLDPC_W_SPLIT build), A/B of the end
# game on A and of the W split form on W, tail / wait traces, the per-frame latency.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q3}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "split_tail or keep_edges or compat or precheck" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
FPLDPC_LIB_PATH=build/ab/wsplit.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "split_tail or full_batch or every_variant or int16_range" > $OUT/pytest_wsplit.log 2>&1; rc=$?; tail -2 $OUT/pytest_wsplit.log; [ $rc = 0 ] || exit $rc
TAG=$TAG/abA REPS=2 VARIANTS="base|build/ab/base.so| new|| eg256||FPLDPC_ENDGAME=256 eg512||FPLDPC_ENDGAME=512 eg1024||FPLDPC_ENDGAME=1024 eg2048||FPLDPC_ENDGAME=2048" CASES="A:--config A;A45:--config A --ebn0 4.5" bash tools/ab_env.sh > $OUT/abA.txt 2>&1 || { tail -5 $OUT/abA.txt; exit 1; }
tail -13 $OUT/abA.txt
TAG=$TAG/abW REPS=2 VARIANTS="new|| wsplit|build/ab/wsplit.so| wsplit1k|build/ab/wsplit.so|FPLDPC_ENDGAME=1024 wsplit2k|build/ab/wsplit.so|FPLDPC_ENDGAME=2048" CASES="W:--config W;W2:--config W --ebn0 2.0" bash tools/ab_env.sh > $OUT/abW.txt 2>&1 || { tail -5 $OUT/abW.txt; exit 1; }
tail -9 $OUT/abW.txt
for w in "eg512 A45 --ebn0 4.5" "eg0 A45 --ebn0 4.5" "eg512 A0" ; do
  set -- $w; eg=${1#eg}; name=$2; shift 2
  FPLDPC_ENDGAME=$eg FPLDPC_WG_TRACE=$OUT/tail_${name}_eg$eg.bin FPLDPC_LIB_PATH=build/tail/libfpldpc.so timeout -k 10 300 python bench.py "$@" --steps 3 --warmup 3 --no-cpu > $OUT/tail_${name}_eg$eg.json 2>&1 || exit 1
  python tools/tail_trace.py $OUT/tail_${name}_eg$eg.bin --json $OUT/tail_${name}_eg$eg.summary.json | head -7
done
for cfg in R A W; do
  FPLDPC_WG_TRACE=$OUT/wait_$cfg.bin FPLDPC_LIB_PATH=build/wait/libfpldpc.so timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 2 --no-cpu > $OUT/wait_$cfg.json 2>&1 || exit 1
  python tools/wait_trace.py $OUT/wait_$cfg.bin.waves --json $OUT/wait_$cfg.summary.json | head -1
done
timeout -k 10 600 python tools/frame_latency.py > $OUT/frame_latency.jsonl 2> $OUT/frame_latency.err; rc=$?; cat $OUT/frame_latency.jsonl; exit $rc
