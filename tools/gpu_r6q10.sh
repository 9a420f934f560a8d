#!/bin/bash
# Round-6 call: the per-frame path with its c2v double buffer and index table in LDS (flood_edges<DC,
# true>): its parity tests (and the global-memory form forced by FPLDPC_EDGES_GLOBAL), then latency.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q10}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_compat.py tests/test_gpu_perftest.py -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_compat.log 2>&1; rc=$?; tail -2 $OUT/pytest_compat.log; [ $rc = 0 ] || exit $rc
FPLDPC_EDGES_GLOBAL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_compat.py -m gpu -q -rf --timeout 300 --timeout-method thread -k keep_edges > $OUT/pytest_compat_global.log 2>&1; rc=$?; tail -2 $OUT/pytest_compat_global.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/frame_latency.py > $OUT/frame_latency.jsonl 2> $OUT/frame_latency.err; rc=$?; cat $OUT/frame_latency.jsonl; [ $rc = 0 ] || exit $rc
TAG=${TAG:-r6q10}/abR REPS=2 VARIANTS="base|| mtrknpr|build/ab/m_trk_npr.so| mnpr|build/ab/m_npr.so| mnone|build/ab/m_none.so|" CASES="R:--config R" bash tools/ab_env.sh > $OUT/abR.txt 2>&1 || { tail -5 $OUT/abR.txt; exit 1; }
tail -6 $OUT/abR.txt
