set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6q3; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "split_tail or keep_edges or compat or precheck" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
TAG=r6q3/ab REPS=2 VARIANTS="base|build/ab/base.so| new|| eg256||FPLDPC_ENDGAME=256 eg512||FPLDPC_ENDGAME=512 eg1024||FPLDPC_ENDGAME=1024 eg2048||FPLDPC_ENDGAME=2048" CASES="A:--config A;A45:--config A --ebn0 4.5" bash tools/ab_env.sh > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
tail -14 $OUT/ab.txt
for w in "eg512 A45 --ebn0 4.5" "eg0 A45 --ebn0 4.5" "eg512 A0" ; do
  set -- $w; eg=${1#eg}; name=$2; shift 2
  FPLDPC_ENDGAME=$eg FPLDPC_WG_TRACE=$OUT/tail_${name}_eg$eg.bin FPLDPC_LIB_PATH=build/tail/libfpldpc.so timeout -k 10 300 python bench.py "$@" --steps 3 --warmup 3 --no-cpu > $OUT/tail_${name}_eg$eg.json 2>&1 || exit 1
  python tools/tail_trace.py $OUT/tail_${name}_eg$eg.bin --json $OUT/tail_${name}_eg$eg.summary.json | head -7
done
for cfg in R A W; do
  FPLDPC_WG_TRACE=$OUT/wait_$cfg.bin FPLDPC_LIB_PATH=build/wait/libfpldpc.so timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 2 --no-cpu > $OUT/wait_$cfg.json 2>&1 || exit 1
done
timeout -k 10 600 python tools/frame_latency.py > $OUT/frame_latency.jsonl 2> $OUT/frame_latency.err; rc=$?; cat $OUT/frame_latency.jsonl; exit $rc
