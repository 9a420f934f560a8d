export TMPDIR=/tmp
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kat.py -m gpu > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && grep -q "FAILED" $O/pytest.log && ! grep -qi "fault\|core dumped\|aborted" $O/pytest.log || [ $rc -eq 0 ] || exit $rc
for sp in 1 0 1 0; do
  FPLDPC_SPLIT_TAIL=$sp timeout -k 10 120 python bench.py --ebn0 4.5 --steps 50 --warmup 20 --no-cpu > $O/a45_s$sp.json 2>$O/a45_s$sp.err || exit 3
  FPLDPC_SPLIT_TAIL=$sp timeout -k 10 120 python bench.py --steps 50 --warmup 20 --no-cpu > $O/a0_s$sp.json 2>$O/a0_s$sp.err || exit 3
done
python -c "
import json,glob
for f in sorted(glob.glob('$O/a*_s*.json')):
    d=json.loads(open(f).read().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['parity_vs_cpu_oracle'])
"
