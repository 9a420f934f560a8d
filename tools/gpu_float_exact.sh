#!/bin/bash
# Float decoder: exp_neg bit-exactness against the libm's exp, decoder outputs of the SGPR-constant /
# exp_neg build against the libm build bit for bit, then speed A/B (A, W float lines), 3 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-flx}
mkdir -p "$OUT"
timeout -k 10 60 build/float_exp_check > "$OUT/exp_check.txt" 2>&1 \
&& timeout -k 10 120 python tools/float_dump.py "$OUT/new.npz" > "$OUT/dump_new.log" 2>&1 \
&& FPLDPC_LIB_PATH=build/ab/fl_libm.so timeout -k 10 120 python tools/float_dump.py "$OUT/libm.npz" > "$OUT/dump_libm.log" 2>&1 \
&& python - "$OUT" > "$OUT/compare.txt" <<'P'
import sys, numpy as np
a = np.load(sys.argv[1] + "/new.npz"); b = np.load(sys.argv[1] + "/libm.npz")
bad = [k for k in a.files if a[k].tobytes() != b[k].tobytes()]
print("fields differing:", bad, "of", a.files)
sys.exit(1 if bad else 0)
P
[ $? -eq 0 ] && timeout -k 10 600 python tools/ab.py "$OUT/ab" ${REPS:-3} 'Af=--decoder float --steps 5 --warmup 2' 'Wf=--config W --decoder float --steps 5 --warmup 2' -- 'new=' 'libm=FPLDPC_LIB_PATH=build/ab/fl_libm.so'
rc=$?; cat "$OUT/exp_check.txt" "$OUT/compare.txt"; echo "exit $rc"; exit $rc
