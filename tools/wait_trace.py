#!/usr/bin/env python3
"""Per-wave split of the packed loop's time, from the FPLDPC_WAIT_TRACE diagnostic build's
`<FPLDPC_WG_TRACE>.waves` file ([grid][64] uint64: wave w's {check-step cycles, per-step barrier
cycles, packed-loop cycles, steps, the other barriers' cycles (refills, stores, the final-update
syndrome pass, the range check)} at 5w..5w+4, s_memtime shader cycles).

For each wave index: the share of the loop in the check step (ck.step plus the flag ballots), at the
step barrier (waiting for the workgroup's other waves), and elsewhere (LLR copy, frame ends,
refills, stores; of it the other barriers).  Waves of one SIMD are w, w + 4, w + 8 (round-robin).
Builds with FPLDPC_WAIT_TRACE=2 / 3 put other regions into the fifth word ("other barriers" in the
output): 2, the per-step LLR copy; 3, everything after the per-step barrier (the end decisions,
stores, refills) -- tools/gpu_waitsplit.sh runs all three.

    FPLDPC_WG_TRACE=/tmp/t.bin FPLDPC_LIB_PATH=build/wait/libfpldpc.so python bench.py --config R ...
    tools/wait_trace.py /tmp/t.bin.waves [--json out.json]
"""
import argparse
import json

import numpy as np


def analyse(path):
    raw = np.fromfile(path, dtype=np.uint64).reshape(-1, 64)[:, :60].reshape(-1, 12, 5).astype(np.float64)
    live = raw[:, :, 2] > 0
    nw = int(live.any(axis=0).sum())
    rows = []
    for i in range(nw):
        sel = live[:, i]
        step, bar, loop, steps, bar2 = (raw[sel, i, j].sum() for j in range(5))
        rows.append({"wave": i, "simd": i % 4, "step_share": step / loop, "barrier_share": bar / loop,
                     "other_barrier_share": bar2 / loop, "other_share": 1 - (step + bar + bar2) / loop,
                     "cycles_per_step": loop / max(steps, 1), "step_cycles_per_step": step / max(steps, 1),
                     "barrier_cycles_per_step": bar / max(steps, 1)})
    tot = {k: float(np.mean([r[k] for r in rows]))
           for k in ("step_share", "barrier_share", "other_barrier_share", "other_share")}
    return {"waves": nw, "mean": tot, "per_wave": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("waves")
    ap.add_argument("--json")
    a = ap.parse_args()
    r = analyse(a.waves)
    print(f"waves per workgroup {r['waves']}; mean shares {r['mean']}")
    for x in r["per_wave"]:
        print(f"  wave {x['wave']:2d} (SIMD {x['simd']}): step {x['step_share']:.3f}  barrier {x['barrier_share']:.3f}  "
              f"other barriers {x['other_barrier_share']:.3f}  other {x['other_share']:.3f}   per step: {x['cycles_per_step']:.0f} cyc (step {x['step_cycles_per_step']:.0f}, "
              f"barrier {x['barrier_cycles_per_step']:.0f})")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(r, f, indent=1)


if __name__ == "__main__":
    main()
