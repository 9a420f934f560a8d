#!/usr/bin/env python3
"""Summarise an FPLDPC_WG_TRACE file (diagnostic): per-workgroup {xcc<<32 | HW_ID, start, end,
frames, 4 stamp sums} of one packed-kernel launch.  Prints how frames spread over workgroups and compute units
and how long the tail after the median workgroup end is.

    FPLDPC_WG_TRACE=/tmp/t.bin python bench.py --steps 1 --warmup 0 --no-cpu && tools/wg_trace.py /tmp/t.bin
"""
import collections
import sys

import numpy as np


def main(path):
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    t = t[t[:, 2] > 0]
    ids, t0, t1, fr = t[:, 0], t[:, 1].astype(np.int64), t[:, 2].astype(np.int64), t[:, 3].astype(np.int64)
    xcc = (ids >> np.uint64(32)).astype(np.int64) & 0xF
    hw = (ids & np.uint64(0xFFFFFFFF)).astype(np.int64)
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    base = t0.min()
    s_us, e_us = (t0 - base) / 100.0, (t1 - base) / 100.0  # 100 MHz s_memrealtime
    st = t[:, 4:8].astype(np.float64)
    if st.sum() > 0:  # traces from builds that recorded per-phase cycles of wave 0 (round 1-3 diagnostics)
        for f in sorted(set(fr.tolist())):
            sel = fr == f
            cyc = st[sel].mean(axis=0) / (f / 2 * 30)  # per flooding step (2 frames per workgroup, 30 steps)
            print(f"  {f:2d}-frame workgroups: cycles per step: gather {cyc[0]:.0f}  phase-1 {cyc[1]:.0f}  "
                  f"phase-2+scatter {cyc[2]:.0f}  flags/barrier/copy {cyc[3]:.0f}  total {cyc.sum():.0f}")
    print(f"workgroups {len(t)}  distinct CUs {len(set(key.tolist()))}  frames {fr.sum()}")
    print("frames per workgroup:", dict(sorted(collections.Counter(fr.tolist()).items())))
    wg_per_cu = collections.Counter(key.tolist())
    print("workgroups per CU:", dict(sorted(collections.Counter(wg_per_cu.values()).items())))
    f_cu = collections.defaultdict(int)
    for k, f in zip(key.tolist(), fr.tolist()):
        f_cu[k] += f
    print("frames per CU:", dict(sorted(collections.Counter(f_cu.values()).items())))
    print(f"start spread {s_us.max() - s_us.min():.1f} us; end: min {e_us.min():.1f}  median {np.median(e_us):.1f}  "
          f"max {e_us.max():.1f} us")
    for q in (10, 50, 90, 99):
        print(f"  end p{q}: {np.percentile(e_us, q):.1f} us")
    by_f = collections.defaultdict(list)
    for f, e in zip(fr.tolist(), e_us.tolist()):
        by_f[f].append(e)
    for f in sorted(by_f):
        v = np.array(by_f[f])
        print(f"  workgroups with {f} frames: {len(v)}, end {v.min():.1f}..{v.max():.1f} us (mean {v.mean():.1f})")


if __name__ == "__main__":
    main(sys.argv[1])
