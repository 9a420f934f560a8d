#!/usr/bin/env python3
"""The early-termination tail of one packed-kernel launch, from an FPLDPC_WG_TRACE file of the
FPLDPC_TAIL_TRACE=1 diagnostic build (flood_pk: trace words 4..7 = thread 0's s_memrealtime when a
pull first found the queue empty, when the workgroup entered the split tail, the steps it then ran
with two live frames | one live frame (packed) << 32, and the steps in the split form).

Prints (and with --json writes) when the queue emptied, how the launch's workgroup-time after that
splits into two live frames / one live frame / the split form, the histogram of how long each
workgroup ran in each state, and the live-workgroup curve over the launch (the empty wave slots).

    FPLDPC_WG_TRACE=/tmp/t.bin FPLDPC_LIB_PATH=build/tail/libfpldpc.so python bench.py --ebn0 4.5 ...
    tools/tail_trace.py /tmp/t.bin [--json out.json]
"""
import argparse
import json

import numpy as np


def analyse(path):
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    t = t[t[:, 2] > 0]
    t0, t1 = t[:, 1].astype(np.int64), t[:, 2].astype(np.int64)
    temp, tsp = t[:, 4].astype(np.int64), t[:, 5].astype(np.int64)
    two = (t[:, 6] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    one = (t[:, 6] >> np.uint64(32)).astype(np.int64)
    spl = t[:, 7].astype(np.int64)
    base = t0.min()
    us = lambda x: (x - base) / 100.0  # noqa: E731  (100 MHz s_memrealtime)
    start, end = us(t0), us(t1)
    empty = np.where(temp > 0, us(temp), np.nan)
    split = np.where(tsp > 0, us(tsp), np.nan)
    q_empty = np.nanmin(empty)  # the first pull anywhere that found the queue empty
    launch = end.max()
    # per workgroup after its own queue-empty stamp: two live (until the split entry or, without a
    # split, in proportion to the step counts), one live packed, split
    after = np.maximum(end - np.nan_to_num(empty, nan=end), 0)
    t_split = np.where(np.isnan(split), 0.0, end - np.nan_to_num(split))
    rest = np.maximum(after - t_split, 0)
    steps = np.maximum(two + one, 1)
    t_two = rest * two / steps
    t_one = rest * one / steps
    # live workgroups over time (3 per CU resident: the wave-slot occupancy)
    grid = np.linspace(0, launch, 400)
    live = np.array([(start <= x).sum() - (end <= x).sum() for x in grid])
    occ = np.trapezoid(live, grid) / (len(t) * launch)
    occ_after = np.trapezoid(live[grid >= q_empty], grid[grid >= q_empty]) / (len(t) * max(launch - q_empty, 1e-9))
    # per compute unit (xcc, se, sh, cu from HW_ID): its frames, its end, and how long its last
    # workgroup ran alone (one wave per SIMD: half the issue rate of two or more)
    ids = t[:, 0]
    xcc = ((ids >> np.uint64(32)) & np.uint64(0xF)).astype(np.int64)
    hw = (ids & np.uint64(0xFFFFFFFF)).astype(np.int64)
    key = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
    alone, cu_end = [], []
    for k in np.unique(key):
        e = np.sort(end[key == k])
        cu_end.append(e[-1])
        alone.append(e[-1] - e[-2] if len(e) > 1 else 0.0)
    hist = lambda v: {f"{lo}-{lo + 25}us": int(((v >= lo) & (v < lo + 25)).sum()) for lo in range(0, int(v.max()) + 25, 25)}  # noqa: E731
    wg_time = float(after.sum())
    out = {
        "workgroups": int(len(t)), "launch_us": float(launch), "queue_empty_us": float(q_empty),
        "queue_empty_frac_of_launch": float(q_empty / launch),
        "wave_slot_occupancy": float(occ), "wave_slot_occupancy_after_queue_empty": float(occ_after),
        "wg_us_after_own_empty": {"total": wg_time, "two_live": float(t_two.sum()), "one_live_packed": float(t_one.sum()),
                                  "split": float(t_split.sum())},
        "workgroups_two_live_at_empty": int((two > 0).sum()),
        "steps_after_empty": {"two_live": int(two.sum()), "one_live_packed": int(one.sum()), "split": int(spl.sum())},
        "hist_us_two_live": hist(t_two), "hist_us_split": hist(t_split),
        "cus": int(len(cu_end)), "cu_end_us_percentiles": {q: float(np.percentile(cu_end, q)) for q in (0, 10, 50, 90, 100)},
        "cu_last_workgroup_alone_us": {"mean": float(np.mean(alone)), "p90": float(np.percentile(alone, 90)),
                                        "max": float(np.max(alone))},
        "end_us_percentiles": {q: float(np.percentile(end, q)) for q in (10, 50, 90, 99, 100)},
        "live_curve": [[float(x), int(v)] for x, v in zip(grid[::20], live[::20])],
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--json")
    a = ap.parse_args()
    r = analyse(a.trace)
    for k, v in r.items():
        if k != "live_curve":
            print(f"{k}: {v}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(r, f, indent=1)


if __name__ == "__main__":
    main()
