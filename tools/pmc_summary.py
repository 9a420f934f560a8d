#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/gpu_pmc.sh into profiles/<round>/pmc_traffic.json.

HBM bytes per launch of the decode kernel = 2 * FETCH_SIZE + WRITE_SIZE (KiB units), following
/opt/skills/guides/MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE tallies 128-B read requests at
64 B, i.e. half the bytes.  The factor is calibrated on this kernel's own known read: the LLR input
(frames * n * 2 B, read exactly once per launch) -- the raw FETCH_SIZE comes out at ~0.51x of it
(see the "calibration" field).

usage: tools/pmc_summary.py gpurun_out/<tag> profiles/<round>/pmc_traffic.json
"""
import csv
import json
import os
import sys

N = {"A": 2209, "W": 1944, "R": 2209}


def per_launch(d, counter, scale=1024.0):
    """Mean counter value per decode call: one decode launches each kernel (packed kernel +
    fallback pass) once, so per-kernel means are summed."""
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    by = {}
    for r in rows:
        if r["Counter_Name"] == counter and ("flood" in r["Kernel_Name"] or "bp_float" in r["Kernel_Name"]):
            v = by.setdefault(r["Kernel_Name"], [[], []])
            v[0].append(float(r["Counter_Value"]) * scale)
            v[1].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    total = sum(sum(v[0]) / len(v[0]) for v in by.values())
    dur = sum(sum(v[1]) / len(v[1]) for v in by.values())
    per_kernel = {k: {"bytes": sum(v[0]) / len(v[0]), "seconds": sum(v[1]) / len(v[1]), "launches": len(v[0])}
                  for k, v in by.items()}
    return total, dur, sorted(by), per_kernel


def main(src, dst):
    out = {}
    # one entry per profiled workload: fetch_<key> / write_<key> / sq_<key> passes of one bench command
    # (key: A, W, R, A_float, A_b8192, A_4.5dB, ...); "workload" is the config (+ _float) bench.py matches
    keys = sorted(d[len("fetch_"):] for d in os.listdir(src) if d.startswith("fetch_") and os.path.isdir(os.path.join(src, d)))
    for cfg in keys:
        fdir, wdir = os.path.join(src, f"fetch_{cfg}"), os.path.join(src, f"write_{cfg}")
        if not (os.path.isdir(fdir) and os.path.isdir(wdir)):
            continue
        fetch, tf, names, kf = per_launch(fdir, "FETCH_SIZE")
        write, tw, _, kw = per_launch(wdir, "WRITE_SIZE")
        bench = json.loads(open(os.path.join(src, f"fetch_{cfg}.json")).read().strip().splitlines()[-1])
        frames = bench["config"]["frames_per_gpu"]
        workload = bench["config"]["workload"][0] + ("_float" if bench.get("dtype") == "f64" else "")
        llr_bytes = frames * N[workload[0]] * (8 if workload.endswith("_float") else 2)
        out[cfg] = {
            "workload": workload,
            "kernel": names,
            "describe": bench["config"]["kernel"].split(" ")[0],
            "kernel_build_id": bench["config"]["kernel_build_id"],  # bench.py reports these counters only for this build
            "per_kernel": {"FETCH_SIZE": kf, "WRITE_SIZE": kw},
            "fetch_size_raw_bytes": fetch,
            "write_size_bytes": write,
            "hbm_bytes_per_launch": 2 * fetch + write,
            "calibration": {"known_llr_read_bytes": llr_bytes, "raw_fetch_over_llr": fetch / llr_bytes},
            "avg_launch_s_under_pmc": (tf + tw) / 2,
            "algorithmic_bytes_per_launch": frames * (bench["roofline"].get("hbm_streaming_equivalent") or {}).get("bytes_per_frame", bench["roofline"].get("bytes_per_frame_algorithmic", 0)),
            "profiled_frames": frames,
            "profiled_ebn0_db": bench["config"].get("ebn0_db"),
            "profiled_avg_iters": bench["ber"]["avg_iters"],
            "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE --kernel-trace, bench.py ({cfg})",
        }
        sdir = os.path.join(src, f"sq_{cfg}")
        if os.path.isdir(sdir):  # issue counters of the same kernels (separate --pmc pass)
            names = sorted({r["Counter_Name"] for r in csv.DictReader(open(os.path.join(sdir, "run_counter_collection.csv")))})
            sq = {c: per_launch(sdir, c, scale=1.0)[0] for c in names}
            t_sq = per_launch(sdir, "SQ_INSTS_VALU", scale=1.0)[1]
            out[cfg]["sq"] = dict(sq, avg_launch_s_under_pmc=t_sq,
                                  clock_ghz=sq["GRBM_GUI_ACTIVE"] / 8 / t_sq / 1e9 if t_sq and "GRBM_GUI_ACTIVE" in sq else None,
                                  source=f"rocprofv3 --pmc {' '.join(names)} --kernel-trace, bench.py ({cfg})")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
