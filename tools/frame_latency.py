#!/usr/bin/env python3
"""Per-frame drop-in latency: the reference's callers decode one frame per call
(PerfTest.cpp:121-128, :178-182, :304).  For each workload, the same AWGN frames go
  * through FP_Decoder::decode_general_fp / decode_fixpoint one call per frame
    (fpldpc_perftest frame_time: staging, the flood_edges launch, the copies back, the sync), and
  * through the CPU port of decode_general_fp (oracle/, one thread, the bench's cpu_baseline),
and one JSON line per workload gives microseconds per frame for both.  Run on the GPU box:
  python tools/frame_latency.py [--frames N] > profiles/r6/frame_latency.jsonl
"""
import argparse
import json
import math
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, code, Eb/N0, MAX_ITER, WIDTH_MASK, decode_fixpoint?)
WORKLOADS = [("A_30it", "A", 0.0, 30, 0xFF, 0), ("A_4.5dB", "A", 4.5, 30, 0xFF, 0), ("A_4.5dB_fixpoint", "A", 4.5, 30, 0xFF, 1),
             ("W_-2dB", "W", -2.0, 30, 0xFF, 0), ("W_2dB", "W", 2.0, 30, 0xFF, 0), ("R_50it", "R", 2.0, 50, 0x3F, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import fixedpointldpc_amd as F
    from oracle import oracle as O
    codes = {"A": F.Code.array(47, 5), "W": F.Code.wifi_1944_r12(), "R": F.Code.array(47, 24)}
    cli = os.path.join(ROOT, "fixedpointldpc_amd", "fpldpc_perftest")
    with tempfile.TemporaryDirectory() as d:
        for name, key, eb, max_iter, mask, fix in WORKLOADS:
            if args.only and args.only not in name:
                continue
            code = codes[key]
            alist = os.path.join(d, key + ".alist")
            with open(alist, "w") as f:
                f.write(code.write_alist())
            ocode = O.OracleCode.from_alist_text(code.write_alist())
            nf = args.frames if key != "R" else max(20, args.frames // 5)
            rate = 0.5 if key == "W" else code.rate
            snr = 2 * math.pow(10.0, eb / 10) * rate
            llr = O.gen_llr(123456789, 0, nf, code.n, snr, math.sqrt(1 / snr), 4)
            path = os.path.join(d, name + ".llr")
            llr.astype("<i4").tofile(path)
            p = subprocess.run([cli, "frame_time", alist, path, str(fix), str(max_iter), hex(mask)], capture_output=True,
                               text=True, timeout=600)
            if p.returncode:
                raise SystemExit(p.stderr)
            gpu = json.loads(p.stdout.strip().splitlines()[-1])
            t0 = time.perf_counter()
            ref = O.decode_batch(ocode, llr, max_iter=max_iter, mask=mask, precheck=bool(fix), nthreads=1, want_post=True)
            cpu_s = time.perf_counter() - t0
            assert int(ref["iters"].sum()) == gpu["iterations"], (name, int(ref["iters"].sum()), gpu["iterations"])
            rec = {"workload": name, "code": key, "ebn0_db": eb, "max_iter": max_iter, "mask": hex(mask),
                   "call": "decode_fixpoint" if fix else "decode_general_fp", "frames": nf,
                   "mean_iters": gpu["iterations"] / nf, "gpu_us_per_frame": gpu["us_mean"],
                   "gpu_us_median": gpu["us_median"], "gpu_us_min": gpu["us_min"], "gpu_us_max": gpu["us_max"],
                   "cpu_port_us_per_frame_1core": cpu_s / nf * 1e6, "gpu_vs_cpu_1core": cpu_s / nf * 1e6 / gpu["us_mean"]}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
