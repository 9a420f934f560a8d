#!/usr/bin/env python3
"""Calibrate the CPU baseline (bench.py cpu_baseline, "kind": "port") against the reference.

BASELINE.md / SURVEY §8(d): the oracle's C restatement of decode_general_fp must run within +-15%
of the reference's own decoder per core, and bit-exactly, so the baseline is neither a straw man
nor a secret speed-up.  Runs in the build container only (it needs the reference builds
oracle/_ref/ref_{wifi,a47r5,a47r24}: the reference's ArrayLDPC_Decoder.cpp compiled unmodified,
-O2, with the dimension enums of each config, oracle/Makefile).

For each config, on the same core (taskset to one CPU), the same frames (all-iteration Eb/N0, so
the work is deterministic) are decoded by
  reference: ref_<dims> decode <alist> llr.bin  (setState(PCV) + decode_general_fp per frame,
             plus getPost_fp / DecodedCodeword out to a file; the I/O is < 1% of the time)
  port:      oracle.decode_batch(..., nthreads=1)  (fpldpc_oracle.c, gcc -O2)
and the outputs are compared.  Writes profiles/<round>/cpu_calibration.json.
"""
import json
import math
import os
import platform
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = "/root/reference"
SEED = 123456789

CONFIGS = {  # config: (ref binary, alist, max_iter, mask, Eb/N0, rate, frames)
    "A": ("ref_a47r5", "H_array_p47_r5_forward.txt", 30, 0xFF, 0.0, 1 - (5 * 47 - 5 + 1) / 47 ** 2, 300),
    "W": ("ref_wifi", "H_802.11_IndZero.txt", 30, 0xFF, -2.0, 0.5, 400),
    "R": ("ref_a47r24", "codes/H_array_p47_r24_forward.txt", 50, 0x3F, 2.0, 1 - (24 * 47 - 24 + 1) / 47 ** 2, 40),
}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    from oracle import oracle as O
    O.build(ref=True)
    cpu = sorted(os.sched_getaffinity(0))[-1]
    os.sched_setaffinity(0, {cpu})
    reps = 9
    out = {"host_cpu": cpu_model(), "core": cpu, "reps": reps, "configs": {}}
    for cfg, (binary, alist, max_iter, mask, eb, rate, nf) in CONFIGS.items():
        path = os.path.join(REF, alist)
        ocode = O.OracleCode.from_alist(path)
        e = int(ocode._cdeg.sum())
        snr = 2 * math.pow(10.0, eb / 10) * rate
        llr = O.gen_llr(SEED, 0, nf, ocode.n, snr, math.sqrt(1 / snr), 4, nthreads=1)
        t_ref, t_port = [], []
        with tempfile.TemporaryDirectory() as td:
            lp, op = os.path.join(td, "l.bin"), os.path.join(td, "o.bin")
            llr.astype(np.int32).tofile(lp)
            for _ in range(reps):  # interleaved, so a load change on the host hits both alike
                t = time.perf_counter()
                subprocess.run(["taskset", "-c", str(cpu), os.path.join(ROOT, "oracle", "_ref", binary), "decode", path,
                                lp, str(nf), op], check=True)
                t_ref.append(time.perf_counter() - t)
                t = time.perf_counter()
                r = O.decode_batch(ocode, llr, max_iter=max_iter, mask=mask, nthreads=1)
                t_port.append(time.perf_counter() - t)
            rec = np.fromfile(op, np.int32).reshape(nf, 2 * ocode.n + 1)
        exact = bool((rec[:, 0] == r["iters"]).all() and (rec[:, 1:ocode.n + 1] == r["post"]).all())
        iters = int(r["iters"].sum())
        ns_ref = min(t_ref) / (iters * e) * 1e9
        ns_port = min(t_port) / (iters * e) * 1e9
        k = {"A": 1978, "W": 972, "R": 1104}[cfg]
        out["configs"][cfg] = {
            "frames": nf, "edges": e, "iterations_total": iters, "bit_exact": exact,
            "reference_s": [round(x, 4) for x in t_ref], "port_s": [round(x, 4) for x in t_port],
            "reference_ns_per_edge_iter": round(ns_ref, 3), "port_ns_per_edge_iter": round(ns_port, 3),
            "port_over_reference_time": round(ns_port / ns_ref, 4),
            # the same, as the median of the per-rep (interleaved, paired) ratios: robust to host load
            "port_over_reference_time_median_paired": round(float(np.median(np.array(t_port) / np.array(t_ref))), 4),
            "reference_info_mbps": round(nf * k / min(t_ref) / 1e6, 4),
            "port_info_mbps": round(nf * k / min(t_port) / 1e6, 4),
            "within_15pct": abs(ns_port / ns_ref - 1) <= 0.15,
            "reference_s_spread": round(max(t_ref) / min(t_ref), 3),
        }
        print(cfg, json.dumps(out["configs"][cfg]), flush=True)
    dst = os.path.join(ROOT, "profiles", sys.argv[1] if len(sys.argv) > 1 else "r2", "cpu_calibration.json")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main()
