#!/usr/bin/env python3
"""Throughput of the frame-generation kernels on either side of the decoder (fpldpc_gen.hip):
the device channel (Lehmer skip-ahead + Odeh-Evans + quantisation) and the batched encoder, plus
the host channel for comparison.  Prints one JSON line per measurement.

usage: python tools/bench_gen.py [--frames 65536]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=65536)
    args = ap.parse_args()
    import torch
    import fixedpointldpc_amd as F
    dev = torch.device("cuda", 0)
    B = args.frames
    for key, code in (("A", F.Code.array(47, 5)), ("W", F.Code.wifi_1944_r12())):
        n = code.n
        snr, sigma = F.snr_sigma(2.0, 0.5)
        out = torch.empty((B, n), dtype=torch.int16, device=dev)
        ovf = torch.zeros(1, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        t = timed(lambda: F.channel_llr_ptrs(123456789, 0, B, n, snr, sigma, 4, 0, 0, out.data_ptr(), F.FPLDPC_LLR_I16,
                                             ovf.data_ptr(), s))
        print(json.dumps({"kernel": "channel_kernel", "code": key, "frames": B, "seconds": t,
                          "Gllr_per_s": round(B * n / t / 1e9, 3), "write_GB_per_s": round(B * n * 2 / t / 1e9, 1)}))
        nh = min(B, 8192)
        t0 = time.perf_counter()
        F.channel_llr(123456789, 0, nh, n, snr, sigma, 4, None, np.int16, nthreads=16)
        th = time.perf_counter() - t0
        print(json.dumps({"kernel": "host channel (16 threads)", "code": key, "frames": nh, "seconds": th,
                          "Gllr_per_s": round(nh * n / th / 1e9, 4)}))
        enc = F.Encoder.from_code(code)
        info = torch.randint(0, 2, (B, enc.k), dtype=torch.uint8, device=dev)
        cw = torch.empty((B, n), dtype=torch.uint8, device=dev)
        enc.encode_ptrs(info.data_ptr(), B, cw.data_ptr(), s)
        t = timed(lambda: enc.encode_ptrs(info.data_ptr(), B, cw.data_ptr(), s))
        print(json.dumps({"kernel": "pack_info_kernel + encode_kernel", "code": key, "frames": B, "seconds": t,
                          "Mframes_per_s": round(B / t / 1e6, 3), "coded_Gb_per_s": round(B * n / t / 1e9, 2),
                          "hbm_GB_per_s_min": round(B * (enc.k + n) / t / 1e9, 1)}))


if __name__ == "__main__":
    main()
