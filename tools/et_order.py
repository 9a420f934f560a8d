#!/usr/bin/env python3
"""Diagnostic (early-termination tail): decode time of one 4096-frame A batch at 4.5 dB in three frame
orders -- the channel stream's own, longest-first and longest-last by the oracle's iteration counts --
to see how much of the launch is the tail of long frames that start late.  Also the WG trace of each
(FPLDPC_WG_TRACE) when --trace DIR is given.

usage: tools/et_order.py [--ebn0 4.5] [--frames 4096] [--config A|W] [--trace DIR]"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ebn0", type=float, default=4.5)
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--config", default="A")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--trace", default=None, help="directory: one FPLDPC_WG_TRACE launch per order (wg_trace.py)")
    args = ap.parse_args()
    import torch
    import fixedpointldpc_amd as F
    from oracle import oracle as O
    code = F.Code.array(47, 5) if args.config == "A" else F.Code.wifi_1944_r12()
    rate = code.rate if args.config == "A" else 0.5
    snr, sigma = F.snr_sigma(args.ebn0, rate)
    llr = F.channel_llr(123456789, 0, args.frames, code.n, snr, sigma, 4, None, np.int16, nthreads=16)
    it = O.decode_batch(O.OracleCode.from_alist_text(code.write_alist()), llr, want_post=False, nthreads=16)["iters"]
    dev = torch.device("cuda:0")
    dec = F.Decoder(code)
    hist = np.bincount(it, minlength=31)
    out = {"config": args.config, "ebn0": args.ebn0, "frames": args.frames, "avg_iters": float(it.mean()),
           "iters_hist": hist.tolist(), "orders": {}}
    k = code.n - code.rank
    for name, order in (("stream", np.arange(args.frames)), ("longest_first", np.argsort(-it, kind="stable")),
                        ("longest_last", np.argsort(it, kind="stable"))):
        x = torch.from_numpy(np.ascontiguousarray(llr[order])).to(dev)
        iters = torch.empty(args.frames, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream(dev)
        for _ in range(5):
            dec.decode_ptrs(x.data_ptr(), F.FPLDPC_LLR_I16, args.frames, 0, iters.data_ptr(), 0, 0, 0, 0, s.cuda_stream)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record(s)
            dec.decode_ptrs(x.data_ptr(), F.FPLDPC_LLR_I16, args.frames, 0, iters.data_ptr(), 0, 0, 0, 0, s.cuda_stream)
            b.record(s)
        torch.cuda.synchronize()
        ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        ok = bool((iters.cpu().numpy() == it[order]).all())
        out["orders"][name] = {"launch_ms": round(ms, 4), "mbps": round(args.frames * k / ms / 1e3, 1), "parity": ok}
        print(name, out["orders"][name], flush=True)
        if args.trace:  # one traced launch (the trace is read at decoder creation, written after each call)
            os.makedirs(args.trace, exist_ok=True)
            os.environ["FPLDPC_WG_TRACE"] = os.path.join(args.trace, f"{args.config}_{name}.bin")
            tdec = F.Decoder(code)
            del os.environ["FPLDPC_WG_TRACE"]
            tdec.decode_ptrs(x.data_ptr(), F.FPLDPC_LLR_I16, args.frames, 0, iters.data_ptr(), 0, 0, 0, 0, s.cuda_stream)
            torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
