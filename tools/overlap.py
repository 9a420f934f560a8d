#!/usr/bin/env python3
"""Diagnostic: consecutive A batches on one stream (the bench's step) against the same batches
alternating over two decoders on two streams, so that one launch's tail (the youngest workgroup of
each CU finishing its last frame pair alone) overlaps the next launch's start."""
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import fixedpointldpc_amd as F
    dev = torch.device("cuda:0")
    code = F.Code.array(47, 5)
    snr, sigma = F.snr_sigma(0.0, code.rate)
    B, K = 4096, 60
    llr = torch.from_numpy(F.channel_llr(123456789, 0, B, code.n, snr, sigma, 4, None, np.int16, nthreads=16)).to(dev)
    k = code.n - code.rank
    for nstreams in (1, 2, 3, 1, 2, 3):
        decs = [F.Decoder(code) for _ in range(nstreams)]
        streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
        iters = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(nstreams)]
        def run(n):
            for i in range(n):
                j = i % nstreams
                decs[j].decode_ptrs(llr.data_ptr(), F.FPLDPC_LLR_I16, B, 0, iters[j].data_ptr(), 0, 0, 0, 0,
                                    streams[j].cuda_stream)
        run(20)
        torch.cuda.synchronize()
        t = time.perf_counter()
        run(K)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        ok = all(bool((it == 30).all()) for it in iters)
        print(f"streams {nstreams}: {K} batches in {dt * 1e3:.2f} ms = {B * K * k / dt / 1e6:.1f} Mb/s, "
              f"{dt / K * 1e3:.4f} ms per batch, iterations ok {ok}", flush=True)


if __name__ == "__main__":
    main()
