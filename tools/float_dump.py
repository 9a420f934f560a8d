#!/usr/bin/env python3
"""Float decoder outputs (iterations, hard decisions, posteriors) on fixed AWGN frames of A and W, saved
to an npz: run once per library build (FPLDPC_LIB_PATH) and compare the files bit for bit
(tools/gpu_float_exact.sh).  usage: tools/float_dump.py OUT.npz"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    import torch
    import fixedpointldpc_amd as F
    res = {}
    for key, code, eb, B in (("A", F.Code.array(47, 5), 3.5, 1024), ("W", F.Code.wifi_1944_r12(), 1.5, 1024)):
        snr = 2 * math.pow(10.0, eb / 10) * code.rate
        rng = np.random.default_rng(7)
        llr = 2 * snr * (1.0 + rng.normal(0.0, math.sqrt(1 / snr), size=(B, code.n)))
        dec = F.Decoder(code)
        o = dec.decode_float_torch(torch.from_numpy(llr).to("cuda:0"), post=True)
        for k, v in o.items():
            res[f"{key}_{k}"] = v.cpu().numpy()
    np.savez(out, **res)
    print(out, {k: v.shape for k, v in res.items()})


if __name__ == "__main__":
    main(sys.argv[1])
