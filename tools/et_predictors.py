#!/usr/bin/env python3
"""CPU analysis (oracle only): how well cheap, decode-free difficulty scores find the frames that
need many iterations at the early-termination points (A @ 4.5 dB, W @ 2 dB, 4096 frames of the
reference channel stream) -- the frames whose late start makes a launch's tail.

usage: tools/et_predictors.py > profiles/r3/et/predictors.txt"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import fixedpointldpc_amd as F
    from oracle import oracle as O
    for cfg, eb in (("A", 4.5), ("W", 2.0)):
        code = F.Code.array(47, 5) if cfg == "A" else F.Code.wifi_1944_r12()
        snr, sigma = F.snr_sigma(eb, code.rate if cfg == "A" else 0.5)
        llr = F.channel_llr(123456789, 0, 4096, code.n, snr, sigma, 4, None, np.int16, nthreads=8)
        it = O.decode_batch(O.OracleCode.from_alist_text(code.write_alist()), llr, want_post=False, nthreads=8)["iters"]
        toks = list(map(int, code.write_alist().split()))
        n, m = toks[0], toks[1]
        p = 4
        vdeg = toks[p:p + n]
        p += n
        cdeg = toks[p:p + m]
        p += m + sum(vdeg)
        hard = (llr <= 0).astype(np.int64)
        syn = np.zeros(len(llr), np.int64)
        for d in cdeg:
            syn += hard[:, toks[p:p + d]].sum(axis=1) & 1
            p += d
        a = np.abs(llr.astype(np.int64))
        med = float(np.median(a))
        long = it >= 20
        print(f"{cfg} @ {eb} dB: 4096 frames, mean iterations {it.mean():.3f}, {int(long.sum())} need >= 20, "
              f"{int((it >= 30).sum())} run 30")
        scores = [("channel syndrome weight", syn)]
        for fr in (0.125, 0.25, 0.5):
            scores.append((f"count of |LLR| < {med * fr:.0f}", (a < med * fr).sum(axis=1)))
        scores.append(("-sum |LLR|", -a.sum(axis=1)))
        for name, sc in scores:
            order = np.argsort(-sc, kind="stable")
            print(f"  {name:28s}: long frames in its top 10 % {int(long[order[:410]].sum()):4d}, "
                  f"top 25 % {int(long[order[:1024]].sum()):4d}; corr with iterations {np.corrcoef(sc, it)[0, 1]:.3f}")


if __name__ == "__main__":
    main()
