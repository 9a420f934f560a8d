#!/usr/bin/env python3
"""fpldpc_ber_sim with one chunk in flight (FPLDPC_SIM_OVERLAP=0) against two (the default): the
published KAT-W run (802.11n, 2 dB, stop at 100 frame errors: 393,214 frames) and A at 4.5 dB
(decode_fixpoint, a fixed 262,144 frames), device channel, several chunk sizes.  Prints one JSON
line per run; the counters of both modes must agree."""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import fixedpointldpc_amd as F
    g = os.path.join(ROOT, "tests", "golden")
    kw_w = np.load(os.path.join(g, "kat_w.npz"), allow_pickle=False)
    ka = np.load(os.path.join(g, "kat_a.npz"), allow_pickle=False)
    snr_w = 2 * math.pow(10.0, 2.0 / 10) * 0.5
    wdec = F.Decoder(F.Code.wifi_1944_r12())
    acode = F.Code.array(47, 5)
    adec = F.Decoder(acode, precheck=True)
    snr_a, sig_a = F.snr_sigma(4.5, acode.rate)
    cases = [
        ("KAT-W", wdec, dict(snr=snr_w, sigma=math.sqrt(1 / snr_w), info_index=kw_w["info_idx"], info_bits=kw_w["info_bits"],
                             codeword=kw_w["cw"], max_frame_errors=100), 1944 - 972),
        ("A@4.5dB", adec, dict(snr=snr_a, sigma=sig_a, info_index=ka["info_idx"], info_bits=ka["info_bits"], codeword=ka["cw"],
                               max_frame_errors=0, max_frames=262144), acode.n - acode.rank),
    ]
    for name, dec, kw, k in cases:
        for chunk in (4096, 16384):
            res = {}
            for ov in ("0", "1", "0", "1"):
                os.environ["FPLDPC_SIM_OVERLAP"] = ov
                r = dec.ber_sim(kw["snr"], kw["sigma"], device_channel=True, chunk=chunk,
                                **{a: b for a, b in kw.items() if a not in ("snr", "sigma")})
                res.setdefault(ov, []).append(r)
            same = all(res["0"][0][c] == res["1"][0][c] for c in ("bit_errors", "frame_errors", "frames", "iter_sum"))
            for ov, rs in res.items():
                t = min(r["seconds"] for r in rs)
                r = rs[0]
                print(json.dumps({"case": name, "chunk": chunk, "chunks_in_flight": 2 if ov == "1" else 1,
                                  "frames": r["frames"], "frames_decoded": r["frames_decoded"],
                                  "bit_errors": r["bit_errors"], "frame_errors": r["frame_errors"],
                                  "seconds_min_of_2": round(t, 4),
                                  "info_Mbps": round(r["frames_decoded"] * k / t / 1e6, 1), "counters_equal": same}),
                      flush=True)


if __name__ == "__main__":
    main()
