#!/usr/bin/env python3
"""Debug: the lock-step kernel against the default one on the same 40 A frames (posteriors, hard
decisions, iterations) -- which outputs differ and where."""
import math, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import fixedpointldpc_amd as F
from oracle import oracle as O
code = F.Code.array(47, 5)
snr = 2 * math.pow(10.0, 3.0 / 10) * code.rate
llr = O.gen_llr(123456789, 4242, 40, code.n, snr, math.sqrt(1 / snr), 4)
t = torch.from_numpy(llr).to("cuda:0")
out = {}
for name in ("flood_array2<P=47,W=3>", "flood_lock<P=47,S=3>"):
    os.environ["FPLDPC_KERNEL"] = name
    dec = F.Decoder(code)
    print(name, dec.describe())
    out[name] = {k: v.cpu().numpy() for k, v in dec.decode_torch(t, post=True).items()}
a, b = out.values()
print("iters equal", (a["iters"] == b["iters"]).all(), a["iters"][:12], b["iters"][:12])
for f in range(8):
    dp = np.nonzero(a["post"][f] != b["post"][f])[0]
    hw = np.nonzero(a["hard"][f] != b["hard"][f])[0]
    print(f, "post diffs", dp.size, dp[:6], "hard word diffs", hw[:10], "ok", a["syndrome_ok"][f], b["syndrome_ok"][f])
    if hw.size:
        w = hw[0]; print("   words", hex(a["hard"][f][w]), hex(b["hard"][f][w]))
