# Debug: W packed kernel vs int32 kernel at scale, per frame.
import math, os, sys
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
import fixedpointldpc_amd as F
code = F.Code.wifi_1944_r12()
kw = np.load("tests/golden/kat_w.npz")
snr = 2 * math.pow(10.0, 2.0 / 10) * 0.5
sig = math.sqrt(1 / snr)
dev = torch.device("cuda:0")
for cw_name, cw in (("zero", None), ("kat", kw["cw"])):
    for B in (64, 600, 4096):
        llr = F.channel_llr(123456789, 0, B, 1944, snr, sig, 4, cw=cw, dtype=np.int16)
        t = torch.from_numpy(llr).to(dev)
        outs = {}
        for k in ("flood_tab2", "flood_reg<DC=8,CPL=4>"):
            os.environ["FPLDPC_KERNEL"] = k
            d = F.Decoder(code)
            o = d.decode_torch(t, post=True)
            torch.cuda.synchronize()
            outs[k] = {kk: v.cpu().numpy() for kk, v in o.items()}
        a, b = outs["flood_tab2"], outs["flood_reg<DC=8,CPL=4>"]
        bad = np.nonzero((a["iters"] != b["iters"]) | (a["hard"] != b["hard"]).any(1) | (a["post"] != b["post"]).any(1))[0]
        print(cw_name, B, "mismatch frames:", len(bad), bad[:10], "iters tab", a["iters"][bad[:10]], "ref", b["iters"][bad[:10]], flush=True)
