#!/usr/bin/env python3
"""Multi-GPU BER/FER simulation with the reference harness's stop rule (fixedpointldpc_amd/sim_dist.py).

  python tools/ber_dist.py                       # KAT-W: ArrayLDPC_Debug_Wifi at 2 dB, one GPU
  torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/ber_dist.py [--backend gloo]

Rank 0 prints one JSON line: bit errors, frame errors, frames (equal for every N), seconds.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["W", "A"], default="W")
    ap.add_argument("--ebn0", type=float, default=None)
    ap.add_argument("--max-frame-errors", type=int, default=100)
    ap.add_argument("--max-frames", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import fixedpointldpc_amd as F
    from fixedpointldpc_amd.sim_dist import ber_sim_sharded

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    golden = os.path.join(ROOT, "tests", "golden")
    if args.config == "W":  # ArrayLDPC_Debug_Wifi (PerfTest.cpp:23-140): rate hard-coded 0.5
        g = np.load(os.path.join(golden, "kat_w.npz"))
        code, dec_kw, eb = F.Code.wifi_1944_r12(), {}, 2.0 if args.ebn0 is None else args.ebn0
        rate = 0.5
    else:  # ArrayLDPC_Debug (:217-316): decode_fixpoint, getRate()
        g = np.load(os.path.join(golden, "kat_a.npz"))
        code, dec_kw, eb = F.Code.array(47, 5), {"precheck": True}, 4.5 if args.ebn0 is None else args.ebn0
        rate = code.rate
    snr = 2 * math.pow(10.0, eb / 10) * rate
    dec = F.Decoder(code, device=local, **dec_kw)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    r = ber_sim_sharded(dec, snr, math.sqrt(1 / snr), g["info_idx"], g["info_bits"], g["cw"],
                        max_frame_errors=args.max_frame_errors, max_frames=args.max_frames, chunk=args.chunk,
                        device=dev)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if (dist.get_rank() if world > 1 else 0) == 0:
        r.update({"config": args.config, "ebn0_db": eb, "ranks": world, "seconds": round(dt, 4),
                  "FER": r["frame_errors"] / r["frames"], "BER": r["bit_errors"] / r["frames"] / code.n})
        print(json.dumps(r), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
