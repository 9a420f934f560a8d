"""The reference harness's frame loop (PerfTest.cpp:97-135: decode frames until the frame that
brings the frame-error count to N) sharded over ranks, one process per GPU.

Each round, rank r generates and decodes frames [base + r*C, base + (r+1)*C) entirely on its GPU
(device channel, skip-ahead to draw frame*n; decoder; per-frame bit errors), then the ranks combine
their per-rank counts in rank order (fixedpointldpc_amd/dist.py: all-gather of 3 int64 per rank,
prefix scan, broadcast of the stopping rank's partial sums).  The result -- bit errors, frame
errors, frames up to and including the stopping frame -- equals the serial loop's for any number of
ranks, e.g. the published KAT-W 2732 / 100 / 393214.  The only collectives are those per-round
exchanges of a few int64 (RCCL over xGMI on the GPU box, gloo in the tests).
"""
import numpy as np
import torch

from . import dist as D
from ._lib import channel_llr_torch


def ber_sim_sharded(dec, snr, sigma, info_index, info_bits, codeword=None, seed=123456789, max_frame_errors=100,
                    max_frames=0, chunk=65536, device=None, frac_bits=4):
    """Returns dict(bit_errors, frame_errors, frames, rounds).  `dec` is this rank's
    fixedpointldpc_amd.Decoder (on `device`); codeword: uint8 [n] (None = all-zero)."""
    device = torch.device(device if device is not None else "cuda")
    world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
    dev_cw = None if codeword is None else torch.from_numpy(np.ascontiguousarray(codeword, np.uint8)).to(device)
    dec.set_reference(np.asarray(info_index, np.int32), np.asarray(info_bits, np.uint8))
    coll_dev = device if torch.distributed.is_initialized() and torch.distributed.get_backend() == "nccl" else None
    n = dec.code.n
    base, be, fe, fr, rounds = 0, 0, 0, 0, 0
    while True:
        C = chunk if not max_frames else min(chunk, -(-(max_frames - fr) // world))
        lo = base + rank * C
        llr, ovf = channel_llr_torch(seed, lo, C, n, snr, sigma, frac_bits, dev_cw, torch.int16, device)
        out = dec.decode_torch(llr, bit_errors=True)
        blk = out["bit_errors"].cpu().numpy().astype(np.int64)
        if D.any_rank(int(ovf.item()), device=coll_dev):  # every rank fails together, none hangs
            raise RuntimeError("LLR outside int16 on at least one rank")
        if max_frames:  # frames past the global limit do not count
            blk = blk[:max(0, min(C, max_frames - fr - rank * C))]
        (b, f, m), hit = D.ordered_stop(blk, max_frame_errors - fe if max_frame_errors else 1 << 62, device=coll_dev)
        be, fe, fr, rounds = be + b, fe + f, fr + m, rounds + 1
        base += world * C
        if hit or (max_frames and fr >= max_frames):
            return {"bit_errors": be, "frame_errors": fe, "frames": fr, "rounds": rounds}
