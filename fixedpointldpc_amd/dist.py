"""Multi-GPU bookkeeping for the decode path: one process per GPU, torch.distributed (RCCL over
xGMI on the GPU box, gloo in the CPU tests).

Codewords are independent, so the data path has no collective: rank r decodes the contiguous frame
range [first + r*F, first + (r+1)*F) of the reference's single RNG stream (skip-ahead to draw
frame*n, rngs.cpp:52-69), which makes every per-frame result independent of the rank count.  The
collectives are
  * one all-reduce of the four int64 counters {bit errors, frame errors, frames, iteration sum}
    (and a MAX of the elapsed time) at the end of a run -- 32 B, latency-bound;
  * for the harness's ordered stop rule ("stop at the frame that brings the frame-error count to
    N", PerfTest.cpp:97): one all-gather of the per-rank totals, a prefix scan on every rank, and a
    broadcast of the stop frame's counters from the rank that holds it.
"""
import numpy as np
import torch
import torch.distributed as dist


def frame_range(rank, world, frames_per_rank, first_frame=0):
    """[lo, hi) frames of this rank (weak scaling: frames_per_rank fixed as world grows)."""
    lo = first_frame + rank * frames_per_rank
    return lo, lo + frames_per_rank


def allreduce_counters(totals, elapsed_s, device=None):
    """Sum the int64[4] counters over ranks and take the max elapsed time.  Returns (list, float)."""
    t = torch.as_tensor(totals, dtype=torch.int64, device=device).clone()
    e = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    if dist.is_initialized():  # at one rank too: a 1-rank RCCL group runs the same collective
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return [int(x) for x in t.cpu().tolist()], float(e.item())


def any_rank(flag, device=None):
    """True on every rank if `flag` is true on any rank (MAX all-reduce of one int64), so that an
    error seen by one rank ends the run on all of them instead of leaving the others blocked in
    their next collective."""
    t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item())


def ordered_stop(blk, max_frame_errors, device=None):
    """The reference's serial stop rule over frames sharded in rank order.

    blk: this rank's per-frame error counts (int, in frame order).  Returns the global
    (bit_errors, frame_errors, frames) up to and including the frame at which the frame-error count
    reaches max_frame_errors, or the totals over all frames if it is never reached, and a flag."""
    blk = np.asarray(blk, np.int64)
    local = torch.tensor([int(blk.sum()), int((blk > 0).sum()), len(blk)], dtype=torch.int64, device=device)
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if world > 1:
        parts = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(parts, local)
    else:
        parts = [local]
    tot = np.array([p.cpu().tolist() for p in parts], np.int64)  # [world][3]
    cum_fe = np.cumsum(tot[:, 1])
    hit = np.nonzero(cum_fe >= max_frame_errors)[0]
    if hit.size == 0:
        s = tot.sum(axis=0)
        return (int(s[0]), int(s[1]), int(s[2])), False
    j = int(hit[0])
    before = tot[:j].sum(axis=0) if j else np.zeros(3, np.int64)
    res = torch.zeros(3, dtype=torch.int64, device=device)
    if rank == j:
        need = max_frame_errors - int(before[1])
        fe = np.cumsum(blk > 0)
        stop = int(np.nonzero(fe >= need)[0][0])  # index of the stopping frame within this rank
        res = torch.tensor([int(before[0]) + int(blk[:stop + 1].sum()), max_frame_errors,
                            int(before[2]) + stop + 1], dtype=torch.int64, device=device)
    if world > 1:
        dist.broadcast(res, src=j)
    r = res.cpu().tolist()
    return (int(r[0]), int(r[1]), int(r[2])), True
