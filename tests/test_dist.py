"""Multi-rank bookkeeping (fixedpointldpc_amd/dist.py) on CPU with gloo, world size 2 (and 3):
sharded frame ranges + all-reduce / ordered stop == the single-process serial loop.  The per-frame
decode here is the CPU oracle (the GPU path is exercised by the -m gpu tests); what is under test is
the partitioning and the collectives."""
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT

SEED = 123456789


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frames_blk(f0, nfr):
    import sys
    sys.path.insert(0, ROOT)
    import fixedpointldpc_amd as F
    from oracle import oracle as O
    kw = np.load(os.path.join(GOLDEN, "kat_w.npz"))
    code = F.Code.wifi_1944_r12()
    oc = O.OracleCode.from_alist_text(code.write_alist())
    snr = 2 * math.pow(10.0, 1.0 / 10) * 0.5
    llr = O.gen_llr(SEED, f0, nfr, 1944, snr, math.sqrt(1 / snr), 4, cw=kw["cw"], nthreads=2)
    r = O.decode_batch(oc, llr, want_post=False, nthreads=2)
    blk = (r["hard"][:, kw["info_idx"]] != kw["info_bits"][None, :]).sum(axis=1)
    return blk, r["iters"]


def _worker(rank, world, port, per_rank, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from fixedpointldpc_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = D.frame_range(rank, world, per_rank)
    blk, it = _frames_blk(lo, hi - lo)
    totals = [int(blk.sum()), int((blk > 0).sum()), len(blk), int(it.sum())]
    red, el = D.allreduce_counters(totals, 0.5 + rank)
    stop, hit = D.ordered_stop(blk, 7)
    # an error flag raised on one rank only reaches every rank (sim_dist: all fail, none hangs)
    anys = (D.any_rank(rank == world - 1), D.any_rank(False))
    q.put((rank, red, el, stop, hit, anys))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_serial(world):
    per_rank = 120
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, per_rank, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    blk, it = _frames_blk(0, world * per_rank)
    want_tot = [int(blk.sum()), int((blk > 0).sum()), len(blk), int(it.sum())]
    fe = np.cumsum(blk > 0)
    s = int(np.nonzero(fe >= 7)[0][0])
    want_stop = (int(blk[:s + 1].sum()), 7, s + 1)
    assert (blk > 0).sum() >= 7, "test SNR must produce enough frame errors"
    for rank, red, el, stop, hit, anys in res:
        assert anys == (True, False)
        assert red == want_tot
        assert el == 0.5 + world - 1
        assert hit and stop == want_stop
