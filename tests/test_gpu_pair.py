"""fpldpc_decode_pair / _pair_host (fixedpointldpc_amd/csrc/fpldpc_pair.cpp): one batch as two launches
in flight on two decoders of the same code.  The same frames through the same kernels, so every output
must equal fpldpc_decode's on the whole batch (iterations, hard decisions, syndrome verdicts,
posteriors, bit errors, totals) -- and the early-termination tail of a single launch is filled."""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
SEED = 123456789


def _batch(O, code, cfg, eb, frames, skip):
    g = np.load(os.path.join(GOLDEN, "kat_w.npz" if cfg == "W" else "kat_a.npz"))
    rate = 0.5 if cfg == "W" else code.rate
    snr = 2 * math.pow(10.0, eb / 10) * rate
    cw = g["cw"] if cfg != "R" else None
    return O.gen_llr(SEED, skip, frames, code.n, snr, math.sqrt(1 / snr), 4, cw=cw).astype(np.int16)


@pytest.mark.parametrize("cfg,eb,frames", [("A", 4.5, 4096), ("W", 2.0, 2047), ("R", 6.5, 1024), ("A", 0.0, 3)])
def test_pair_equals_single(F, O, codes, torch_dev, cfg, eb, frames):
    import torch
    code, _ = codes[cfg]
    kw = dict(max_iter=50, width_mask=0x3F) if cfg == "R" else {}
    a, b = F.Decoder(code, **kw), F.Decoder(code, **kw)
    k = code.n - code.rank
    rs = np.random.default_rng(3)
    idx = np.sort(rs.choice(code.n, size=k, replace=False)).astype(np.int32)
    bits = rs.integers(0, 2, size=k).astype(np.uint8)
    for d in (a, b):
        d.set_reference(idx, bits)
    llr = torch.from_numpy(_batch(O, code, cfg, eb, frames, 40000)).to(torch_dev)
    t1 = torch.tensor([5, 6, 7, 8], dtype=torch.int64, device=torch_dev)
    t2 = t1.clone()
    one = a.decode_torch(llr, post=True, bit_errors=True, totals=t1)
    two = a.decode_pair_torch(b, llr, post=True, bit_errors=True, totals=t2)
    torch.cuda.synchronize()
    for key in one:
        assert torch.equal(one[key], two[key]), key
    assert t1.tolist() == t2.tolist()


def test_pair_host_equals_single(F, O, codes):
    """Host buffers, incl. decode_fixpoint's pre-check passes (posteriors seeded from the caller's
    buffer and left in place) and totals accumulated into the caller's values."""
    code, _ = codes["A"]
    a, b = F.Decoder(code, precheck=True), F.Decoder(code, precheck=True)
    llr = _batch(O, code, "A", 4.5, 301, 50000)
    snr = 2 * math.pow(10.0, 4.5 / 10) * code.rate
    llr[1::5] = int(2 * snr * 16)  # noiseless frames: the pre-check passes
    seed_post = np.random.default_rng(9).integers(-500, 500, (len(llr), code.n)).astype(np.int32)
    one = a.decode_host(llr, post=seed_post.copy(), totals=np.array([1, 2, 3, 4], np.int64))
    two = a.decode_pair_host(b, llr, post=seed_post.copy(), totals=np.array([1, 2, 3, 4], np.int64))
    for key in one:
        assert (one[key] == two[key]).all(), key
    assert (one["iters"][1::5] == 0).all() and (two["post"][1::5] == seed_post[1::5]).all()


def test_pair_fills_the_tail(F, O, codes, torch_dev):
    """A @ 4.5 dB, 4096 frames: a single launch waits on late 30-iteration frames; two launches in
    flight take the CUs it leaves idle (16.3 vs 28.3 Gb/s as separate calls)."""
    import torch
    code, _ = codes["A"]
    a, b = F.Decoder(code), F.Decoder(code)
    llr = torch.from_numpy(_batch(O, code, "A", 4.5, 4096, 60000)).to(torch_dev)

    def timed(fn, reps=20):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    t1 = timed(lambda: a.decode_torch(llr))
    t2 = timed(lambda: a.decode_pair_torch(b, llr))
    print(f"A @ 4.5 dB, 4096 frames: one launch {t1:.3f} ms, two in flight {t2:.3f} ms ({t1 / t2:.2f}x)")
    assert t2 < 0.85 * t1


def test_pair_argument_errors(F, codes, torch_dev):
    import torch
    a = F.Decoder(codes["A"][0])
    w = F.Decoder(codes["W"][0])
    llr = torch.zeros((4, a.code.n), dtype=torch.int16, device=torch_dev)
    with pytest.raises(Exception, match="distinct"):
        a.decode_pair_torch(a, llr)
    with pytest.raises(Exception, match="different codes"):
        a.decode_pair_torch(w, llr)
    r = F.Decoder(codes["A"][0], max_iter=20)
    with pytest.raises(Exception, match="different parameters"):
        a.decode_pair_torch(r, llr)
