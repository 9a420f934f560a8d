"""GPU decode vs the CPU oracle, bit-exact (iterations, hard decisions, syndrome, posteriors).

Calls the product through its C ABI (fixedpointldpc_amd binds libfpldpc.so with ctypes); inputs
come from the oracle's restatement of the reference channel model (PerfTest.cpp:108-120).
"""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_same

pytestmark = pytest.mark.gpu

SEED = 123456789  # rngs.cpp:45 DEFAULT


def _rate(code):
    return code.rate


# (config, Eb/N0 points): waterfall points plus a forced-30-iteration point per code.
POINTS = [("A", [0.0, 4.0, 4.5, 5.0]), ("W", [-2.0, 1.5, 2.0]), ("R", [2.0, 5.0, 8.0])]


@pytest.mark.parametrize("cfg,snrs", POINTS)
def test_awgn_parity(F, O, codes, torch_dev, cfg, snrs):
    import torch
    code, ocode = codes[cfg]
    max_iter = 50 if cfg == "R" else 30
    mask = 0x3F if cfg == "R" else 0xFF
    dec = F.Decoder(code, max_iter=max_iter, width_mask=mask)
    B = 96
    for i, eb in enumerate(snrs):
        snr = 2 * math.pow(10.0, eb / 10) * code.rate
        sigma = math.sqrt(1 / snr)
        llr = O.gen_llr(SEED, 1000 * i, B, code.n, snr, sigma, 4)
        ref = O.decode_batch(ocode, llr, max_iter=max_iter, mask=mask)
        gpu = dec.decode_torch(torch.from_numpy(llr.astype(np.int16)).to(torch_dev), post=True)
        torch.cuda.synchronize()
        gpu = {k: v.cpu().numpy() for k, v in gpu.items()}
        assert_same(gpu, ref, code.n, where=f"{cfg}@{eb}dB [{dec.describe()}]")


@pytest.mark.parametrize("cfg", ["A", "W", "R"])
def test_random_llr_parity(F, O, codes, torch_dev, cfg):
    """Non-codeword inputs over the whole int16 range: exercises the WIDTH_MASK wrap of the
    masked sum/difference and the sgn(0) = -1 rule, and always runs to max_iter."""
    import torch
    code, ocode = codes[cfg]
    rng = np.random.default_rng(7)
    B = 64
    llr = np.concatenate([
        rng.integers(-300, 301, size=(B // 2, code.n)),
        rng.integers(-32768, 32768, size=(B // 4, code.n)),
        rng.integers(-3, 4, size=(B // 4, code.n)),  # many exact zeros
    ]).astype(np.int32)
    for mask in (0xFF, 0x3F):
        dec = F.Decoder(code, max_iter=12, width_mask=mask)
        ref = O.decode_batch(ocode, llr, max_iter=12, mask=mask)
        gpu = dec.decode_torch(torch.from_numpy(llr).to(torch_dev), post=True)
        torch.cuda.synchronize()
        assert_same({k: v.cpu().numpy() for k, v in gpu.items()}, ref, code.n, where=f"{cfg} mask={mask:#x}")


def _base(cfg):
    """The config's own iteration cap and WIDTH_MASK (R: 50 iterations, 0x3f, BASELINE configs[4])."""
    return dict(max_iter=50, width_mask=0x3F) if cfg == "R" else dict(max_iter=30, width_mask=0xFF)


PACKED = {"A": "flood_array2<P=47,W=3>", "W": "flood_tab2<DC=8,CPL=4,lo=3>", "R": "flood_array2<P=47,CPL=2,ldsoffs,mix>"}


@pytest.mark.parametrize("cfg", ["A", "W", "R"])
def test_precheck_and_modes(F, O, codes, torch_dev, cfg):
    """decode_fixpoint pre-check (noiseless frames -> 0 iterations, posteriors untouched,
    ArrayLDPC_Decoder.cpp:443-450), early_term off, and max_iter 1/2/7 -- on each config's packed
    kernel (R: the MixChecks kernel, whose two-lanes-per-check units run the pre-check too)."""
    import torch
    code, ocode = codes[cfg]
    base = _base(cfg)
    oit, omask = base["max_iter"], base["width_mask"]
    snr = 2 * math.pow(10.0, (4.0 if cfg != "R" else 6.5) / 10) * code.rate
    sigma = math.sqrt(1 / snr)
    llr = O.gen_llr(SEED, 77, 48, code.n, snr, sigma, 4)
    llr[::3] = 40  # noiseless all-zero codeword: channel decision already satisfies H
    t = torch.from_numpy(llr).to(torch_dev)
    dec = F.Decoder(code, precheck=True, **base)
    assert dec.describe().startswith(PACKED[cfg]), dec.describe()
    ref = O.decode_batch(ocode, llr, precheck=True, max_iter=oit, mask=omask)
    gpu = {k: v.cpu().numpy() for k, v in dec.decode_torch(t, post=True).items()}
    assert (ref["iters"][::3] == 0).all()
    assert_same(gpu, ref, code.n, check_post=False, where=f"{cfg} precheck")
    assert (gpu["post"][::3] == 0).all()  # untouched (zero-initialised by decode_torch)
    keep = np.ones(len(llr), bool)
    keep[::3] = False
    assert (gpu["post"][keep] == ref["post"][keep]).all()
    for kw in (dict(early_term=False), dict(max_iter=1), dict(max_iter=2), dict(max_iter=7)):
        dec = F.Decoder(code, **{**base, **kw})
        gpu = {k: v.cpu().numpy() for k, v in dec.decode_torch(t, post=True).items()}
        if "max_iter" in kw:
            ref = O.decode_batch(ocode, llr, max_iter=kw["max_iter"], mask=omask)
            assert_same(gpu, ref, code.n, where=f"{cfg} {kw}")
        else:  # every frame runs the cap; its flag is its final hard decision's syndrome
            assert (gpu["iters"] == oit).all()
            hard = F.unpack_hard(gpu["hard"], code.n)
            assert [code.syndrome_ok(h) for h in hard] == [bool(o) for o in gpu["syndrome_ok"]]


def test_batch_shapes_and_dtypes(F, O, codes, torch_dev):
    """batch 1, batch larger than the resident grid (persistent loop), int16 == int32 input."""
    import torch
    code, ocode = codes["W"]
    snr = 2 * math.pow(10.0, 2.0 / 10) * 0.5
    sigma = math.sqrt(1 / snr)
    llr = O.gen_llr(SEED, 5000, 3000, code.n, snr, sigma, 4)
    dec = F.Decoder(code)
    ref = O.decode_batch(ocode, llr[:1])
    g1 = {k: v.cpu().numpy() for k, v in dec.decode_torch(torch.from_numpy(llr[:1]).to(torch_dev), post=True).items()}
    assert_same(g1, ref, code.n, where="batch1")
    a = dec.decode_torch(torch.from_numpy(llr).to(torch_dev), post=True)
    b = dec.decode_torch(torch.from_numpy(llr.astype(np.int16)).to(torch_dev), post=True)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    sub = np.arange(0, 3000, 37)
    ref = O.decode_batch(ocode, llr[sub])
    assert_same({k: v.cpu().numpy()[sub] for k, v in a.items()}, ref, code.n, where="batch3000")


# Every kernel variant that can run each code, forced with FPLDPC_KERNEL (the default picks only one):
# the defaults, their fallback chains and the variants other codes default to.
VARIANTS = {
    "A": ["flood_array2<P=47,W=3>", "flood_array2<P=47,CPL=2>", "flood_array2<P=47,CPL=2,ldsoffs>", "flood_array<P=47>",
          "flood_lds16<P=47>", "flood_reg<DC=47,CPL=1,regular>", "flood_gmem<DC=48>", "flood_gmem<DC=64>"],
    "W": ["flood_tab2<DC=8,CPL=4,lo=3>", "flood_tab2<DC=8,CPL=4>", "flood_reg<DC=8,CPL=4>", "flood_gmem<DC=8>", "flood_gmem<DC=16>"],
    "R": ["flood_array2<P=47,CPL=2,ldsoffs,mix>", "flood_array2<P=47,CPL=2,ldsoffs>", "flood_array2<P=47,CPL=2>", "flood_lds16<P=47>",
          "flood_gmem<DC=48>"],
}


@pytest.mark.parametrize("cfg", ["A", "W", "R"])
def test_every_variant_parity(F, O, codes, torch_dev, cfg, monkeypatch):
    import torch
    code, ocode = codes[cfg]
    max_iter = 50 if cfg == "R" else 30
    mask = 0x3F if cfg == "R" else 0xFF
    snr = 2 * math.pow(10.0, (3.0 if cfg != "R" else 6.0) / 10) * code.rate
    llr = O.gen_llr(SEED, 4242, 40, code.n, snr, math.sqrt(1 / snr), 4)
    rng = np.random.default_rng(11)
    llr[-4:] = rng.integers(-20000, 20000, size=(4, code.n))  # forces the int16 kernels' fallback pass
    ref = O.decode_batch(ocode, llr, max_iter=max_iter, mask=mask)
    t = torch.from_numpy(llr).to(torch_dev)
    for name in VARIANTS[cfg]:
        monkeypatch.setenv("FPLDPC_KERNEL", name)
        dec = F.Decoder(code, max_iter=max_iter, width_mask=mask)
        assert dec.describe().startswith(name), (name, dec.describe())
        gpu = {k: v.cpu().numpy() for k, v in dec.decode_torch(t, post=True).items()}
        assert_same(gpu, ref, code.n, where=f"{cfg} {name}")


@pytest.mark.parametrize("cfg,eb", [("W", 2.0), ("A", 4.5)])
def test_full_batch_early_termination(F, O, codes, torch_dev, cfg, eb):
    """Every frame of a 4096-frame batch at a waterfall SNR with the harness codeword (early
    termination, refills of the packed kernels' halves at scale) -- a smaller batch missed a
    parity-combining bug that only shows on a few frames in thousands."""
    import torch
    code, ocode = codes[cfg]
    g = np.load(os.path.join(GOLDEN, "kat_w.npz" if cfg == "W" else "kat_a.npz"))
    rate = 0.5 if cfg == "W" else code.rate
    snr = 2 * math.pow(10.0, eb / 10) * rate
    llr = O.gen_llr(SEED, 20000, 4096, code.n, snr, math.sqrt(1 / snr), 4, cw=g["cw"])
    ref = O.decode_batch(ocode, llr, want_post=False)
    dec = F.Decoder(code)
    gpu = {k: v.cpu().numpy() for k, v in dec.decode_torch(torch.from_numpy(llr.astype(np.int16)).to(torch_dev)).items()}
    assert_same(gpu, ref, code.n, check_post=False, where=f"{cfg}@{eb} [{dec.describe()}]")


def test_r_full_batch_refills(F, O, codes, torch_dev):
    """R's default kernel (MixChecks: whole checks on threads 0..511, the last 104 checks two lanes
    per check) over 4096 frames at Eb/N0 where iteration counts vary per frame (6.0 / 6.5 / 7.0 dB:
    2..5 iterations or all 50, ArrayLDPC_Decoder.cpp:157-167), so a workgroup refills one frame
    half (and its split lanes' state) while the partner half is still decoding -- the grid holds
    256 x 2 frames, so 3584 frames are refills.  Every frame's iterations, hard bits, syndrome and
    posteriors against the oracle."""
    import torch
    code, ocode = codes["R"]
    dec = F.Decoder(code, max_iter=50, width_mask=0x3F)
    assert dec.describe().startswith("flood_array2<P=47,CPL=2,ldsoffs,mix>"), dec.describe()
    parts = []
    for i, eb in enumerate((6.5, 6.0, 7.0, 6.5)):
        snr = 2 * math.pow(10.0, eb / 10) * code.rate
        parts.append(O.gen_llr(SEED, 30000 + 1024 * i, 1024, code.n, snr, math.sqrt(1 / snr), 4))
    llr = np.concatenate(parts)
    ref = O.decode_batch(ocode, llr, max_iter=50, mask=0x3F)
    it = ref["iters"]
    assert len(np.unique(it)) >= 4 and (it == 50).sum() > 100 and (it <= 3).sum() > 1000, np.bincount(it)
    gpu = dec.decode_torch(torch.from_numpy(llr.astype(np.int16)).to(torch_dev), post=True)
    torch.cuda.synchronize()
    fb = dec.fallback_counts()
    assert_same({k: v.cpu().numpy() for k, v in gpu.items()}, ref, code.n,
                where=f"R 4096 refills [{dec.describe()}] fallbacks={fb}")
    print(f"R refills: iteration histogram {dict(zip(*np.unique(it, return_counts=True)))}, fallbacks {fb}")


@pytest.mark.parametrize("cfg,split", [("A", "1"), ("A", "0"), ("W", "1"), ("W", "0"), ("R", "1")],
                         ids=["A-split_tail", "A-no_split_tail", "W-split_tail", "W-no_split_tail", "R"])
def test_split_tail_parity(F, O, codes, torch_dev, monkeypatch, cfg, split):
    """The packed kernels' tail (flood_pk + ArrayChecks::split_step / TableChecks::split_step): once
    the queue is empty a workgroup's lone frame continues in the split form -- A: its check split over
    the lane halves; W: a lane's checks q and q + 2 in its two halves, the high half's degree masked
    per half -- moved to half 0 first when it was in half 1.  Batches sized so that lone
    frames occur from the first step (1, 3 frames: a pre-check at step 0 in the split form), with
    both halves' frames ending at different steps (mixed Eb/N0 and random LLRs, so the lone frame is
    sometimes in half 1), over the whole grid, with and without precheck, early_term off and
    max_iter 1; every output against the oracle -- and FPLDPC_SPLIT_TAIL=0 (the packed step
    throughout) the same.  R (MixChecks, 50 iterations, mask 0x3f; no split form, its grid holds
    512 frames) runs the same modes and mixes over batches that end inside, at and past one grid."""
    import torch
    monkeypatch.setenv("FPLDPC_SPLIT_TAIL", split)
    code, ocode = codes[cfg]
    base = _base(cfg)
    rs = np.random.default_rng(3)
    parts = []
    ebs = {"R": (5.5, 6.5, 7.5, 6.0, 7.0), "W": (0.5, 1.5, 2.5, 1.0, 2.0)}.get(cfg, (3.0, 4.5, 6.0, 3.5, 5.0))
    for i, eb in enumerate(ebs):
        snr = 2 * math.pow(10.0, eb / 10) * (0.5 if cfg == "W" else code.rate)
        parts.append(O.gen_llr(SEED, 60000 + 400 * i, 400, code.n, snr, math.sqrt(1 / snr), 4))
    llr = np.concatenate(parts)
    llr[rs.choice(len(llr), 60, replace=False)] = rs.integers(-60, 61, (60, code.n))  # never converge
    llr[rs.choice(len(llr), 40, replace=False)] = 40  # noiseless: pre-check passes
    llr = llr[rs.permutation(len(llr))]
    batches = {"R": (1, 3, 511, 513, 1100), "W": (1, 3, 1025, 1500, 2000)}.get(cfg, (1, 3, 769, 1537, 2000))
    for kw in (dict(), dict(precheck=True), dict(early_term=False, max_iter=7), dict(max_iter=1)):
        dec = F.Decoder(code, **{**base, **kw})
        assert dec.describe().startswith(PACKED[cfg]), dec.describe()
        for B in batches:
            x = llr[:B]
            ref = O.decode_batch(ocode, x, max_iter=kw.get("max_iter", base["max_iter"]),
                                 mask=base["width_mask"], precheck=kw.get("precheck", False))
            gpu = {k: v.cpu().numpy() for k, v in dec.decode_torch(torch.from_numpy(x.astype(np.int16)).to(torch_dev),
                                                                   post=True).items()}
            if kw.get("early_term", True):
                assert_same(gpu, ref, code.n, check_post=not kw.get("precheck"),
                            where=f"{cfg} split={split} {kw} B={B} [{dec.describe()}]")
            else:  # (the oracle always stops early) every frame runs 7 updates; its flag is its syndrome's
                assert (gpu["iters"] == 7).all()
                hard = F.unpack_hard(gpu["hard"], code.n)
                assert [code.syndrome_ok(h) for h in hard[:64]] == [bool(o) for o in gpu["syndrome_ok"][:64]]


@pytest.mark.parametrize("cfg", ["A", "W", "R"])
def test_int16_range_fallback(F, O, codes, torch_dev, cfg):
    """The packed kernels' int16-range guard (fpldpc_kernels.hip flood_pk: |LLR| <= kLlrMax = 8000
    and every c2v magnitude below cmax = 2^b - 1) tripped by the c2v-range taint with in-range
    LLRs: frames whose LLRs all have magnitudes 5000..8000 produce c2v above cmax (A 4095, W 2047,
    R 511: the largest 2^b - 1 with 8000 + (dv_max + 1)(2^(b+1) - 1) + 64 <= 32767) in their first
    iteration.  Exactly those frames (plus at most one partner each, sharing their posterior words)
    must go down the exact fallback chain, and every output must still equal the oracle.  A batch
    of plain AWGN frames at the bench's Eb/N0 must not touch the fallback chain (A, W)."""
    import torch
    code, ocode = codes[cfg]
    max_iter, mask = (50, 0x3F) if cfg == "R" else (30, 0xFF)
    eb = {"A": 0.0, "W": -2.0, "R": 2.0}[cfg]
    dec = F.Decoder(code, max_iter=max_iter, width_mask=mask)
    snr = 2 * math.pow(10.0, eb / 10) * code.rate
    sigma = math.sqrt(1 / snr)
    rng = np.random.default_rng(11)
    B, nbig = 64, 12
    llr = O.gen_llr(SEED, 0, B, code.n, snr, sigma, 4)
    assert np.abs(llr).max() <= 8000
    big = np.sort(rng.choice(B, nbig, replace=False))
    llr[big] = rng.integers(5000, 8001, (nbig, code.n)) * rng.choice([-1, 1], (nbig, code.n))
    ref = O.decode_batch(ocode, llr, max_iter=max_iter, mask=mask)
    gpu = dec.decode_torch(torch.from_numpy(llr.astype(np.int16)).to(torch_dev), post=True)
    torch.cuda.synchronize()
    fb = dec.fallback_counts()
    gpu = {k: v.cpu().numpy() for k, v in gpu.items()}
    assert_same(gpu, ref, code.n, where=f"{cfg} range fallback [{dec.describe()}] fallbacks={fb}")
    assert nbig <= fb[0] <= 2 * nbig, fb
    print(f"{cfg}: {nbig} large-LLR frames -> fallback counts {fb}")
    if cfg in ("A", "W"):
        llr = O.gen_llr(SEED, 4096, 256, code.n, snr, sigma, 4)
        dec.decode_torch(torch.from_numpy(llr.astype(np.int16)).to(torch_dev))
        torch.cuda.synchronize()
        assert dec.fallback_counts() == (0, 0)


@pytest.mark.parametrize("cfg", ["A", "W", "R"])
def test_bit_errors_masked_and_list(F, O, codes, torch_dev, cfg):
    """calculateBER per frame and the totals (ArrayLDPC_Decoder.cpp:707-722): with distinct info
    positions the packed kernels count errors from their hard-decision words (the packed mask
    form), with repeated positions from the index list; both = the count over the list, from the
    oracle's hard decisions, every repeat counted."""
    import torch
    code, ocode = codes[cfg]
    max_iter = 50 if cfg == "R" else 30
    mask = 0x3F if cfg == "R" else 0xFF
    snr = 2 * math.pow(10.0, (3.5 if cfg != "R" else 6.0) / 10) * code.rate
    llr = O.gen_llr(SEED, 900, 200, code.n, snr, math.sqrt(1 / snr), 4)
    ref = O.decode_batch(ocode, llr, max_iter=max_iter, mask=mask, want_post=False)
    rng = np.random.default_rng(5)
    k = code.n - code.rank
    distinct = np.sort(rng.choice(code.n, size=k, replace=False)).astype(np.int32)
    repeated = np.concatenate([distinct[: k - 40], distinct[:40]]).astype(np.int32)  # 40 positions twice
    dec = F.Decoder(code, max_iter=max_iter, width_mask=mask)
    t = torch.from_numpy(llr.astype(np.int16)).to(torch_dev)
    for idx in (distinct, repeated):
        bits = rng.integers(0, 2, size=len(idx)).astype(np.uint8)
        dec.set_reference(idx, bits)
        tot = torch.zeros(4, dtype=torch.int64, device=torch_dev)
        out = dec.decode_torch(t, bit_errors=True, totals=tot)
        want = (ref["hard"][:, idx] != bits[None, :]).sum(axis=1)
        be = out["bit_errors"].cpu().numpy()
        assert (be == want).all(), np.nonzero(be != want)[0][:8]
        assert tot.cpu().tolist() == [int(want.sum()), int((want > 0).sum()), len(llr), int(ref["iters"].sum())]


@pytest.mark.parametrize("r", [17, 22, 23])
def test_array_rows_mixed_split(F, O, torch_dev, r):
    """p47 array codes whose check counts exercise the R kernel's layout edges: r = 17 (799 checks:
    second checks on part of threads 0..255, no split checks), r = 22 (1034: 10 split checks, one
    partly active split wave) and r = 23 (1081: 57 split checks, split waves partly and fully idle),
    50 iterations, mask 0x3f, against the oracle."""
    import torch
    code = F.Code.array(47, r)
    ocode = O.OracleCode.from_alist_text(code.write_alist())
    dec = F.Decoder(code, max_iter=50, width_mask=0x3F)
    assert dec.describe().startswith("flood_array2<P=47,CPL=2,ldsoffs,mix>"), dec.describe()
    llr = np.concatenate([O.gen_llr(SEED, 700 + 50 * i, 24, code.n, snr, math.sqrt(1 / snr), 4)
                          for i, snr in enumerate(2 * math.pow(10.0, eb / 10) * code.rate for eb in (3.0, 6.0, 9.0))])
    ref = O.decode_batch(ocode, llr, max_iter=50, mask=0x3F)
    gpu = {k: v.cpu().numpy() for k, v in dec.decode_torch(torch.from_numpy(llr).to(torch_dev), post=True).items()}
    assert_same(gpu, ref, code.n, where=f"p47 r{r}")


def test_empty_batch_and_negative_batch(F, codes, torch_dev):
    """An empty batch is a no-op on every decode entry point (device and host, fixed and float; no
    buffers needed), totals untouched; a negative batch is an argument error."""
    import torch
    code, _ = codes["A"]
    dec = F.Decoder(code)
    tot = torch.zeros(4, dtype=torch.int64, device=torch_dev)
    out = dec.decode_torch(torch.empty((0, code.n), dtype=torch.int16, device=torch_dev), post=True, totals=tot)
    assert out["hard"].shape == (0, dec.hard_words) and out["iters"].shape == (0,) and out["post"].shape == (0, code.n)
    assert tot.cpu().tolist() == [0, 0, 0, 0]
    h = dec.decode_host(np.empty((0, code.n), np.int16), post=True, totals=np.zeros(4, np.int64))
    assert h["iters"].shape == (0,) and h["totals"].tolist() == [0, 0, 0, 0]
    assert dec.decode_float_torch(torch.empty((0, code.n), dtype=torch.float64, device=torch_dev))["iters"].shape == (0,)
    assert dec.decode_float_host(np.empty((0, code.n)))["iters"].shape == (0,)
    with pytest.raises(Exception, match="negative batch"):
        dec.decode_ptrs(0, 1, -1, 0, 0, 0, 0, 0, 0, 0)
