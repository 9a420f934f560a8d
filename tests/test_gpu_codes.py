"""Codes beyond the three BASELINE configs, GPU vs the CPU oracle, bit-exact.

The reference's decode_general_fp is alist-generic (ReadH, ArrayLDPC_Decoder.cpp:642-674): any H
with sorted rows decodes.  These tests feed the product codes that land on every kernel family --
other array codes in both shift directions (the array kernels are specialised to p = 47, so these
take the table / generic kernels), random irregular codes with degree-2 checks, and high check
degrees (the global-memory kernel) -- and compare iterations, hard decisions, syndrome verdicts and
posteriors with the oracle, plus the floating-point decoder at BER level.
"""
import math

import numpy as np
import pytest

from conftest import assert_same

pytestmark = pytest.mark.gpu
SEED = 123456789


def random_alist(n, m, cdegs, seed):
    """alist text of a random H: check c has degree cdegs[c % len(cdegs)], every var used, rows sorted."""
    rs = np.random.default_rng(seed)
    H = np.zeros((m, n), np.uint8)
    for c in range(m):
        d = cdegs[c % len(cdegs)]
        H[c, rs.choice(n, d, replace=False)] = 1
    for v in np.nonzero(H.sum(axis=0) == 0)[0]:  # every variable in at least one check
        H[rs.integers(m), v] = 1
    vl = [np.nonzero(H[:, v])[0] for v in range(n)]
    cl = [np.nonzero(H[c])[0] for c in range(m)]
    dv, dc = max(len(x) for x in vl), max(len(x) for x in cl)
    out = [f"{n} {m}", f"{dv} {dc}", " ".join(str(len(x)) for x in vl), " ".join(str(len(x)) for x in cl)]
    out += [" ".join(map(str, x)) for x in vl] + [" ".join(map(str, x)) for x in cl]
    return "\n".join(out) + "\n"


def permute_checks(text, seed):
    """The same code with its checks listed in a random order (variable lists renumbered, sorted)."""
    ln = text.strip("\n").split("\n")
    n, m = map(int, ln[0].split())
    vl = [list(map(int, x.split())) for x in ln[4:4 + n]]
    cl = [x for x in ln[4 + n:4 + n + m]]
    cdeg = ln[3].split()
    perm = np.random.default_rng(seed).permutation(m)  # new position j holds old check perm[j]
    inv = np.empty(m, int)
    inv[perm] = np.arange(m)
    out = ln[:3] + [" ".join(cdeg[i] for i in perm)]
    out += [" ".join(str(c) for c in sorted(int(inv[c]) for c in x)) for x in vl] + [cl[i] for i in perm]
    return "\n".join(out) + "\n"


CODES = {
    "array31x4_fwd": lambda F: F.Code.array(31, 4, True),
    "array31x4_bwd": lambda F: F.Code.array(31, 4, False),
    "array53x6_fwd": lambda F: F.Code.array(53, 6, True),
    "array47x5_bwd": lambda F: F.Code.array(47, 5, False),
    "rand_irregular": lambda F: F.Code.parse(random_alist(600, 300, [2, 3, 6, 7, 8, 12], 1)),
    "rand_deg60": lambda F: F.Code.parse(random_alist(600, 40, [58, 45, 20], 2)),
    "rand_small": lambda F: F.Code.parse(random_alist(40, 20, [2, 3, 4], 3)),
    # degrees 7 / 8 with >= 768 of degree 7: the table kernel whose first three passes fold 7 slots
    # (checks listed by degree on the device); the degree-8 checks scattered through the code
    "rand_78_edge": lambda F: F.Code.parse(random_alist(1200, 960, [7, 7, 7, 7, 8], 13)),  # exactly 768 of degree 7
    "wifi_rows_permuted": lambda F: F.Code.parse(permute_checks(F.Code.wifi_1944_r12().write_alist(), 5)),
}


@pytest.mark.parametrize("name", sorted(CODES))
def test_generic_code_parity(F, O, torch_dev, name):
    import torch
    code = CODES[name](F)
    ocode = O.OracleCode.from_alist_text(code.write_alist())
    rate = max(code.rate, 0.3)
    for mask in (0xFF, 0x3F):
        try:
            dec = F.Decoder(code, max_iter=20, width_mask=mask)
        except F.FpldpcError as e:  # a code outside every kernel's envelope must say so, not decode wrong
            assert e.code == -4, e
            pytest.skip(f"{name}: {e}")
        for i, eb in enumerate((1.0, 3.0, 6.0)):
            snr = 2 * math.pow(10.0, eb / 10) * rate
            llr = O.gen_llr(SEED, 100 * i, 48, code.n, snr, math.sqrt(1 / snr), 4)
            ref = O.decode_batch(ocode, llr, max_iter=20, mask=mask)
            gpu = dec.decode_torch(torch.from_numpy(llr.astype(np.int16)).to(torch_dev), post=True)
            gpu = {k: v.cpu().numpy() for k, v in gpu.items()}
            assert_same(gpu, ref, code.n, where=f"{name} mask {mask:#x} {eb} dB [{dec.describe()}]")
        rng = np.random.default_rng(5)
        llr = rng.integers(-2000, 2001, (16, code.n)).astype(np.int32)
        ref = O.decode_batch(ocode, llr, max_iter=8, mask=mask)
        dec8 = F.Decoder(code, max_iter=8, width_mask=mask)
        gpu = {k: v.cpu().numpy() for k, v in dec8.decode_torch(torch.from_numpy(llr).to(torch_dev), post=True).items()}
        assert_same(gpu, ref, code.n, where=f"{name} random LLRs mask {mask:#x}")


@pytest.mark.parametrize("name", ["rand_78_edge", "wifi_rows_permuted"])
def test_degree_sorted_table_kernel_chosen(F, name):
    """Both mixed 7 / 8 codes land on the degree-sorted table kernel (the parity test above then
    covers it with the degree-8 checks away from the end of the code's check order)."""
    assert F.Decoder(CODES[name](F)).describe().startswith("flood_tab2<DC=8,CPL=4,lo=3>")


@pytest.mark.parametrize("name", ["array31x4_fwd", "rand_irregular", "rand_deg60"])
def test_generic_code_float(F, O, torch_dev, name):
    import torch
    code = CODES[name](F)
    ocode = O.OracleCode.from_alist_text(code.write_alist())
    snr, sigma = F.snr_sigma(2.0, max(code.rate, 0.3))
    llr = O.gen_llr_f64(SEED, 0, 64, code.n, snr, sigma)
    ref = O.decode_float_batch(ocode, llr, max_iter=20)
    dec = F.Decoder(code, max_iter=20)
    out = dec.decode_float_torch(torch.from_numpy(llr).to(torch_dev))
    it = out["iters"].cpu().numpy()
    hard = F.unpack_hard(out["hard"].cpu().numpy(), code.n)
    same = (it == ref["iters"]) & (hard == ref["hard"]).all(axis=1)
    assert same.mean() >= 0.98, f"{name}: {int((~same).sum())} of 64 frames differ"
