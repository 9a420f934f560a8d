"""GPU parity across the runtime parameters that replace the reference's compile-time enums.

The reference fixes WIDTH_MASK and FRAC_WIDTH by enum (ArrayLDPCMacro.h:28-39; Constant =
int((5.0/8.0) * (1 << FRAC_WIDTH)), :175) and folds with sxor (ArrayLDPC_Decoder.cpp:677-694).  The
C ABI takes both at run time (fpldpc_params.frac_bits 0..16, width_mask > 0), and the kernel choice
depends on them (fpldpc_kernels.hip choose_kernel): contiguous masks 2^w - 1 up to 0xffff run the
packed int16-pair kernels (bit-field extract, C and the mask as u16 pairs, the int16 range guard
packed_cmax, which depends on C), non-contiguous masks the general-mask int32 kernels, masks above
16 bits no packed kernel, and a C too large for the int16 argument no int16 kernel at all.

Every case decodes AWGN frames quantised at that FRAC_WIDTH (PerfTest.cpp:108-120) plus random LLRs
over the whole int16 range, in ±2000 and in ±3 (exact zeros: sgn(0) = -1), and compares iterations,
hard decisions, syndrome verdicts and posteriors with the oracle at the same C and mask.  With
FPLDPC_PARAM_REPORT=<file> each case appends one JSON line (config, FRAC, mask, the variant that ran
from dec.describe(), the fallback counts) -- profiles/r6/param_sweep.jsonl is that report.
"""
import json
import math
import os

import numpy as np
import pytest

from conftest import assert_same

pytestmark = pytest.mark.gpu

SEED = 123456789
FRACS = (2, 3, 5, 6, 8)
MASKS = (0x0F, 0x1F, 0x7F, 0x1FF, 0xFFF, 0xFFFF, 0xF3, 0x1FFFF)
# beyond the verdict's grid: FRAC 0 (C = 0) and the large-C end, where packed_cmax shrinks (12),
# leaves R's int16 LDS-state fallback out (15: C = 20480 > 2^14) and rules out every int16 kernel (16)
EXTRA = [(f, m) for f in (0, 12, 15, 16) for m in (0xFF, 0xFFFF)]
CFG = {"A": (30, (3.0, 0.0)), "W": (30, (1.5, -2.0)), "R": (50, (6.0, 2.0))}
PACKED = {"A": "flood_array2<P=47,W=3>", "W": "flood_tab2<DC=8,CPL=4,lo=3>", "R": "flood_array2<P=47,CPL=2,ldsoffs,mix>"}
GENERAL_MASK = {"A": "flood_reg<DC=47,CPL=1,regular>", "W": "flood_reg<DC=8,CPL=4>", "R": "flood_gmem<DC=48>"}
WIDE_MASK = {"A": "flood_array<P=47>", "W": "flood_reg<DC=8,CPL=4>", "R": "flood_gmem<DC=48>"}


def _constant(frac):
    return int((5.0 / 8.0) * (1 << frac))


def _packed_ok(code, frac):
    """packed_cmax > 0 (fpldpc_kernels.hip), and for R's chain C <= 2^14 (flood_lds16)."""
    C = _constant(frac)
    return 8000 + (code.dv_max + 1) + max(64, C) <= 32767


def _expected(cfg, code, frac, mask):
    low = mask >= 3 and (mask & (mask + 1)) == 0
    if not low:
        return GENERAL_MASK[cfg]
    if mask > 0xFFFF:
        return WIDE_MASK[cfg]
    if not _packed_ok(code, frac) or (cfg == "R" and _constant(frac) > (1 << 14)):
        return {"A": "flood_array<P=47>", "W": "flood_reg<DC=8,CPL=4>", "R": "flood_gmem<DC=48>"}[cfg]
    return PACKED[cfg]


def _inputs(O, code, frac, eb_pair, salt):
    rng = np.random.default_rng(1000 + salt)
    parts = []
    for i, eb in enumerate(eb_pair):
        snr = 2 * math.pow(10.0, eb / 10) * code.rate
        parts.append(O.gen_llr(SEED, 5000 * salt + 100 * i, 16, code.n, snr, math.sqrt(1 / snr), frac))
    parts += [rng.integers(-32768, 32768, (8, code.n)), rng.integers(-2000, 2001, (8, code.n)),
              rng.integers(-3, 4, (4, code.n))]
    return np.concatenate(parts).astype(np.int32)


def _report(rec):
    path = os.environ.get("FPLDPC_PARAM_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def _run_case(F, O, codes, torch_dev, cfg, frac, mask):
    import torch
    code, ocode = codes[cfg]
    max_iter, ebs = CFG[cfg]
    llr = _inputs(O, code, frac, ebs, frac * 37 + MASKS.index(mask) if mask in MASKS else frac)
    dec = F.Decoder(code, max_iter=max_iter, frac_bits=frac, width_mask=mask)
    desc = dec.describe()
    ref = O.decode_batch(ocode, llr, max_iter=max_iter, frac_bits=frac, mask=mask)
    gpu = dec.decode_torch(torch.from_numpy(llr).to(torch_dev), post=True)
    torch.cuda.synchronize()
    fb = dec.fallback_counts()
    gpu = {k: v.cpu().numpy() for k, v in gpu.items()}
    _report({"config": cfg, "frac_bits": frac, "C": _constant(frac), "width_mask": hex(mask), "variant": desc.split()[0],
             "describe": desc, "fallback_counts": list(fb), "frames": len(llr),
             "iters_hist": {int(k): int(v) for k, v in zip(*np.unique(ref["iters"], return_counts=True))}})
    assert_same(gpu, ref, code.n, where=f"{cfg} frac={frac} mask={mask:#x} [{desc}] fallbacks={fb}")
    want = _expected(cfg, code, frac, mask)
    assert desc.startswith(want), (cfg, frac, hex(mask), desc, want)


@pytest.mark.parametrize("frac", FRACS)
@pytest.mark.parametrize("cfg", ["A", "W", "R"])
def test_param_sweep(F, O, codes, torch_dev, cfg, frac):
    for mask in MASKS:
        _run_case(F, O, codes, torch_dev, cfg, frac, mask)


@pytest.mark.parametrize("cfg", ["A", "W", "R"])
def test_param_extremes(F, O, codes, torch_dev, cfg):
    for frac, mask in EXTRA:
        _run_case(F, O, codes, torch_dev, cfg, frac, mask)
