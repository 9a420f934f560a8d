"""Code-generation guard for the default kernels (CPU only: device-only hipcc compiles for gfx950).

The packed kernels are bound by VALU issue, and their speed rests on register allocation and on the
per-unit scheduler options (fixedpointldpc_amd/_build.py SOURCE_FLAGS, DESIGN.md §5 "Code generation
per kernel"): A at 3 waves per SIMD needs <= 168 VGPRs; a VGPR spill or scratch in a step loop costs
far more than any scheduling gain.  This test recompiles the device translation units with the
library's own per-source options (tools/resource_usage.py) and fails when
  * a default variant's VGPRs no longer allow its waves per SIMD, or it spills VGPRs / uses scratch,
    or its SGPR spills grow past the shipped build's;
  * the A or W unit loses its options: without -disable-post-ra A's step block carries ~160 s_nop
    hazard waits instead of ~690 (the post-RA scheduler hoists them away and A runs 3 % slower; W
    127 instead of 273), which is how a dropped or renamed option shows in the ISA;
  * any product device code reads the kernel arguments through __builtin_amdgcn_kernarg_segment_ptr()
    (the round-5 out-of-line split-tail callee that did so faulted).
"""
import concurrent.futures
import glob
import os
import re
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
CSRC = os.path.join(ROOT, "fixedpointldpc_amd", "csrc")

# mangled-name fragment -> (max VGPRs, min waves / SIMD, max SGPR spills, max scratch bytes / lane), as
# shipped (round 6).  The float decoder's register-resident kernels spill by design.
BUDGET = {
    # A: flood_pk<ArrayChecks<47>, 3>, fpldpc_kernels_a1.hip
    "flood_pkINS0_11ArrayChecksILi47ELi1ELi256ELb1ELb0EEELi3ELi256E": (168, 3, 67, 0),
    # W: flood_pk<TableChecks<8, 4, 7, 3>, 4>, fpldpc_kernels_w1.hip (with its split tail since round 6:
    # 124 VGPRs, 125 SGPR spills with the quick exit and the 16-byte LLR copy, still 4 waves per SIMD
    # and no scratch)
    "flood_pkINS0_11TableChecksILi8ELi4ELi7ELi3ELi256EEELi4ELi256E": (128, 4, 125, 0),
    # R: flood_pk<MixChecks<47, 768>, 1, 768>
    "flood_pkINS0_9MixChecksILi47ELi768EEELi1ELi768E": (168, 3, 31, 0),
    # the R fallback chain's int16 LDS-state kernel, the A fallback
    "flood_lds16ILi47ELi1024E": (128, 4, 16, 0),
    "flood_arrayILi47E": (128, 4, 105, 0),
    # float decoder (f3): occupancy and scratch as shipped
    "bp_float_regILi47ELb1ELb1E": (128, 4, 46, 208),
    "bp_float_regILi8ELb0ELb0E": (72, 7, 105, 104),
    # device channel
    "channel_kernel": (64, 8, 0, 0),
}


@pytest.fixture(scope="module")
def usage():
    import resource_usage
    srcs = ["fpldpc_kernels_a1.hip", "fpldpc_kernels_w1.hip", "fpldpc_kernels.hip", "fpldpc_float.hip", "fpldpc_gen.hip"]
    with concurrent.futures.ThreadPoolExecutor(5) as ex:
        rows = list(ex.map(lambda s: resource_usage.usage(os.path.join(CSRC, s)), srcs))
    return [r for rs in rows for r in rs]


def test_default_kernels_register_budget(usage):
    assert usage, "hipcc produced no resource remarks"
    for frag, (vmax, occ, smax, scratch) in BUDGET.items():
        rows = [r for r in usage if frag in r["name"]]
        assert rows, f"kernel {frag} not found in the device units"
        for r in rows:
            vg, oc = int(r["VGPRs"]), int(r["Occupancy [waves/SIMD]"])
            assert vg <= vmax and oc >= occ, (frag, vg, oc)
            assert int(r["ScratchSize [bytes/lane]"]) <= scratch, (frag, r["ScratchSize [bytes/lane]"])
            if scratch == 0:
                assert int(r["VGPRs Spill"]) == 0, (frag, r["VGPRs Spill"])
            assert int(r["SGPRs Spill"]) <= smax, (frag, r["SGPRs Spill"])


@pytest.mark.parametrize("unit,opts,min_nops", [("fpldpc_kernels_a1.hip", ("-mllvm=-disable-post-ra", "-mllvm=-misched=ilpmax"), 400),
                                                ("fpldpc_kernels_w1.hip", ("-mllvm=-disable-post-ra",), 200)])
def test_unit_scheduler_options_in_effect(unit, opts, min_nops):
    """The A and W units' ISA carries the signature of their options: -disable-post-ra leaves the
    hazard s_nop waits where the pre-RA schedule put them (A: 686 against 164 with hipcc's defaults;
    W: 273 against 127)."""
    from fixedpointldpc_amd._build import SOURCE_FLAGS
    flags = SOURCE_FLAGS[unit]
    assert all(o in flags for o in opts), flags
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-I", os.path.join(ROOT, "include"), "-I", CSRC, "--offload-device-only", "-S",
           os.path.join(CSRC, unit), "-o", "-", *flags]
    asm = subprocess.run(cmd, capture_output=True, text=True, check=True).stdout
    nops = len(re.findall(r"^\s+s_nop\b", asm, flags=re.M))
    assert nops >= min_nops, f"{nops} s_nop: {unit} compiled as if without -disable-post-ra"


def test_no_kernarg_pointer_reads_in_product():
    for p in glob.glob(os.path.join(CSRC, "*")):
        if p.endswith((".hip", ".cpp", ".hpp", ".h")):
            assert "kernarg_segment_ptr" not in open(p).read(), p
