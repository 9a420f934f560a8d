import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_DIR = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the device)")


@pytest.fixture(scope="session")
def F():
    import fixedpointldpc_amd
    return fixedpointldpc_amd


@pytest.fixture(scope="session")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a HIP device"
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def O():
    from oracle import oracle
    return oracle


# The three BASELINE configs' codes, built natively by the product (token-equal to the
# reference's alist files, tests/test_codes.py) and handed to the oracle as alist text.
CODES = {
    "A": lambda F: F.Code.array(47, 5),        # H_array_p47_r5_forward.txt
    "W": lambda F: F.Code.wifi_1944_r12(),     # H_802.11_IndZero.txt
    "R": lambda F: F.Code.array(47, 24),       # codes/H_array_p47_r24_forward.txt
}


@pytest.fixture(scope="session")
def codes(F, O):
    out = {}
    for k, mk in CODES.items():
        c = mk(F)
        out[k] = (c, O.OracleCode.from_alist_text(c.write_alist()))
    return out


def assert_same(gpu, ref, n, check_post=True, where=""):
    from fixedpointldpc_amd import unpack_hard
    it_g, it_r = np.asarray(gpu["iters"]), np.asarray(ref["iters"])
    bad = np.nonzero(it_g != it_r)[0]
    assert bad.size == 0, f"{where}: iteration mismatch at frames {bad[:8]} gpu={it_g[bad[:8]]} ref={it_r[bad[:8]]}"
    hard = unpack_hard(np.asarray(gpu["hard"]), n)
    bad = np.nonzero((hard != ref["hard"]).any(axis=1))[0]
    assert bad.size == 0, f"{where}: hard-decision mismatch at frames {bad[:8]}"
    assert (np.asarray(gpu["syndrome_ok"]) == ref["syndrome_ok"]).all(), f"{where}: syndrome mismatch"
    if check_post and "post" in gpu and ref.get("post") is not None:
        bad = np.nonzero((np.asarray(gpu["post"]) != ref["post"]).any(axis=1))[0]
        assert bad.size == 0, f"{where}: posterior mismatch at frames {bad[:8]}"


def stale_profile_ok(line):
    """A bench line without a roofline fraction is accepted only while FPLDPC_ALLOW_STALE_PROFILE=1
    (intermediate GPU runs after a kernel edit, before its profiling pass is committed: bench.py
    quotes roofline.frac only from counters of the same kernel build) and only with that reason."""
    return os.environ.get("FPLDPC_ALLOW_STALE_PROFILE") == "1" and "no committed" in line["roofline"].get("basis", "")
