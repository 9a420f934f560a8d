"""Systematic encoder (fpldpc_encoder.cpp) on the host, against the reference's KAT codewords
(tests/golden/kat_{w,a}.npz, produced by the reference's own FP_Encoder / G files).  CPU only."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, REF_DIR


def _g(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.mark.parametrize("key,fixture", [("W", "kat_w.npz"), ("A", "kat_a.npz")])
def test_native_encoder_matches_reference_kat(F, key, fixture):
    """Encoder derived from H alone = the reference's G-file encoder: same info positions
    (getInfoIndex), same codeword for the harness's info string."""
    g = _g(fixture)
    code = F.Code.wifi_1944_r12() if key == "W" else F.Code.array(47, 5)
    enc = F.Encoder.from_code(code)
    assert enc.k == code.k and (enc.info_index == g["info_idx"]).all()
    cw = enc.encode(g["info_bits"])[0]
    assert (cw == g["cw"]).all()
    assert code.syndrome_ok(cw)


def test_unpack_info_bytes(F):
    """setInfoBit (ArrayLDPC_Decoder.cpp:178-197) on the WiFi harness string (PerfTest.cpp:33)."""
    g = _g("kat_w.npz")
    s = b"OMG  how long   dd   should this string be to make it 243"
    assert (F.unpack_info_bytes(s, 122, 972) == g["info_bits"]).all()


def test_random_codewords_satisfy_h(F):
    rs = np.random.default_rng(3)
    for code in (F.Code.wifi_1944_r12(), F.Code.array(47, 5), F.Code.array(47, 24)):
        enc = F.Encoder.from_code(code)
        cw = enc.encode(rs.integers(0, 2, (8, enc.k)), nthreads=3)
        assert all(code.syndrome_ok(c) for c in cw)
        assert (cw[:, enc.info_index] <= 1).all()


@pytest.mark.skipif(not os.path.isdir(REF_DIR), reason="reference G files only in the build container")
def test_g_file_loader_matches_native(F):
    """FP_Encoder(char*, int) (ArrayLDPC_Encoder.cpp:34-157) on the reference's own G files."""
    for gfile, code in (("H_802.11_IndZerog.txt", F.Code.wifi_1944_r12()),
                        ("codes/G_array_forward.txt", F.Code.array(47, 5))):
        eg = F.Encoder.load_g(os.path.join(REF_DIR, gfile))
        en = F.Encoder.from_code(code)
        assert (eg.info_index == en.info_index).all() and (eg.parity_index == en.parity_index).all()
        u = np.random.default_rng(1).integers(0, 2, (4, eg.k))
        assert (eg.encode(u) == en.encode(u)).all()


def test_g_file_errors(F, tmp_path):
    p = tmp_path / "g.txt"
    p.write_text("4 2\n1 1\n1 1 0 2\n")
    with pytest.raises(F.FpldpcError):
        F.Encoder.load_g(str(p))
    with pytest.raises(F.FpldpcError) as e:
        F.Encoder.load_g(str(tmp_path / "missing.txt"))
    assert e.value.code == -2
