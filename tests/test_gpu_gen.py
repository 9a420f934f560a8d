"""Device-side frame generation (fpldpc_gen.hip) through the C ABI: the batched encoder
(fpldpc_encoder_encode) against the host encoder, and the device channel (fpldpc_channel_llr)
against the host channel, which tests/test_oracle.py pins to the reference's own Random()/Normal()
(oracle/_ref) and to the published KAT-W run.

Bar: bit-exact.  The device channel shares the host's Lehmer states exactly; its normals use the
device libm (log/sqrt in double), so this file compares the WHOLE published KAT-W stream
(393214 frames x 1944 draws = 764 M LLRs) element by element.
"""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
SEED = 123456789


def _g(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.mark.parametrize("key", ["A", "W", "R"])
def test_device_encoder_matches_host(F, torch_dev, codes, key):
    import torch
    code = codes[key][0]
    enc = F.Encoder.from_code(code)
    rs = np.random.default_rng(11)
    for batch in (1, 7, 3000):
        info = rs.integers(0, 2, (batch, enc.k)).astype(np.uint8)
        ref = enc.encode(info, nthreads=8)
        got = enc.encode_torch(torch.from_numpy(info).to(torch_dev)).cpu().numpy()
        assert (got == ref).all(), f"{key} batch {batch}: {np.argwhere(got != ref)[:4]}"
    # bytes with junk above the LSB: only bit 0 counts (as encode_host)
    info = rs.integers(0, 256, (5, enc.k)).astype(np.uint8)
    got = enc.encode_torch(torch.from_numpy(info).to(torch_dev)).cpu().numpy()
    assert (got == enc.encode(info & 1)).all()
    assert all(code.syndrome_ok(c) for c in got)


def test_device_encoder_kat_codewords(F, torch_dev):
    import torch
    for fx, code in (("kat_w.npz", F.Code.wifi_1944_r12()), ("kat_a.npz", F.Code.array(47, 5))):
        g = _g(fx)
        enc = F.Encoder.from_code(code)
        got = enc.encode_torch(torch.from_numpy(g["info_bits"][None]).to(torch_dev)).cpu().numpy()[0]
        assert (got == g["cw"]).all(), fx


def test_device_encoder_empty_batch(F, torch_dev):
    import torch
    enc = F.Encoder.from_code(F.Code.array(47, 5))
    assert enc.encode_torch(torch.empty((0, enc.k), dtype=torch.uint8, device=torch_dev)).shape == (0, enc.n)


@pytest.mark.parametrize("dtype", ["i16", "i32"])
def test_device_channel_matches_host(F, torch_dev, dtype):
    import torch
    tdt, ndt = (torch.int16, np.int16) if dtype == "i16" else (torch.int32, np.int32)
    g = _g("kat_w.npz")
    cw_np = g["cw"].astype(np.uint8)
    cw = torch.from_numpy(cw_np).to(torch_dev)
    for ebn0, first, frames, frac in ((2.0, 0, 2000, 4), (-3.0, 123457, 777, 4), (6.0, 10 ** 6, 333, 6)):
        snr, sigma = F.snr_sigma(ebn0, 0.5)
        for c_np, c_t in ((None, None), (cw_np, cw)):
            ref = F.channel_llr(SEED, first, frames, 1944, snr, sigma, frac, c_np, ndt, nthreads=16)
            got, ovf = F.channel_llr_torch(SEED, first, frames, 1944, snr, sigma, frac, c_t, tdt, torch_dev)
            got = got.cpu().numpy()
            assert int(ovf.item()) == 0
            bad = np.argwhere(got != ref)
            assert bad.size == 0, f"{ebn0} dB first {first}: {bad[:4]} got {got[tuple(bad[0])]} ref {ref[tuple(bad[0])]}"


def test_device_channel_per_frame_codewords_and_odd_n(F, torch_dev):
    """cw_per_frame = 1 (each frame its own codeword, e.g. from fpldpc_encoder_encode) and n not a
    multiple of the 16-draw chunk."""
    import torch
    rs = np.random.default_rng(5)
    for n in (2209, 1944, 17, 1):
        frames = 300
        cws = rs.integers(0, 2, (frames, n)).astype(np.uint8)
        snr, sigma = F.snr_sigma(1.0, 0.5)
        ref = np.stack([F.channel_llr(SEED, 40 + f, 1, n, snr, sigma, 4, cws[f], np.int32)[0] for f in range(frames)])
        got, _ = F.channel_llr_torch(SEED, 40, frames, n, snr, sigma, 4, torch.from_numpy(cws).to(torch_dev),
                                     torch.int32, torch_dev)
        assert (got.cpu().numpy() == ref).all(), n


def test_device_channel_int16_overflow_count(F, torch_dev):
    import torch
    snr, sigma = 2000.0, math.sqrt(1 / 2000.0)  # 2*snr*2^4 > 32767 for every bit
    got, ovf = F.channel_llr_torch(SEED, 0, 9, 64, snr, sigma, 4, None, torch.int16, torch_dev)
    assert int(ovf.item()) == 9 * 64  # every value
    with pytest.raises(F.FpldpcError):
        F.channel_llr(SEED, 0, 9, 64, snr, sigma, 4, None, np.int16)
    with pytest.raises(F.FpldpcError):  # argument checks as the host's
        F.channel_llr_torch(0, 0, 1, 64, 1.0, 1.0, 4, None, torch.int16, torch_dev)


def test_device_channel_whole_kat_w_stream(F, torch_dev):
    """Every LLR of the published KAT-W run (frames 0..393213, 2 dB, R = 0.5, the KAT codeword)."""
    import torch
    g = _g("kat_w.npz")
    cw_np = g["cw"].astype(np.uint8)
    cw = torch.from_numpy(cw_np).to(torch_dev)
    snr = 2 * math.pow(10.0, 2.0 / 10) * 0.5
    sigma = math.sqrt(1 / snr)
    total, chunk, bad = 393214, 32768, 0
    for first in range(0, total, chunk):
        fr = min(chunk, total - first)
        ref = F.channel_llr(SEED, first, fr, 1944, snr, sigma, 4, cw_np, np.int16, nthreads=16)
        got, ovf = F.channel_llr_torch(SEED, first, fr, 1944, snr, sigma, 4, cw, torch.int16, torch_dev)
        bad += int((got.cpu().numpy() != ref).sum())
        assert int(ovf.item()) == 0
    assert bad == 0, f"{bad} of {total * 1944} LLRs differ from the host channel"


def test_encode_channel_decode_on_device(F, torch_dev, codes, O):
    """The whole simulation chain on the device: random info -> encoder -> channel (per-frame
    codewords) -> decoder, checked against the oracle decoding the host-generated LLRs."""
    import torch
    code, ocode = codes["A"]
    enc = F.Encoder.from_code(code)
    rs = np.random.default_rng(9)
    frames = 512
    info = rs.integers(0, 2, (frames, enc.k)).astype(np.uint8)
    cw_d = enc.encode_torch(torch.from_numpy(info).to(torch_dev))
    snr, sigma = F.snr_sigma(5.5, code.rate)
    llr_d, _ = F.channel_llr_torch(SEED, 0, frames, code.n, snr, sigma, 4, cw_d, torch.int16, torch_dev)
    cw_h = enc.encode(info)
    llr_h = np.stack([F.channel_llr(SEED, f, 1, code.n, snr, sigma, 4, cw_h[f], np.int16)[0] for f in range(frames)])
    assert (llr_d.cpu().numpy() == llr_h).all()
    dec = F.Decoder(code)
    got = dec.decode_torch(llr_d)
    ref = O.decode_batch(ocode, llr_h, max_iter=30, mask=0xFF, want_post=False)
    assert (got["iters"].cpu().numpy() == ref["iters"]).all()
    hard = F.unpack_hard(got["hard"].cpu().numpy(), code.n)
    assert (hard == ref["hard"]).all()
    # most frames decode to the transmitted codeword at 5.5 dB (rate 0.895: 3 dB is below capacity)
    assert (hard == cw_h).all(axis=1).mean() > 0.9
