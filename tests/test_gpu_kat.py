"""End-to-end known-answer tests on the GPU, through the C ABI (fpldpc_ber_sim / fpldpc_decode).

KAT-W: the reference's only published result (wifi_results_4_4_2dB_30iter.txt: 2732 bit errors,
100 frame errors, 393214 frames at 2 dB) -- the whole 393214-frame run, decoded on the GPU.
KAT-A: ArrayLDPC_Debug at 4.5 dB with decode_fixpoint (2515 / 100 / 2108).
Per-frame reference decodes compared directly with the GPU (no oracle in between):
frames_w.npz (the unmodified reference build), frames_a.npz / fixpoint_a.npz (p47/r5 build:
decode_general_fp, decode_fixpoint incl. pre-check passes, DecodeTrial) and frames_r.npz (p47/r24
build: 50 iterations, mask 0x3f).
"""
import json
import math
import os
import zlib

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
SEED = 123456789


def _g(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.mark.parametrize("device_channel", [False, True], ids=["host_channel", "device_channel"])
def test_kat_w_full_published_run(F, device_channel):
    kj = json.load(open(os.path.join(GOLDEN, "kat_w.json")))
    kw = _g("kat_w.npz")
    code = F.Code.wifi_1944_r12()
    dec = F.Decoder(code)
    snr = 2 * math.pow(10.0, 2.0 / 10) * 0.5  # PerfTest.cpp:62 (rate hard-coded 0.5)
    sigma = math.sqrt(1 / snr)
    r = dec.ber_sim(snr, sigma, info_index=kw["info_idx"], info_bits=kw["info_bits"], codeword=kw["cw"],
                    max_frame_errors=100, host_threads=16, device_channel=device_channel)
    got = (r["bit_errors"], r["frame_errors"], r["frames"])
    assert got == (kj["bit_errors"], kj["frame_errors"], kj["frames"]), got
    fer = r["frame_errors"] / r["frames"]
    ber = r["bit_errors"] / r["frames"] / 1944  # PerfTest.cpp:137 divides by CWD_LENGTH
    assert f"{fer:g}" == kj["fer_text"] and f"{ber:g}".replace("e-0", "e-00") == kj["ber_text"]
    print(f"KAT-W (device_channel={device_channel}) {got} in {r['seconds']:.2f} s ({r['frames_decoded']} frames decoded)")


def test_kat_w_checkpoints_sharded(F):
    """Frame ranges decoded independently (the multi-GPU partitioning, skip-ahead per range) sum to
    the reference's cumulative checkpoints."""
    kj = json.load(open(os.path.join(GOLDEN, "kat_w.json")))
    kw = _g("kat_w.npz")
    dec = F.Decoder(F.Code.wifi_1944_r12())
    snr = 2 * math.pow(10.0, 2.0 / 10) * 0.5
    sigma = math.sqrt(1 / snr)
    be = fe = 0
    for f0 in range(0, 50000, 10000):
        r = dec.ber_sim(snr, sigma, info_index=kw["info_idx"], info_bits=kw["info_bits"], codeword=kw["cw"],
                        first_frame=f0, max_frames=10000, max_frame_errors=0, chunk=4096)
        be += r["bit_errors"]
        fe += r["frame_errors"]
        assert [f0 + 10000, be, fe] == kj["checkpoints"][f0 // 10000]


@pytest.mark.parametrize("device_channel", [False, True], ids=["host_channel", "device_channel"])
def test_kat_a(F, device_channel):
    kj = json.load(open(os.path.join(GOLDEN, "kat_a.json")))
    ka = _g("kat_a.npz")
    code = F.Code.array(47, 5)
    dec = F.Decoder(code, precheck=True)  # decode_fixpoint
    snr = 2 * math.pow(10.0, 4.5 / 10) * code.rate
    r = dec.ber_sim(snr, math.sqrt(1 / snr), info_index=ka["info_idx"], info_bits=ka["info_bits"],
                    codeword=ka["cw"], max_frame_errors=100, chunk=1024, device_channel=device_channel)
    assert (r["bit_errors"], r["frame_errors"], r["frames"]) == (kj["bit_errors"], kj["frame_errors"], kj["frames"])


@pytest.mark.parametrize("device_channel", [False, True], ids=["host_channel", "device_channel"])
def test_sim_two_chunks_in_flight_equals_serial(F, monkeypatch, device_channel):
    """fpldpc_ber_sim keeps two chunks in flight (two decoders on two streams, the next chunk
    submitted before this one is waited for); FPLDPC_SIM_OVERLAP=0 runs them one after another.  The
    counters are the same: a frame-error stop inside a chunk, with the chunk after it already
    decoded, and a frame-limit stop."""
    ka = _g("kat_a.npz")
    code = F.Code.array(47, 5)
    snr, sigma = F.snr_sigma(4.0, code.rate)
    dec = F.Decoder(code, precheck=True)
    for kw in (dict(max_frame_errors=37, chunk=512), dict(max_frame_errors=0, max_frames=5000, chunk=700)):
        res = {}
        for ov in ("0", "1"):
            monkeypatch.setenv("FPLDPC_SIM_OVERLAP", ov)
            res[ov] = dec.ber_sim(snr, sigma, info_index=ka["info_idx"], info_bits=ka["info_bits"], codeword=ka["cw"],
                                  device_channel=device_channel, **kw)
        for k in ("bit_errors", "frame_errors", "frames", "iter_sum"):
            assert res["0"][k] == res["1"][k], (k, res)
        assert res["1"]["frames_decoded"] >= res["1"]["frames"]
        print(kw, {ov: round(r["seconds"], 4) for ov, r in res.items()})


@pytest.mark.parametrize("device_channel", [False, True], ids=["host_channel", "device_channel"])
def test_count_iters_mode_and_shortening(F, O, codes, device_channel):
    """ArrayLDPC_PerfTest/TimeTrial count decode_fixpoint's return value as errors
    (PerfTest.cpp:507-510); ArrayLDPC_Debug_Shorten forces 7*16 at the first info positions
    (:410-414).  Both against the oracle frame by frame."""
    code, ocode = codes["A"]
    ka = _g("kat_a.npz")
    snr = 2 * math.pow(10.0, 4.0 / 10) * code.rate
    sigma = math.sqrt(1 / snr)
    dec = F.Decoder(code, precheck=True)
    r = dec.ber_sim(snr, sigma, max_frames=600, max_frame_errors=0, count_mode=F._lib.FPLDPC_COUNT_ITERS,
                    device_channel=device_channel)
    llr = O.gen_llr(SEED, 0, 600, code.n, snr, sigma, 4)
    ref = O.decode_batch(ocode, llr, precheck=True, want_post=False)
    assert r["bit_errors"] == int(ref["iters"].sum()) == r["iter_sum"]
    assert r["frame_errors"] == int((ref["iters"] > 0).sum())
    forced = ka["info_idx"][:976]
    r = dec.ber_sim(snr, sigma, info_index=ka["info_idx"], info_bits=ka["info_bits"], codeword=ka["cw"],
                    forced_index=forced, forced_llr=112, max_frames=500, max_frame_errors=0, chunk=128,
                    device_channel=device_channel)
    llr = O.gen_llr(SEED, 0, 500, code.n, snr, sigma, 4, cw=ka["cw"])
    llr[:, forced] = 112
    ref = O.decode_batch(ocode, llr, precheck=True, want_post=False)
    e = (ref["hard"][:, ka["info_idx"]] != ka["info_bits"][None, :]).sum(axis=1)
    assert (r["bit_errors"], r["frame_errors"], r["iter_sum"]) == (int(e.sum()), int((e > 0).sum()),
                                                                   int(ref["iters"].sum()))


def test_frames_w_vs_reference_fixtures(F, torch_dev):
    """GPU decode of the reference's own per-frame fixtures (no oracle in between)."""
    import torch
    g = _g("frames_w.npz")
    dec = F.Decoder(F.Code.wifi_1944_r12())
    for tag in ("m2", "p15", "p2", "rnd"):
        llr = torch.from_numpy(g[f"{tag}_llr"].astype(np.int32)).to(torch_dev)
        out = dec.decode_torch(llr, post=True)
        torch.cuda.synchronize()
        assert (out["iters"].cpu().numpy() == g[f"{tag}_iters"]).all(), tag
        hard = F.unpack_hard(out["hard"].cpu().numpy(), 1944)
        assert (np.packbits(hard, axis=1, bitorder="little") == g[f"{tag}_hard"]).all(), tag
        post = out["post"].cpu().numpy()
        crc = np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in post], np.uint32)
        assert (crc == g[f"{tag}_postcrc"]).all(), tag


def _check_gpu_frames(F, dec, g, tag, n, torch_dev):
    import torch
    llr = torch.from_numpy(g[f"{tag}_llr"]).to(torch_dev)  # int16 input, as the bench feeds it
    out = dec.decode_torch(llr, post=True)
    torch.cuda.synchronize()
    assert (out["iters"].cpu().numpy() == g[f"{tag}_iters"]).all(), tag
    hard = F.unpack_hard(out["hard"].cpu().numpy(), n)
    assert (np.packbits(hard, axis=1, bitorder="little") == g[f"{tag}_hard"]).all(), tag
    crc = np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in out["post"].cpu().numpy()], np.uint32)
    assert (crc == g[f"{tag}_postcrc"]).all(), tag


def test_frames_a_vs_reference_fixtures(F, torch_dev):
    """Config A (p47/r5, 30 it, mask 0xff): the reference's own per-frame decode_general_fp."""
    g = _g("frames_a.npz")
    dec = F.Decoder(F.Code.array(47, 5))
    for tag in ("e0", "e40", "e45", "e50", "rnd"):
        _check_gpu_frames(F, dec, g, tag, 2209, torch_dev)


def test_frames_r_vs_reference_fixtures(F, torch_dev):
    """Config R (p47/r24, 50 it, mask 0x3f): the reference's own per-frame decodes."""
    g = _g("frames_r.npz")
    dec = F.Decoder(F.Code.array(47, 24), max_iter=50, width_mask=0x3F)
    for tag in ("e2", "e5", "e8", "rnd"):
        _check_gpu_frames(F, dec, g, tag, 2209, torch_dev)


def test_fixpoint_a_vs_reference_fixtures(F):
    """decode_fixpoint (params.precheck = 1) against the reference's p47/r5 build frame by frame.
    Pre-check passes (the noiseless frames) return 0 with the channel hard decision and leave the
    posterior buffer untouched (the reference keeps the previous frame's Posteriori_fp,
    ArrayLDPC_Decoder.cpp:443-450); DecodeTrial's 100 frames (PerfTest.cpp:148-192) give the
    reference's return values and hard decisions."""
    g = _g("fixpoint_a.npz")
    code = F.Code.array(47, 5)
    dec = F.Decoder(code, precheck=True)
    for tag in ("x45", "x70"):
        llr = g[f"{tag}_llr"].astype(np.int32)
        sentinel = np.full(llr.shape, 0x5A5A5A5A, np.int32)
        out = dec.decode_host(llr, post=sentinel.copy())
        it = np.asarray(out["iters"])
        assert (it == g[f"{tag}_iters"]).all(), tag
        hard = F.unpack_hard(np.asarray(out["hard"]), 2209)
        assert (np.packbits(hard, axis=1, bitorder="little") == g[f"{tag}_hard"]).all(), tag
        post = out["post"]
        live = it > 0
        crc = np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in post], np.uint32)
        assert (crc[live] == g[f"{tag}_postcrc"][live]).all(), tag
        assert (post[~live] == 0x5A5A5A5A).all(), tag
    eb = float(g["trial_meta"][0])
    snr = 2 * math.pow(10.0, eb / 10) * code.rate
    llr = F.channel_llr(SEED, 0, 100, 2209, snr, math.sqrt(1 / snr), 4, dtype=np.int32)
    assert (np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in llr], np.uint32) == g["trial_llrcrc"]).all()
    out = dec.decode_host(llr)
    assert (np.asarray(out["iters"]) == g["trial_iters"]).all()
    hard = F.unpack_hard(np.asarray(out["hard"]), 2209)
    assert (np.packbits(hard, axis=1, bitorder="little") == g["trial_hard"]).all()
