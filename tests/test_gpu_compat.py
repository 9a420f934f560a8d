"""The drop-in C++ API frame by frame on the GPU (include/fpldpc_compat.hpp), against the reference's
own per-frame fixtures -- no oracle in between.

`fpldpc_perftest frames` runs the reference callers' sequence (PerfTest.cpp:121-130 and :505-507,
INTEGRATION.md §2): ReadH(path), setInfoBit, setInfoIndex, then per frame setState(PCV),
decode_general_fp / decode_fixpoint, resetBER (every `reset` frames only: calculateBER accumulates
until reset, ArrayLDPCMacro.h:146), calculateBER, getPost_fp(0..n-1).  decode_fixpoint's pre-check
passes return 0 and leave the previous frame's posteriors in place (ArrayLDPC_Decoder.cpp:443-450):
the fixture's posterior CRC of such a frame is its predecessor's, so every frame is compared.

Also ArrayLDPC_PerfTest (PerfTest.cpp:433-517) against the oracle's decode_fixpoint of the same
stream: it counts decode_fixpoint's return value (an iteration count) as bit errors and stops at the
100th frame whose return value is > 0."""
import math
import os
import re
import subprocess
import zlib

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
CLI = os.path.join(ROOT, "fixedpointldpc_amd", "fpldpc_perftest")
SEED = 123456789


def _frames(F, tmp_path, code, llr, fix, max_iter, mask, reset, fill=0):
    F.lib()
    alist = tmp_path / "H.txt"
    alist.write_text(code.write_alist())
    lf, of = tmp_path / "llr.bin", tmp_path / "out.bin"
    np.ascontiguousarray(llr, dtype="<i4").tofile(lf)
    p = subprocess.run([CLI, "frames", str(alist), str(lf), str(of), str(int(fix)), str(max_iter), hex(mask), str(reset),
                        hex(fill)],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    raw = np.fromfile(of, "<i4")
    k = int(raw[0])
    idx = raw[1:1 + k]
    rec = raw[1 + k:].reshape(len(llr), 2 + 2 * code.n)
    return idx, rec[:, 0], rec[:, 1], rec[:, 2:2 + code.n], rec[:, 2 + code.n:]


def _expect_ber(hard, idx, reset, bit):
    """calculateBER after each frame: errors over the info positions (info stream of all-`bit`
    bits), accumulated, cleared before frame f when f % reset == 0."""
    e = (hard[:, idx] != bit).astype(np.int64).sum(axis=1)
    out, acc = [], 0
    for f, x in enumerate(e):
        if f % reset == 0:
            acc = 0
        acc += int(x)
        out.append(acc)
    return np.array(out)


def _check(F, tmp_path, code, g, tags, fix, max_iter, mask, reset=3, fill=0):
    llr = np.concatenate([g[f"{t}_llr"] for t in tags]).astype(np.int32)
    want_it = np.concatenate([g[f"{t}_iters"] for t in tags])
    want_hard = np.concatenate([g[f"{t}_hard"] for t in tags])
    want_crc = np.concatenate([g[f"{t}_postcrc"] for t in tags])
    idx, it, ber, post, hard = _frames(F, tmp_path, code, llr, fix, max_iter, mask, reset, fill)
    assert (it == want_it).all(), np.nonzero(it != want_it)[0][:8]
    assert (np.packbits(hard.astype(np.uint8), axis=1, bitorder="little") == want_hard).all()
    crc = np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in post], np.uint32)
    bad = np.nonzero(crc != want_crc)[0]
    assert bad.size == 0, f"posterior mismatch at frames {bad[:8]}"
    off = 0
    for t in tags:  # full posteriors of each block's first two frames
        assert (post[off:off + 2] == g[f"{t}_post2"]).all(), t
        off += len(g[f"{t}_iters"])
    assert (ber == _expect_ber(hard, idx, reset, fill & 1)).all()
    assert ber.max() > 0, "the fixture frames must produce bit errors for calculateBER to be exercised"
    return it


def test_compat_frames_a_decode_general_fp(F, tmp_path):
    g = np.load(os.path.join(GOLDEN, "frames_a.npz"))
    _check(F, tmp_path, F.Code.array(47, 5), g, ("e0", "e40", "e45", "e50", "rnd"), False, 30, 0xFF)


def test_compat_frames_w_decode_general_fp(F, tmp_path):
    g = np.load(os.path.join(GOLDEN, "frames_w.npz"))
    _check(F, tmp_path, F.Code.wifi_1944_r12(), g, ("m2", "p15", "p2", "rnd"), False, 30, 0xFF)


def test_compat_frames_r_decode_general_fp(F, tmp_path):
    g = np.load(os.path.join(GOLDEN, "frames_r.npz"))
    _check(F, tmp_path, F.Code.array(47, 24), g, ("e2", "e5", "e8", "rnd"), False, 50, 0x3F)


def test_compat_fixpoint_keeps_previous_posteriors(F, tmp_path):
    """x45 / x70: AWGN frames with noiseless frames between them (pre-check passes).  Every frame
    decodes to the all-zero codeword here, so the info stream is all ones (0xff bytes): every info
    position is a bit error and calculateBER's accumulate-until-reset is still exercised."""
    g = np.load(os.path.join(GOLDEN, "fixpoint_a.npz"))
    it = _check(F, tmp_path, F.Code.array(47, 5), g, ("x45", "x70"), True, 30, 0xFF, reset=5, fill=0xFF)
    assert (it == 0).sum() >= 6 and (it > 0).sum() >= 6  # both paths exercised


def test_perftest_vs_oracle(O, codes, tmp_path):
    """fpldpc_perftest perftest 3.0 3.0 1 f.txt == the reference loop (PerfTest.cpp:485-512) run
    through the oracle's decode_fixpoint on the same channel stream."""
    import fixedpointldpc_amd as F
    F.lib()
    code, ocode = codes["A"]
    p = subprocess.run([CLI, "perftest", "3.0", "3.0", "1", "f.txt"], capture_output=True, text=True, timeout=300,
                       cwd=tmp_path)
    assert p.returncode == 0, p.stderr
    assert (tmp_path / "f.txt").exists() and (tmp_path / "f.txt_log.txt").exists()
    m = re.search(r"(\d+) (\d+) (\d+)\n FER: (\S+) BER: (\S+)$", p.stdout, re.M)
    assert m, p.stdout
    be, fe, fr = int(m.group(1)), int(m.group(2)), int(m.group(3))
    snr = 2 * math.pow(10.0, 3.0 / 10) * code.rate
    llr = O.gen_llr(SEED, 0, 400, code.n, snr, math.sqrt(1 / snr), 4)
    it = O.decode_batch(ocode, llr, precheck=True, want_post=False)["iters"]
    stop = int(np.nonzero(np.cumsum(it > 0) >= 100)[0][0])
    assert (be, fe, fr) == (int(it[:stop + 1].sum()), 100, stop + 1)
    assert m.group(4) == f"{100 / (stop + 1):g}"


def _fsm(F, tmp_path, llr, flags):
    F.lib()
    code = F.Code.array(47, 5)
    alist = tmp_path / "H.txt"
    alist.write_text(code.write_alist())
    lf, of = tmp_path / "llr.bin", tmp_path / "out.bin"
    np.ascontiguousarray(llr, dtype="<i4").tofile(lf)
    p = subprocess.run([CLI, "fsm", str(alist), str(lf), str(of), "30", "0xff", flags], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr
    return np.fromfile(of, "<i4"), p.stdout, code.n


@pytest.mark.parametrize("seq", ["", "c_"], ids=["fsm", "c2v_continuation"])
def test_compat_fsm_across_calls_vs_reference(F, tmp_path, seq):
    """decode_fixpoint's FSM across calls (ArrayLDPC_Decoder.cpp:443-488, :621-630) through the
    drop-in FP_Decoder against the reference's own run of the same sequence (tests/golden/fsm_a.npz,
    ref_a47r5 fsm): setState(PCV) before some frames only; per frame the return value, getState(),
    the hard decisions, the posterior CRC and the CRC of the edge RAM (getEdge_fp) the call left.
    Sequence 1: IDLE after a converged frame (the next call without PCV returns 0 with the channel
    decision and the previous posteriors), PCV kept by a pre-check pass, C2V after a 30-iteration
    frame.  Sequence c_: the C2V continuation -- no setState(PCV) after a frame that ended in C2V,
    so no edge init and the iterations run from the previous frame's edge RAM with the new LLRs
    (fpldpc_decode_frame, keep_edges = 1), ending in IDLE or C2V; a pre-check pass in C2V between
    them keeps the edge RAM."""
    g = np.load(os.path.join(GOLDEN, "fsm_a.npz"))
    flags = "".join(str(int(x)) for x in g[seq + "flags"])
    raw, _, n = _fsm(F, tmp_path, g[seq + "llr"].astype(np.int32), flags)
    e = 47 * 235
    rec = raw.reshape(len(flags), 2 * n + 2 + e)
    assert rec[:, 0].tolist() == g[seq + "iters"].tolist()
    assert rec[:, 1].tolist() == g[seq + "states"].tolist()
    hard = np.unpackbits(g[seq + "hard"], axis=1, bitorder="little")[:, :n]
    assert (rec[:, n + 2:2 * n + 2] == hard).all()
    crc = [zlib.crc32(r.astype("<i4").tobytes()) for r in rec[:, 2:n + 2]]
    assert crc == g[seq + "postcrc"].tolist()
    ecrc = [zlib.crc32(r.astype("<i4").tobytes()) for r in rec[:, 2 * n + 2:]]
    assert ecrc == g[seq + "edgecrc"].tolist()
    if seq:
        f0 = int(g["c_cont"][0])
        assert (rec[f0, 2 * n + 2:] == g["c_edge_first_cont"].ravel()).all()
        assert len(g["c_cont"]) >= 5 and {int(g["c_states"][f]) for f in g["c_cont"]} == {0, 4}


# (code, MAX_ITER, WIDTH_MASK, Eb/N0): A / W / R run flood_edges<48> / <8> / <48>; the array codes
# p13 / p31 / p59 have check degree 13 / 31 / 59, the kernel's DC = 16 / 32 / 64 instances
EDGE_CASES = [("A", 30, 0xFF, 4.0), ("W", 30, 0xFF, 1.5), ("R", 50, 0x3F, 4.0), ((13, 5), 30, 0xFF, 3.0),
              ((31, 4), 20, 0x7F, 4.0), ((59, 3), 20, 0xFF, 5.0)]


@pytest.mark.parametrize("key,max_iter,mask,eb", EDGE_CASES,
                         ids=["A", "W", "R", "p13r5_dc16", "p31r4_dc32", "p59r3_dc64"])
def test_decode_frame_keep_edges_vs_oracle(F, O, codes, key, max_iter, mask, eb):
    """fpldpc_decode_frame_host directly, on A, W, R and array codes of check degree 13, 31 and 59
    (every flood_edges<DC> instance: DC = 8 / 16 / 32 / 48 / 64): a frame that fails (random LLRs, so
    MAX_ITER iterations), then continuations with keep_edges = 1 on AWGN frames -- iterations, hard
    decisions, syndrome flag, posteriors and the whole edge RAM against the oracle's edge-RAM decode
    (oracle.FSMDecoder's decode_general_fp / decode_fixpoint steps); the W code exercises irregular
    check degrees (slots past a check's degree stay untouched)."""
    import ctypes
    rs = np.random.default_rng(5)
    if isinstance(key, tuple):
        code = F.Code.array(*key)
        ocode = O.OracleCode.from_alist_text(code.write_alist())
        key = f"p{key[0]}r{key[1]}"
    else:
        code, ocode = codes[key]
    rate = 0.5 if key == "W" else code.rate
    snr, sigma = F.snr_sigma(eb, rate)
    frames = [rs.integers(-40, 41, code.n).astype(np.int32)] + list(O.gen_llr(SEED, 0, 3, code.n, snr, sigma))
    for precheck in (False, True):
        dec = F.Decoder(code, max_iter=max_iter, width_mask=mask, precheck=precheck)
        od = O.FSMDecoder(ocode, max_iter=max_iter, mask=mask)
        words = ctypes.c_int64()
        F._lib._check(F.lib().fpldpc_edge_ram_words(dec._h, ctypes.byref(words)))
        assert words.value == code.dc_max * code.m == od.edge.size
        edge = np.zeros(words.value, np.int32)
        post = np.zeros(code.n, np.int32)
        for f, llr in enumerate(frames):
            keep = f > 0
            hard = np.zeros(dec.hard_words, np.uint32)
            it, ok = np.zeros(1, np.int32), np.zeros(1, np.uint8)
            F._lib._check(F.lib().fpldpc_decode_frame_host(dec._h, F._lib._ptr(np.ascontiguousarray(llr)), int(keep),
                                                           F._lib._ptr(edge), F._lib._ptr(hard), F._lib._ptr(it),
                                                           F._lib._ptr(ok), F._lib._ptr(post)))
            if precheck:
                od.state = O.C2V if keep else O.PCV
                want = od.decode_fixpoint(llr)
                want_ok = it[0] == 0 or od.state == O.IDLE
            else:
                want, want_ok = od._run(O.lib().orc_decode_general_edges, llr, keep)
            where = f"{key} precheck={precheck} frame {f}"
            assert it[0] == want and bool(ok[0]) == bool(want_ok), where
            assert (F.unpack_hard(hard[None], code.n)[0] == od.hard).all(), where
            assert (post == od.post).all() and (edge == od.edge).all(), where
        assert it[0] > 0

