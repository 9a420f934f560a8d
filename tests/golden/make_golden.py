#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs only in the build container, where /root/reference exists.  The reference's own sources
(ArrayLDPC_Decoder.cpp, ArrayLDPC_Encoder.cpp, rngs.cpp, rvgs.cpp) are compiled unmodified where
they lie by oracle/Makefile into oracle/_ref/ref_wifi (our driver oracle/ref_driver.cpp around
them); every decode / RNG / sxor vector below is that binary's output.  Data files the reference
holds (alist H files, G files, the published result) are read as data.

Fixtures written (all small; tests read them, nothing reads /root/reference at test time):
  rng.json            TestRandom verdict, first 64 Lehmer states and Normal(0,1) values from the
                      default seed 123456789 (rngs.cpp:45), state after 10000 draws from seed 1.
  sxor_ff.npz         sxor(x, y) at FRAC 4 / mask 0xff: full table on [-96, 96]^2, 20000 sampled
                      pairs on [-4096, 4096]^2, SHA-256 of the full int32 table on [-1024, 1024]^2.
  codes.json          token-stream SHA-256 + dims of the three hot-path alist files.
  kat_w.npz / .json   KAT-W: codeword + info positions/bits of ArrayLDPC_Debug_Wifi
                      (PerfTest.cpp:33-96), the published line (wifi_results_4_4_2dB_30iter.txt)
                      and the reference's cumulative (bit errors, frame errors) every 10000 frames.
  frames_w.npz        per-frame reference decodes on the WiFi code (decode_general_fp, 30 it,
                      Q4.4, mask 0xff): AWGN frames at -2 / 1.5 / 2 dB from the KAT stream and
                      random-LLR frames (mask wrap, sgn(0), large magnitudes).
  float_w.npz         the floating-point decoder decode_general (ArrayLDPC_Decoder.cpp:735-933) on
                      the WiFi code: per-frame iterations / hard bits / CRC of the float64
                      posteriors for unquantised AWGN frames at 0 / 1 / 2 dB, and
                      sxor(double, double) (:724-732) on sampled and edge-case pairs.
  kat_a.npz / .json   KAT-A inputs: the array-code codeword ArrayLDPC_Debug encodes
                      (PerfTest.cpp:221-262, G_array_forward.txt, ArrayLDPC_Encoder.cpp:160-225)
                      and the reference's result 2515 / 100 / 2108 at 4.5 dB, re-run here by
                      oracle/_ref/ref_a47r5 kat_a (with cumulative checkpoints every 250 frames).

Array-code fixtures (oracle/_ref/ref_a47r5, ref_a47r24: the same unmodified sources with the
dimension enums of ArrayLDPCMacro.h substituted by oracle/ref_dims.sh):
  frames_a.npz        p47/r5, 30 it, mask 0xff, decode_general_fp on the alist: all-zero-codeword
                      AWGN frames (PerfTest.cpp:587-590 channel, rate = getRate()) at 0 / 4.0 /
                      4.5 / 5.0 dB and random-LLR frames.
  fixpoint_a.npz      p47/r5 decode_fixpoint (ROM addressing + hardDecision pre-check,
                      ArrayLDPC_Decoder.cpp:422-639, :270-294): AWGN frames at 4.5 / 7 dB with
                      noiseless (pre-check passing) frames interleaved, and DecodeTrial
                      (PerfTest.cpp:148-192) at 4.5 dB: 200 packets over its 100 tiled frames.
  frames_r.npz        p47/r24, 50 it, mask 0x3f (BASELINE config R): AWGN frames at 2 / 5 / 8 dB
                      and random-LLR frames.
  sxor_3f.npz         sxor at FRAC 4 / mask 0x3f (ref_a47r24): full-table SHA-256 on
                      [-1024, 1024]^2, [-96, 96]^2 element-wise, 20000 pairs on [-4096, 4096]^2.
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_wifi")
REF_A = os.path.join(ROOT, "oracle", "_ref", "ref_a47r5")
REF_R = os.path.join(ROOT, "oracle", "_ref", "ref_a47r24")
N_W, K_W = 1944, 972
N_A = 2209


def run(*args, binary=REF_BIN, **kw):
    return subprocess.run([binary, *map(str, args)], check=True, capture_output=True, text=True, **kw).stdout


def ref_decode(binary, alist, llr, fixpoint=False):
    """Per-frame reference decode (ref_driver decode): iterations, posteriors, hard decisions."""
    n = llr.shape[1]
    with tempfile.TemporaryDirectory() as td:
        lp, op = os.path.join(td, "l.bin"), os.path.join(td, "o.bin")
        np.ascontiguousarray(llr, np.int32).tofile(lp)
        run("decode", alist, lp, len(llr), op, int(fixpoint), binary=binary)
        rec = np.fromfile(op, np.int32).reshape(len(llr), 2 * n + 1)
    return rec[:, 0].copy(), rec[:, 1:n + 1].copy(), rec[:, n + 1:].astype(np.uint8)


def ref_chan(binary, eb, nframes, skip, rate=0.0):
    """The reference harness's all-zero-codeword LLRs (ref_driver chan), int32 [nframes][n]."""
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "c.bin")
        run("chan", eb, rate, nframes, skip, p, binary=binary)
        return np.fromfile(p, np.int32).reshape(nframes, -1)


def frame_record(out, tag, llr, iters, post, hard, meta):
    out[f"{tag}_llr"] = llr.astype(np.int16)
    assert (out[f"{tag}_llr"] == llr).all(), "LLR exceeds int16"
    out[f"{tag}_iters"] = iters
    out[f"{tag}_hard"] = np.packbits(hard, axis=1, bitorder="little")
    out[f"{tag}_postcrc"] = np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in post], np.uint32)
    out[f"{tag}_post2"] = post[:2].copy()
    out[f"{tag}_meta"] = np.array(meta, np.float64)


def alist_tokens(path):
    with open(path) as f:
        return [int(x) for x in f.read().split()]


def token_sha(tokens):
    return hashlib.sha256(" ".join(map(str, tokens)).encode()).hexdigest()


def c_string_literal(path, anchor_line_re, decl):
    """Return the bytes of the first `decl = "..."` literal after the line matching anchor_line_re,
    with C translation phase 2 (backslash-newline splicing) applied."""
    src = open(path, "rb").read().decode("latin-1")
    m = re.search(anchor_line_re, src, re.M)
    assert m, anchor_line_re
    i = src.index(decl, m.end())
    i = src.index('"', i) + 1
    out = []
    while True:
        c = src[i]
        if c == "\\" and src[i + 1] == "\n":
            i += 2
            continue
        if c == "\\" and src[i + 1:i + 3] == "\r\n":
            i += 3
            continue
        assert c != "\\", "escape sequences not expected in this literal"
        if c == '"':
            break
        out.append(c)
        i += 1
    return "".join(out).encode("latin-1")


def unpack_info(stream, in_len, k):
    """setInfoBit / FP_Encoder::encode bit unpacking (ArrayLDPC_Decoder.cpp:178-197,
    ArrayLDPC_Encoder.cpp:181-196): LSB-first bytes 0..in_len-2, then k % 8 bits of the last."""
    buf = stream.ljust(in_len, b"\0")
    bits = []
    for i in range(in_len - 1):
        bits += [(buf[i] >> j) & 1 for j in range(8)]
    bits += [(buf[in_len - 1] >> j) & 1 for j in range(k % 8)]
    return np.array(bits[:k], np.uint8)


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)

    # ---------------------------------------------------------------- RNG
    out = run("rng", 64).splitlines()
    rng = {"test_random_ok": any("is correct" in l for l in out),
           "states": [int(l.split()[1]) for l in out if l.startswith("state ")],
           "normals_hex": [l.split()[1] for l in out if l.startswith("normal ")],
           "normals": [float.fromhex(l.split()[1]) for l in out if l.startswith("normal ")],
           "seed1_after_10000": int([l for l in out if l.startswith("seed1_after")][0].split()[1]),
           "source": "oracle/_ref/ref_wifi rng 64 (rngs.cpp, rvgs.cpp compiled unmodified)"}
    json.dump(rng, open(os.path.join(HERE, "rng.json"), "w"), indent=1)

    # ---------------------------------------------------------------- sxor
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "t.bin")
        run("sxor", -1024, 1024, p)
        full = np.fromfile(p, np.int32).reshape(2049, 2049)
        sha = hashlib.sha256(full.astype("<i4").tobytes()).hexdigest()
        small = full[1024 - 96:1024 + 97, 1024 - 96:1024 + 97].copy()
        run("sxor", -4096, 4096, p)
        big = np.fromfile(p, np.int32).reshape(8193, 8193)
        rs = np.random.default_rng(2024)
        xs = rs.integers(-4096, 4097, 20000)
        ys = rs.integers(-4096, 4097, 20000)
        samp = big[xs + 4096, ys + 4096]
    np.savez_compressed(os.path.join(HERE, "sxor_ff.npz"), small=small, small_lo=-96, xs=xs.astype(np.int32),
                        ys=ys.astype(np.int32), zs=samp.astype(np.int32), full_sha256=sha, full_lo=-1024, full_hi=1024)

    # ---------------------------------------------------------------- codes
    codes = {}
    for key, rel in (("A", "H_array_p47_r5_forward.txt"), ("W", "H_802.11_IndZero.txt"),
                     ("R", "codes/H_array_p47_r24_forward.txt")):
        t = alist_tokens(os.path.join(REF, rel))
        codes[key] = {"file": rel, "n": t[0], "m": t[1], "dv_max": t[2], "dc_max": t[3],
                      "tokens": len(t), "token_sha256": token_sha(t)}
    json.dump(codes, open(os.path.join(HERE, "codes.json"), "w"), indent=1)

    # ---------------------------------------------------------------- KAT-W inputs
    lines = run("codeword").splitlines()
    cw = np.array(lines[0].split(), np.uint8)
    info_idx = np.array(lines[1].split(), np.int32)
    info_str = c_string_literal(os.path.join(REF, "PerfTest.cpp"), r"^int ArrayLDPC_Debug_Wifi\(\)",
                                "char InfoStream[122]")
    info_bits = unpack_info(info_str, 122, K_W)
    assert cw.shape == (N_W,) and info_idx.shape == (K_W,)
    assert (cw[info_idx] == info_bits).all(), "systematic encoder: codeword info positions carry the info bits"
    np.savez_compressed(os.path.join(HERE, "kat_w.npz"), cw=cw, info_idx=info_idx, info_bits=info_bits)
    pub = open(os.path.join(REF, "wifi_results_4_4_2dB_30iter.txt")).read()
    kat_w = {"ebn0_db": 2.0, "max_iter": 30, "frac_bits": 4, "mask": 255, "rate_used": 0.5,
             "published_text": pub}
    m = re.search(r"(\d+)\s+(\d+)\s+(\d+)\s*\n\s*FER:\s*(\S+)\s+BER:\s*(\S+)", pub)
    kat_w.update(bit_errors=int(m.group(1)), frame_errors=int(m.group(2)), frames=int(m.group(3)),
                 fer_text=m.group(4), ber_text=m.group(5))
    ck = "/tmp/katw_ref.txt"  # `ref_wifi kat_w 2 -1 10000` (about 5 min); regenerated if absent
    if not os.path.exists(ck) or "FER" not in open(ck).read():
        with open(ck, "w") as f:
            subprocess.run([REF_BIN, "kat_w", "2", "-1", "10000"], check=True, stdout=f)
    ckl = open(ck).read().splitlines()
    kat_w["checkpoints"] = [[int(x) for x in l.split()[1:]] for l in ckl if l.startswith("checkpoint")]
    final = [l for l in ckl if not l.startswith("checkpoint")][0].split()
    kat_w["reference_rerun"] = [int(final[0]), int(final[1]), int(final[2])]
    assert kat_w["reference_rerun"] == [kat_w["bit_errors"], kat_w["frame_errors"], kat_w["frames"]]
    kat_w["source"] = "published: wifi_results_4_4_2dB_30iter.txt; checkpoints: oracle/_ref/ref_wifi kat_w 2 -1 10000"
    json.dump(kat_w, open(os.path.join(HERE, "kat_w.json"), "w"), indent=1)

    # ---------------------------------------------------------------- per-frame WiFi goldens
    fw = {}
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "f.bin")
        for tag, eb, nfr, skip in (("m2", -2.0, 24, 500), ("p15", 1.5, 32, 2000), ("p2", 2.0, 32, 0)):
            run("frames", eb, nfr, skip, 1, p)
            rec = np.fromfile(p, np.int32).reshape(nfr, 2 * N_W + 1)
            fw[f"{tag}_llr"] = rec[:, :N_W].astype(np.int16)
            fw[f"{tag}_iters"] = rec[:, N_W].copy()
            post = rec[:, N_W + 1:]
            fw[f"{tag}_hard"] = np.packbits((post <= 0).astype(np.uint8), axis=1, bitorder="little")
            fw[f"{tag}_postcrc"] = np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in post], np.uint32)
            fw[f"{tag}_post2"] = post[:2].copy()
            fw[f"{tag}_meta"] = np.array([eb, nfr, skip], np.float64)
        # random (non-channel) LLRs through the reference decoder: wrap of the masked sum and
        # difference, sgn(0) = -1 ties, post = 0 -> bit 1, large magnitudes
        rs = np.random.default_rng(99)
        llr = np.concatenate([rs.integers(-300, 301, (8, N_W)), rs.integers(-32768, 32768, (8, N_W)),
                              rs.integers(-3, 4, (8, N_W)), rs.integers(-40, 41, (8, N_W))]).astype(np.int32)
        it, post, hard = ref_decode(REF_BIN, os.path.join(REF, "H_802.11_IndZero.txt"), llr)
        assert (hard == (post <= 0)).all()
        fw["rnd_llr"] = llr.astype(np.int16)
        fw["rnd_iters"] = it
        fw["rnd_hard"] = np.packbits(hard, axis=1, bitorder="little")
        fw["rnd_postcrc"] = np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in post], np.uint32)
        fw["rnd_post2"] = post[:2].copy()
    np.savez_compressed(os.path.join(HERE, "frames_w.npz"), **fw)

    # ---------------------------------------------------------------- KAT-A inputs
    # G file (ArrayLDPC_Encoder.cpp:45-83): N M_G / x cmax / ColumnFlag[N] / ChkDeg[M_G] / rows.
    t = alist_tokens(os.path.join(REF, "codes", "G_array_forward.txt"))
    n, mg = t[0], t[1]
    i = 4
    flag = np.array(t[i:i + n]); i += n
    deg = t[i:i + mg]; i += mg
    rows = []
    for d in deg:
        rows.append(t[i:i + d]); i += d
    assert i == len(t)
    info_pos = np.nonzero(flag == 0)[0].astype(np.int32)
    par_pos = np.nonzero(flag == 1)[0]
    k_a = n - mg
    assert len(info_pos) == k_a == 1978
    s = c_string_literal(os.path.join(REF, "PerfTest.cpp"), r"^int ArrayLDPC_Debug\(\)", "char InfoStream[248]")
    assert len(s) <= 248, len(s)
    bits_a = unpack_info(s, 248, k_a)
    cw_a = np.zeros(n, np.uint8)
    cw_a[info_pos] = bits_a  # encode(), ArrayLDPC_Encoder.cpp:197-200
    for r, row in enumerate(rows):  # :211-223, parity r = XOR of the info vars in G row r
        acc = 0
        for v in row:
            if flag[v] == 0:
                acc ^= int(cw_a[v])
        cw_a[par_pos[r]] = acc
    # the codeword must satisfy the array H (forward shift)
    th = alist_tokens(os.path.join(REF, "H_array_p47_r5_forward.txt"))
    nn, mm = th[0], th[1]
    j = 4 + nn + mm + sum(th[4:4 + nn])
    cdeg = th[4 + nn:4 + nn + mm]
    for r in range(mm):
        assert sum(int(cw_a[v]) for v in th[j:j + cdeg[r]]) % 2 == 0
        j += cdeg[r]
    np.savez_compressed(os.path.join(HERE, "kat_a.npz"), cw=cw_a, info_idx=info_pos, info_bits=bits_a)
    kat_a(s)
    print("golden fixtures written to", HERE)


def kat_a(info_stream):
    """KAT-A re-run on the reference (ref_a47r5 kat_a: ArrayLDPC_Debug, PerfTest.cpp:217-316)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    with tempfile.TemporaryDirectory() as td:
        ip = os.path.join(td, "info.bin")
        open(ip, "wb").write(info_stream.ljust(248, b"\0"))
        out = run("kat_a", 4.5, ip, 250, binary=REF_A).splitlines()
    ck = [[int(x) for x in l.split()[1:]] for l in out if l.startswith("checkpoint")]
    final = [int(x) for x in [l for l in out if not l.startswith("checkpoint")][0].split()]
    assert final == [2515, 100, 2108], final
    json.dump({"ebn0_db": 4.5, "max_iter": 30, "frac_bits": 4, "mask": 255, "decoder": "decode_fixpoint (pre-check)",
               "rate": "ROM::getRate = 1 - (r*p - r + 1)/p^2", "bit_errors": final[0], "frame_errors": final[1],
               "frames": final[2], "checkpoints": ck,
               "source": "oracle/_ref/ref_a47r5 kat_a 4.5 (ArrayLDPC_Debug, PerfTest.cpp:217-316, restated around the "
                         "reference sources built with the p47/r5 enum by oracle/ref_dims.sh); matches SURVEY.md's "
                         "measurement; inputs regenerated here from G_array_forward.txt"},
              open(os.path.join(HERE, "kat_a.json"), "w"), indent=1)


def sxor_table_fixture(binary, name):
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "t.bin")
        run("sxor", -1024, 1024, p, binary=binary)
        full = np.fromfile(p, np.int32).reshape(2049, 2049)
        sha = hashlib.sha256(full.astype("<i4").tobytes()).hexdigest()
        small = full[1024 - 96:1024 + 97, 1024 - 96:1024 + 97].copy()
        run("sxor", -4096, 4096, p, binary=binary)
        big = np.fromfile(p, np.int32).reshape(8193, 8193)
        rs = np.random.default_rng(2024)
        xs = rs.integers(-4096, 4097, 20000)
        ys = rs.integers(-4096, 4097, 20000)
        samp = big[xs + 4096, ys + 4096]
    np.savez_compressed(os.path.join(HERE, name), small=small, small_lo=-96, xs=xs.astype(np.int32),
                        ys=ys.astype(np.int32), zs=samp.astype(np.int32), full_sha256=sha, full_lo=-1024, full_hi=1024)


def array_goldens():
    """frames_a.npz, fixpoint_a.npz, frames_r.npz, sxor_3f.npz from the array-dimension builds."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    for b, want in ((REF_A, "NUM_CHK 235 NUM_CGRP 5 NUM_VGRP 47 CHK_DEG 47 VAR_DEG 5 P 47 INFO_LENGTH 1978 "
                             "CWD_LENGTH 2209 MAX_ITER 30 WIDTH_MASK 255 FRAC_WIDTH 4"),
                    (REF_R, "NUM_CHK 1128 NUM_CGRP 24 NUM_VGRP 47 CHK_DEG 47 VAR_DEG 24 P 47 INFO_LENGTH 1128 "
                            "CWD_LENGTH 2209 MAX_ITER 50 WIDTH_MASK 63 FRAC_WIDTH 4")):
        assert want in run("dims", binary=b), (b, run("dims", binary=b))
    h_a = os.path.join(REF, "H_array_p47_r5_forward.txt")
    h_r = os.path.join(REF, "codes", "H_array_p47_r24_forward.txt")

    # ---- p47/r5, decode_general_fp
    fa = {}
    for tag, eb, nfr, skip in (("e0", 0.0, 16, 0), ("e40", 4.0, 16, 64), ("e45", 4.5, 16, 128), ("e50", 5.0, 16, 192)):
        llr = ref_chan(REF_A, eb, nfr, skip)
        it, post, hard = ref_decode(REF_A, h_a, llr)
        assert (hard == (post <= 0)).all()
        frame_record(fa, tag, llr, it, post, hard, [eb, nfr, skip])
    rs = np.random.default_rng(47)
    llr = np.concatenate([rs.integers(-300, 301, (4, N_A)), rs.integers(-32768, 32768, (4, N_A)),
                          rs.integers(-3, 4, (4, N_A)), rs.integers(-40, 41, (4, N_A))]).astype(np.int32)
    it, post, hard = ref_decode(REF_A, h_a, llr)
    frame_record(fa, "rnd", llr, it, post, hard, [0, len(llr), 0])
    np.savez_compressed(os.path.join(HERE, "frames_a.npz"), **fa)

    # ---- p47/r5, decode_fixpoint: AWGN frames with noiseless (pre-check passing) frames between
    fx = {}
    for tag, eb, nfr, skip in (("x45", 4.5, 16, 256), ("x70", 7.0, 16, 320)):
        llr = ref_chan(REF_A, eb, nfr, skip)
        snr = 2 * 10 ** (eb / 10) * float.fromhex(run("dims", binary=REF_A).split("rate ")[1].strip())
        clean = np.full(N_A, int(2 * snr * 16), np.int32)  # noiseless all-zero codeword (PerfTest.cpp:279)
        llr[1::4] = clean
        it, post, hard = ref_decode(REF_A, h_a, llr, fixpoint=True)
        assert (it[1::4] == 0).all()
        frame_record(fx, tag, llr, it, post, hard, [eb, nfr, skip])
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "d.bin")
        run("decodetrial", 4.5, 200, p, binary=REF_A)
        rec = np.fromfile(p, np.int32).reshape(200, N_A + 1)
    assert (rec[100:] == rec[:100]).all()  # the second pass over the 100 tiled frames repeats the first
    fx["trial_iters"] = rec[:100, 0].copy()
    fx["trial_hard"] = np.packbits(rec[:100, 1:].astype(np.uint8), axis=1, bitorder="little")
    fx["trial_meta"] = np.array([4.5, 100, 0], np.float64)
    fx["trial_llrcrc"] = np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in ref_chan(REF_A, 4.5, 100, 0)],
                                  np.uint32)
    np.savez_compressed(os.path.join(HERE, "fixpoint_a.npz"), **fx)

    # ---- p47/r24, 50 it, mask 0x3f
    fr = {}
    for tag, eb, nfr, skip in (("e2", 2.0, 12, 0), ("e5", 5.0, 12, 40), ("e8", 8.0, 12, 80)):
        llr = ref_chan(REF_R, eb, nfr, skip)
        it, post, hard = ref_decode(REF_R, h_r, llr)
        assert (hard == (post <= 0)).all()
        frame_record(fr, tag, llr, it, post, hard, [eb, nfr, skip])
    rs = np.random.default_rng(24)
    llr = np.concatenate([rs.integers(-300, 301, (3, N_A)), rs.integers(-32768, 32768, (3, N_A)),
                          rs.integers(-3, 4, (3, N_A)), rs.integers(-40, 41, (3, N_A))]).astype(np.int32)
    it, post, hard = ref_decode(REF_R, h_r, llr)
    frame_record(fr, "rnd", llr, it, post, hard, [0, len(llr), 0])
    np.savez_compressed(os.path.join(HERE, "frames_r.npz"), **fr)
    sxor_table_fixture(REF_R, "sxor_3f.npz")
    print("array-code fixtures written to", HERE)


def float_w():
    """float_w.npz: the reference's floating-point decoder, frame by frame (ref_driver float_frames)."""
    fw = {}
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "f.bin")
        for tag, eb, nfr, skip, use_cw in (("f0", 0.0, 24, 100, 0), ("f1", 1.0, 48, 0, 1), ("f2", 2.0, 48, 3000, 1)):
            run("float_frames", eb, nfr, skip, use_cw, p)
            rec = np.fromfile(p, np.uint8).reshape(nfr, N_W * 16 + 4)
            llr = rec[:, :N_W * 8].copy().view(np.float64)
            post = rec[:, N_W * 8 + 4:].copy().view(np.float64)
            fw[f"{tag}_iters"] = rec[:, N_W * 8:N_W * 8 + 4].copy().view(np.int32).ravel()
            fw[f"{tag}_hard"] = np.packbits((post <= 0).astype(np.uint8), axis=1, bitorder="little")
            fw[f"{tag}_postcrc"] = np.array([zlib.crc32(r.astype("<f8").tobytes()) for r in post], np.uint32)
            fw[f"{tag}_llrcrc"] = np.array([zlib.crc32(r.astype("<f8").tobytes()) for r in llr], np.uint32)
            fw[f"{tag}_post2"] = post[:2].copy()
            fw[f"{tag}_meta"] = np.array([eb, nfr, skip, use_cw], np.float64)
        rs = np.random.default_rng(7)
        xy = np.concatenate([
            rs.normal(0, 4, (3000, 2)), rs.normal(0, 40, (500, 2)), rs.uniform(-1e-3, 1e-3, (300, 2)),
            np.array([[0.0, 1.0], [1.0, 0.0], [-0.0, 2.0], [0.0, -0.0], [3.0, 3.0], [-3.0, 3.0], [3.0, -3.0],
                      [800.0, 2.0], [2.0, -800.0], [800.0, 800.0], [1e-300, 5.0], [-1e-300, -5.0], [40.0, 40.0],
                      [36.7, 36.7], [0.5, 0.5000000000000001]])])
        ip, op = os.path.join(td, "xy.bin"), os.path.join(td, "r.bin")
        xy.astype("<f8").tofile(ip)
        run("sxor_f64", ip, len(xy), op)
        fw["sxor_xy"] = xy
        fw["sxor_r"] = np.fromfile(op, "<f8")
    np.savez_compressed(os.path.join(HERE, "float_w.npz"), **fw)
    print("float_w.npz written")


def _fsm_run(h_a, llr, flags):
    """ref_a47r5 fsm: per frame (iterations, FSM state, post, hard, edge RAM [47][235])."""
    E = 47 * 235
    with tempfile.TemporaryDirectory() as td:
        lp, op = os.path.join(td, "l.bin"), os.path.join(td, "o.bin")
        llr.tofile(lp)
        run("fsm", h_a, lp, len(llr), op, flags, binary=REF_A)
        rec = np.fromfile(op, np.int32).reshape(len(llr), 2 * N_A + 2 + E)
    return (rec[:, 0], rec[:, 1], rec[:, 2:N_A + 2], rec[:, N_A + 2:2 * N_A + 2].astype(np.uint8),
            rec[:, 2 * N_A + 2:])


def _crc(rows):
    return np.array([zlib.crc32(r.astype("<i4").tobytes()) for r in rows], np.uint32)


def fsm_golden():
    """fsm_a.npz: decode_fixpoint's FSM across calls on ref_a47r5 (ArrayLDPC_Decoder.cpp:443-488,
    :621-630): setState(PCV) before some frames only.
    Sequence 1 (keys without prefix): IDLE after a converged frame (the next call without PCV
    returns 0: channel decision, previous posteriors), PCV kept by a pre-check pass, C2V after a
    frame that runs all MAX_ITER iterations (a pre-check pass then returns 0).
    Sequence 2 (keys c_*): the C2V continuation -- after a frame that ends in C2V, calls without
    setState(PCV) whose pre-check fails iterate from the edge RAM the previous decode left
    (:462 skips the edge init, :488 runs the loop), ending in IDLE or again in C2V; a pre-check pass
    in between leaves the edge RAM alone.  Every frame also records the edge RAM's CRC (and the
    full RAM of the continuation frames), so the edge state itself is pinned."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    h_a = os.path.join(REF, "H_array_p47_r5_forward.txt")
    noisy = ref_chan(REF_A, 4.5, 8, 512)
    rate = float.fromhex(run("dims", binary=REF_A).split("rate ")[1].strip())
    snr = 2 * 10 ** (4.5 / 10) * rate
    clean = np.full(N_A, int(2 * snr * 16), np.int32)
    rnd = np.random.default_rng(7).integers(-40, 41, N_A).astype(np.int32)
    frames = [noisy[0], noisy[1], clean, clean, noisy[2], rnd, clean, noisy[3], noisy[4]]
    flags = "100101010"
    want = [0, 0, 0, 1, 0, 4, 4, 0, 0]  # FSM state after each call (IDLE 0, PCV 1, C2V 4)
    llr = np.stack(frames).astype(np.int32)
    it, st, post, hard, edge = _fsm_run(h_a, llr, flags)
    assert st.tolist() == want, st.tolist()
    assert it[1] == 0 and it[2] == 0 and it[3] == 0 and it[5] == 30 and it[8] == 0 and it[0] > 0, it.tolist()
    assert (post[1] == post[0]).all() and (hard[1] == (llr[1] <= 0)).all()
    out = {"llr": llr.astype(np.int16), "flags": np.frombuffer(flags.encode(), np.uint8) - ord("0"),
           "iters": it.copy(), "states": st.copy(), "hard": np.packbits(hard, axis=1, bitorder="little"),
           "postcrc": _crc(post), "edgecrc": _crc(edge)}
    assert (out["llr"] == llr).all()
    # Sequence 2: frames that fail at 30 iterations (random LLRs; AWGN at 2.5 dB) followed by
    # no-PCV calls on AWGN frames at 4.5 / 3.5 dB and random LLRs
    low = ref_chan(REF_A, 2.5, 6, 900)
    mid = ref_chan(REF_A, 3.5, 6, 1200)
    rs = np.random.default_rng(11)
    rnds = [rs.integers(-40, 41, N_A).astype(np.int32) for _ in range(3)]
    cframes = [rnd, noisy[5], rnds[0], rnds[1], clean, noisy[6], low[0], mid[0], mid[1], low[1], low[2], noisy[7],
               rnds[2], mid[2], low[3], rnd, clean, rnds[0]]
    cflags = "100000110010100100"
    cllr = np.stack(cframes).astype(np.int32)
    cit, cst, cpost, chard, cedge = _fsm_run(h_a, cllr, cflags)
    cont = [f for f in range(len(cflags)) if cflags[f] == "0" and f > 0 and cst[f - 1] == 4 and cit[f] > 0]
    ends = {int(cst[f]) for f in cont}
    assert len(cont) >= 5 and ends == {0, 4}, (cit.tolist(), cst.tolist())
    # a pre-check pass in state C2V keeps the state and the edge RAM, and the next call continues
    assert cit[16] == 0 and cst[16] == 4 and (cedge[16] == cedge[15]).all() and 17 in cont
    out.update({"c_llr": cllr.astype(np.int16), "c_flags": np.frombuffer(cflags.encode(), np.uint8) - ord("0"),
                "c_iters": cit.copy(), "c_states": cst.copy(), "c_hard": np.packbits(chard, axis=1, bitorder="little"),
                "c_postcrc": _crc(cpost), "c_edgecrc": _crc(cedge), "c_cont": np.array(cont, np.int32),
                "c_edge_first_cont": cedge[cont[0]].astype(np.int32), "c_post_first_cont": cpost[cont[0]].astype(np.int32)})
    assert (out["c_llr"] == cllr).all()
    np.savez_compressed(os.path.join(HERE, "fsm_a.npz"), **out)
    print("fsm_a.npz:", "iters", it.tolist(), "states", st.tolist())
    print("  continuation:", "iters", cit.tolist(), "states", cst.tolist(), "continued frames", cont)


if __name__ == "__main__":
    if "--float-only" in sys.argv:
        sys.exit(float_w())
    if "--array-only" in sys.argv:
        sys.exit(array_goldens())
    if "--fsm-only" in sys.argv:
        sys.exit(fsm_golden())
    main()
    float_w()
    array_goldens()
    sys.exit(fsm_golden())
