"""ctypes view of oracle/_build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / the timed CPU baseline.  The product (fixedpointldpc_amd, include/) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ref_wifi")
REF_DIR = "/root/reference"


class OrcCode(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("m", ctypes.c_int), ("dv_max", ctypes.c_int), ("dc_max", ctypes.c_int),
                ("vdeg", ctypes.POINTER(ctypes.c_int)), ("cdeg", ctypes.POINTER(ctypes.c_int)),
                ("vlist", ctypes.POINTER(ctypes.c_int)), ("clist", ctypes.POINTER(ctypes.c_int))]


_lib = None


def build(ref=False):
    targets = ["all"] + (["ref"] if ref and os.path.isdir(REF_DIR) else [])
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "fpldpc_oracle.c")):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        L.orc_code_load_alist.argtypes = [ctypes.c_char_p, ctypes.POINTER(OrcCode)]
        L.orc_code_free.argtypes = [ctypes.POINTER(OrcCode)]
        L.orc_constant.argtypes = [ctypes.c_int]
        L.orc_sxor.argtypes = [ctypes.c_int] * 4
        L.orc_sxor_table.argtypes = [ctypes.c_int] * 4 + [P]
        L.orc_decode_general.argtypes = [ctypes.POINTER(OrcCode), P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P]
        L.orc_decode_fixpoint.argtypes = L.orc_decode_general.argtypes
        L.orc_decode_general_edges.argtypes = [ctypes.POINTER(OrcCode), P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               P, ctypes.c_int, P, P, P]
        L.orc_decode_fixpoint_edges.argtypes = L.orc_decode_general_edges.argtypes
        L.orc_decode_batch.argtypes = [ctypes.POINTER(OrcCode), P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P]
        L.orc_decode_batch.restype = None
        L.orc_random.argtypes = [ctypes.POINTER(ctypes.c_int64)]
        L.orc_random.restype = ctypes.c_double
        L.orc_normal.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_double, ctypes.c_double]
        L.orc_normal.restype = ctypes.c_double
        L.orc_skip.argtypes = [ctypes.c_int64, ctypes.c_uint64]
        L.orc_skip.restype = ctypes.c_int64
        L.orc_gen_llr.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                  ctypes.c_double, ctypes.c_int, P, P, ctypes.c_int]
        L.orc_gen_llr.restype = None
        L.orc_gen_llr_f64.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                      ctypes.c_double, P, P, ctypes.c_int]
        L.orc_gen_llr_f64.restype = None
        L.orc_sxor_f64.argtypes = [ctypes.c_double, ctypes.c_double]
        L.orc_sxor_f64.restype = ctypes.c_double
        L.orc_decode_float_batch.argtypes = [ctypes.POINTER(OrcCode), P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             P, P, P, P]
        L.orc_decode_float_batch.restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleCode:
    """orc_code built from an alist file or from (vdeg, cdeg, vlist, clist) arrays."""

    def __init__(self, n, m, vdeg, cdeg, vlist, clist):
        self.n, self.m = n, m
        self._vdeg = np.ascontiguousarray(vdeg, np.int32)
        self._cdeg = np.ascontiguousarray(cdeg, np.int32)
        self._vlist = np.ascontiguousarray(vlist, np.int32)
        self._clist = np.ascontiguousarray(clist, np.int32)
        c = OrcCode()
        c.n, c.m = n, m
        c.dv_max, c.dc_max = self._vlist.shape[1], self._clist.shape[1]
        ip = ctypes.POINTER(ctypes.c_int)
        c.vdeg = self._vdeg.ctypes.data_as(ip)
        c.cdeg = self._cdeg.ctypes.data_as(ip)
        c.vlist = self._vlist.ctypes.data_as(ip)
        c.clist = self._clist.ctypes.data_as(ip)
        self.c = c

    @classmethod
    def from_alist_text(cls, text):
        t = np.array(text.split(), np.int64)
        n, m, dv, dc = (int(x) for x in t[:4])
        i = 4
        vdeg = t[i:i + n]; i += n
        cdeg = t[i:i + m]; i += m
        vlist = np.full((n, dv), -1, np.int32)
        for v in range(n):
            vlist[v, :vdeg[v]] = t[i:i + vdeg[v]]; i += int(vdeg[v])
        clist = np.full((m, dc), -1, np.int32)
        for r in range(m):
            clist[r, :cdeg[r]] = t[i:i + cdeg[r]]; i += int(cdeg[r])
        assert i == len(t)
        return cls(n, m, vdeg, cdeg, vlist, clist)

    @classmethod
    def from_alist(cls, path):
        with open(path) as f:
            return cls.from_alist_text(f.read())


def constant(frac_bits):
    return lib().orc_constant(frac_bits)


def sxor(x, y, frac_bits=4, mask=0xFF):
    return lib().orc_sxor(int(x), int(y), constant(frac_bits), mask)


def sxor_table(lo, hi, frac_bits=4, mask=0xFF):
    w = hi - lo + 1
    out = np.empty((w, w), np.int32)
    lib().orc_sxor_table(lo, hi, constant(frac_bits), mask, _p(out))
    return out


def decode_batch(code, llr, max_iter=30, frac_bits=4, mask=0xFF, precheck=False, nthreads=0, want_post=True):
    llr = np.ascontiguousarray(llr)
    assert llr.dtype in (np.int16, np.int32) and llr.shape[1] == code.n
    B = llr.shape[0]
    iters = np.zeros(B, np.int32)
    ok = np.zeros(B, np.uint8)
    hard = np.zeros((B, code.n), np.uint8)
    post = np.zeros((B, code.n), np.int32) if want_post else None
    lib().orc_decode_batch(ctypes.byref(code.c), _p(llr), int(llr.dtype == np.int16), B, max_iter,
                           constant(frac_bits), mask, int(precheck), nthreads, _p(iters), _p(ok), _p(hard), _p(post))
    return {"iters": iters, "syndrome_ok": ok, "hard": hard, "post": post}


IDLE, PCV, C2V = 0, 1, 4  # ArrayLDPCMacro.h:40


class FSMDecoder:
    """FP_Decoder's per-frame state across calls (ArrayLDPCMacro.h:121-176): the edge RAM
    (EdgeRAM[k].BRAM_fp[c] = edge[k][c], zero like a static object's), Posteriori_fp,
    DecodedCodeword and the ControlFSM state, with decode_general_fp (:18-171) and decode_fixpoint
    (:422-639) as the reference sequences them (:443-488, :621-630)."""

    def __init__(self, code, max_iter=30, frac_bits=4, mask=0xFF):
        self.code, self.max_iter, self.C, self.mask = code, max_iter, constant(frac_bits), mask
        self.edge = np.zeros(code.c.dc_max * code.m, np.int32)
        self.post = np.zeros(code.n, np.int32)
        self.hard = np.zeros(code.n, np.uint8)
        self.state = IDLE

    def _run(self, fn, llr, keep):
        llr = np.ascontiguousarray(llr, np.int32)
        ok = ctypes.c_int(0)
        post = self.post.copy()
        it = fn(ctypes.byref(self.code.c), _p(llr), self.max_iter, self.C, self.mask, _p(self.edge), int(keep),
                _p(post), _p(self.hard), ctypes.byref(ok))
        self.post = post
        return it, ok.value

    def decode_general_fp(self, llr):
        return self._run(lib().orc_decode_general_edges, llr, False)[0]

    def decode_fixpoint(self, llr):
        if self.state not in (PCV, C2V):  # the loop does not run: the pre-check's channel decision
            self.hard[:] = np.asarray(llr) <= 0
            return 0
        it, ok = self._run(lib().orc_decode_fixpoint_edges, llr, self.state == C2V)
        if it > 0:
            self.state = IDLE if ok else C2V
        return it


def gen_llr(seed, f0, frames, n, snr, sigma, frac_bits=4, cw=None, nthreads=0):
    out = np.empty((frames, n), np.int32)
    cwa = None if cw is None else np.ascontiguousarray(cw, np.uint8)
    lib().orc_gen_llr(seed, f0, frames, n, snr, sigma, frac_bits, _p(cwa), _p(out), nthreads)
    return out


def gen_llr_f64(seed, f0, frames, n, snr, sigma, cw=None, nthreads=0):
    """Unquantised channel LLRs (doubles) for the floating-point decoder."""
    out = np.empty((frames, n), np.float64)
    cwa = None if cw is None else np.ascontiguousarray(cw, np.uint8)
    lib().orc_gen_llr_f64(seed, f0, frames, n, snr, sigma, _p(cwa), _p(out), nthreads)
    return out


def sxor_f64(x, y):
    return lib().orc_sxor_f64(float(x), float(y))


def decode_float_batch(code, llr, max_iter=30, nthreads=0, want_post=True):
    """decode_general (floating-point BP) restatement over [B][n] float64 LLRs."""
    llr = np.ascontiguousarray(llr, np.float64)
    assert llr.shape[1] == code.n
    B = llr.shape[0]
    iters = np.zeros(B, np.int32)
    ok = np.zeros(B, np.uint8)
    hard = np.zeros((B, code.n), np.uint8)
    post = np.zeros((B, code.n), np.float64) if want_post else None
    lib().orc_decode_float_batch(ctypes.byref(code.c), _p(llr), B, max_iter, nthreads, _p(iters), _p(ok), _p(hard),
                                 _p(post))
    return {"iters": iters, "syndrome_ok": ok, "hard": hard, "post": post}


def test_random():
    return bool(lib().orc_test_random())
