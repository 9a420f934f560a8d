"""ctypes binding of libfpldpc.so (include/fpldpc.h).

This is plumbing for tests and bench.py: the decoder itself is the C ABI + HIP kernels.  There is
no Python or CPU decode path; if the library or a GPU is missing, calls raise FpldpcError.
"""
import ctypes
import os

import numpy as np

from . import _build

FPLDPC_LLR_I32 = 0
FPLDPC_LLR_I16 = 1
FPLDPC_LLR_F64 = 2

_ERRORS = {-1: "ARG", -2: "IO", -3: "FORMAT", -4: "UNSUPPORTED", -5: "HIP", -6: "NOMEM"}


class FpldpcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"fpldpc error {code} ({_ERRORS.get(code, '?')}): {msg}")
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [("max_iter", ctypes.c_int32), ("frac_bits", ctypes.c_int32), ("width_mask", ctypes.c_int32),
                ("early_term", ctypes.c_int32), ("precheck", ctypes.c_int32), ("device", ctypes.c_int32)]


class SimParams(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_int64), ("first_frame", ctypes.c_int64), ("snr", ctypes.c_double),
                ("sigma", ctypes.c_double), ("frac_bits", ctypes.c_int32), ("codeword", ctypes.c_void_p),
                ("info_index", ctypes.c_void_p), ("info_bits", ctypes.c_void_p), ("k", ctypes.c_int32),
                ("forced_index", ctypes.c_void_p), ("n_forced", ctypes.c_int32), ("forced_llr", ctypes.c_int32),
                ("max_frame_errors", ctypes.c_int64), ("max_frames", ctypes.c_int64), ("count_mode", ctypes.c_int32),
                ("chunk", ctypes.c_int32), ("host_threads", ctypes.c_int32), ("on_frame", ctypes.c_void_p),
                ("on_frame_ctx", ctypes.c_void_p), ("device_channel", ctypes.c_int32)]


class SimResult(ctypes.Structure):
    _fields_ = [("bit_errors", ctypes.c_int64), ("frame_errors", ctypes.c_int64), ("frames", ctypes.c_int64),
                ("iter_sum", ctypes.c_int64), ("frames_decoded", ctypes.c_int64), ("seconds", ctypes.c_double)]


FPLDPC_COUNT_BITS = 0
FPLDPC_COUNT_ITERS = 1
# void (*on_frame)(void *ctx, int64_t frame, int32_t iterations, int64_t blkerror)
OnFrame = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64)

_lib = None


def lib():
    """Load the in-tree libfpldpc.so (building it first when sources are newer)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 / libhsa-runtime64
    # (same sonames as /opt/rocm's).  Loading torch first makes libfpldpc.so bind to that copy;
    # loading ours first would put two HIP/HSA runtimes in the process and the second one sees no
    # device.  Standalone C/C++ users simply get /opt/rocm's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    path = _build.LIB
    if os.environ.get("FPLDPC_LIB_PATH"):  # experiments: an alternative build of the same sources
        path = os.environ["FPLDPC_LIB_PATH"]
    elif not os.path.exists(path) or os.environ.get("FPLDPC_AUTOBUILD", "1") == "1":
        try:
            path = _build.build()
        except Exception as e:  # a prebuilt .so may still be present (GPU box without hipcc write access)
            if not os.path.exists(path):
                raise FpldpcError(-5, f"libfpldpc.so missing and build failed: {e}") from e
    L = ctypes.CDLL(path)
    P, I32, I64, U64, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_size_t
    sig = {
        "fpldpc_last_error": (ctypes.c_char_p, []),
        "fpldpc_version": (ctypes.c_char_p, []),
        "fpldpc_kernel_build_id": (ctypes.c_char_p, []),
        "fpldpc_code_load_alist": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(P)]),
        "fpldpc_code_parse_alist": (ctypes.c_int, [ctypes.c_char_p, SZ, ctypes.POINTER(P)]),
        "fpldpc_code_array": (ctypes.c_int, [I32, I32, I32, ctypes.POINTER(P)]),
        "fpldpc_code_wifi_1944_r12": (ctypes.c_int, [ctypes.POINTER(P)]),
        "fpldpc_code_dims": (ctypes.c_int, [P, P]),
        "fpldpc_code_rate": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_double)]),
        "fpldpc_code_lists": (ctypes.c_int, [P, P, P, P, P]),
        "fpldpc_code_write_alist": (ctypes.c_int, [P, ctypes.c_char_p, SZ, ctypes.POINTER(SZ)]),
        "fpldpc_code_syndrome_host": (ctypes.c_int, [P, P]),
        "fpldpc_code_free": (None, [P]),
        "fpldpc_params_default": (None, [ctypes.POINTER(Params)]),
        "fpldpc_decoder_create": (ctypes.c_int, [P, ctypes.POINTER(Params), ctypes.POINTER(P)]),
        "fpldpc_decoder_destroy": (ctypes.c_int, [P]),
        "fpldpc_decoder_describe": (ctypes.c_int, [P, ctypes.c_char_p, SZ]),
        "fpldpc_decoder_hard_words": (ctypes.c_int, [P]),
        "fpldpc_decoder_fallback_counts": (ctypes.c_int, [P, P]),
        "fpldpc_set_reference": (ctypes.c_int, [P, P, P, I32]),
        "fpldpc_decode": (ctypes.c_int, [P, P, I32, I32, P, P, P, P, P, P, P]),
        "fpldpc_decode_host": (ctypes.c_int, [P, P, I32, I32, P, P, P, P, P, P]),
        "fpldpc_edge_ram_words": (ctypes.c_int, [P, ctypes.POINTER(I64)]),
        "fpldpc_decode_frame": (ctypes.c_int, [P, P, I32, I32, P, P, P, P, P, P]),
        "fpldpc_decode_frame_host": (ctypes.c_int, [P, P, I32, P, P, P, P, P]),
        "fpldpc_rng_skip": (I64, [I64, U64]),
        "fpldpc_channel_llr_host": (ctypes.c_int, [I64, I64, I32, I32, ctypes.c_double, ctypes.c_double, I32, P, P,
                                                   I32, I32]),
        "fpldpc_encoder_load_g": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(P)]),
        "fpldpc_encoder_from_code": (ctypes.c_int, [P, ctypes.POINTER(P)]),
        "fpldpc_encoder_dims": (ctypes.c_int, [P, P]),
        "fpldpc_encoder_info_index": (ctypes.c_int, [P, P, P]),
        "fpldpc_unpack_info_bytes": (ctypes.c_int, [ctypes.c_char_p, I32, I32, P]),
        "fpldpc_encoder_encode_host": (ctypes.c_int, [P, P, I32, P, I32]),
        "fpldpc_encoder_encode": (ctypes.c_int, [P, P, I32, P, P]),
        "fpldpc_decode_float": (ctypes.c_int, [P, P, I32, P, P, P, P, P, P, P]),
        "fpldpc_decode_float_host": (ctypes.c_int, [P, P, I32, P, P, P, P, P, P]),
        "fpldpc_channel_llr": (ctypes.c_int, [I64, I64, I32, I32, ctypes.c_double, ctypes.c_double, I32, P, I32, P,
                                              I32, P, P]),
        "fpldpc_encoder_free": (None, [P]),
        "fpldpc_sim_params_default": (None, [ctypes.POINTER(SimParams)]),
        "fpldpc_ber_sim": (ctypes.c_int, [P, ctypes.POINTER(SimParams), ctypes.POINTER(SimResult)]),
        "fpldpc_ber_sim_multi": (ctypes.c_int, [P, I32, ctypes.POINTER(SimParams), I32, ctypes.POINTER(SimResult), P]),
        "fpldpc_testing_sim_inject": (None, [I32, I64, I32, I32]),  # include/fpldpc_testing.h (tests only)
    }
    for name, (res, args) in sig.items():
        if os.environ.get("FPLDPC_LIB_PATH") and not hasattr(L, name):
            continue  # an older experimental build without this entry point
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


# Every symbol include/*.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "fpldpc_last_error", "fpldpc_version", "fpldpc_kernel_build_id", "fpldpc_code_load_alist", "fpldpc_code_parse_alist", "fpldpc_code_array",
    "fpldpc_code_wifi_1944_r12", "fpldpc_code_dims", "fpldpc_code_rate", "fpldpc_code_lists",
    "fpldpc_code_write_alist", "fpldpc_code_syndrome_host", "fpldpc_code_free", "fpldpc_params_default",
    "fpldpc_decoder_create", "fpldpc_decoder_destroy", "fpldpc_decoder_describe", "fpldpc_decoder_hard_words",
    "fpldpc_decoder_fallback_counts", "fpldpc_set_reference", "fpldpc_decode", "fpldpc_decode_host",
    "fpldpc_edge_ram_words", "fpldpc_decode_frame", "fpldpc_decode_frame_host", "fpldpc_rng_skip", "fpldpc_channel_llr_host",
    "fpldpc_sim_params_default", "fpldpc_ber_sim", "fpldpc_ber_sim_multi", "fpldpc_encoder_load_g", "fpldpc_encoder_from_code",
    "fpldpc_encoder_dims", "fpldpc_encoder_info_index", "fpldpc_unpack_info_bytes", "fpldpc_encoder_encode_host",
    "fpldpc_encoder_free", "fpldpc_encoder_encode", "fpldpc_channel_llr",
    "fpldpc_decode_float", "fpldpc_decode_float_host",
    "fpldpc_testing_sim_inject",  # include/fpldpc_testing.h: test-only fault injection
]


def _check(st):
    if st != 0:
        raise FpldpcError(st, lib().fpldpc_last_error().decode())
    return st


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Code:
    """A parity-check code held by libfpldpc (fpldpc_code_t)."""

    def __init__(self, handle):
        self._h = handle
        dims = np.zeros(8, np.int32)
        _check(lib().fpldpc_code_dims(self._h, _ptr(dims)))
        (self.n, self.m, self.dv_max, self.dc_max, self.edges, self.qc_z, self.rank, reg) = [int(x) for x in dims]
        self.regular_checks = bool(reg)

    @classmethod
    def from_alist(cls, path):
        h = ctypes.c_void_p()
        _check(lib().fpldpc_code_load_alist(os.fsencode(path), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def parse(cls, text):
        b = text.encode() if isinstance(text, str) else bytes(text)
        h = ctypes.c_void_p()
        _check(lib().fpldpc_code_parse_alist(b, len(b), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def array(cls, p, r, forward=True):
        h = ctypes.c_void_p()
        _check(lib().fpldpc_code_array(p, r, 1 if forward else 0, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def wifi_1944_r12(cls):
        h = ctypes.c_void_p()
        _check(lib().fpldpc_code_wifi_1944_r12(ctypes.byref(h)))
        return cls(h)

    @property
    def rate(self):
        r = ctypes.c_double()
        _check(lib().fpldpc_code_rate(self._h, ctypes.byref(r)))
        return r.value

    @property
    def k(self):
        return self.n - self.rank

    def lists(self):
        vdeg = np.zeros(self.n, np.int32)
        cdeg = np.zeros(self.m, np.int32)
        vlist = np.zeros((self.n, self.dv_max), np.int32)
        clist = np.zeros((self.m, self.dc_max), np.int32)
        _check(lib().fpldpc_code_lists(self._h, _ptr(vdeg), _ptr(cdeg), _ptr(vlist), _ptr(clist)))
        return vdeg, cdeg, vlist, clist

    def write_alist(self):
        need = ctypes.c_size_t()
        _check(lib().fpldpc_code_write_alist(self._h, None, 0, ctypes.byref(need)))
        buf = ctypes.create_string_buffer(need.value + 1)
        _check(lib().fpldpc_code_write_alist(self._h, buf, need.value + 1, ctypes.byref(need)))
        return buf.value.decode()

    def syndrome_ok(self, bits):
        b = np.ascontiguousarray(bits, np.uint8)
        st = lib().fpldpc_code_syndrome_host(self._h, _ptr(b))
        if st < 0:
            _check(st)
        return st == 0

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.fpldpc_code_free(self._h)
            self._h = None


class Decoder:
    """fpldpc_decoder_t: a batched GPU decoder for one code and one parameter set."""

    def __init__(self, code, max_iter=30, frac_bits=4, width_mask=0xFF, early_term=True, precheck=False, device=-1):
        p = Params()
        lib().fpldpc_params_default(ctypes.byref(p))
        p.max_iter, p.frac_bits, p.width_mask = max_iter, frac_bits, width_mask
        p.early_term, p.precheck, p.device = int(bool(early_term)), int(bool(precheck)), device
        self.code = code
        self.params = p
        h = ctypes.c_void_p()
        _check(lib().fpldpc_decoder_create(code._h, ctypes.byref(p), ctypes.byref(h)))
        self._h = h
        self.hard_words = lib().fpldpc_decoder_hard_words(self._h)

    def describe(self):
        buf = ctypes.create_string_buffer(256)
        _check(lib().fpldpc_decoder_describe(self._h, buf, 256))
        return buf.value.decode()

    def fallback_counts(self):
        """(first, second) fallback-kernel frame counts of the last completed decode call."""
        c = np.zeros(2, np.int32)
        _check(lib().fpldpc_decoder_fallback_counts(self._h, _ptr(c)))
        return int(c[0]), int(c[1])

    def set_reference(self, info_index, info_bits):
        idx = np.ascontiguousarray(info_index, np.int32)
        bits = np.ascontiguousarray(info_bits, np.uint8)
        _check(lib().fpldpc_set_reference(self._h, _ptr(idx), _ptr(bits), len(idx)))

    def decode_ptrs(self, llr_ptr, llr_type, batch, hard=0, iters=0, syn_ok=0, post=0, bit_errors=0, totals=0,
                    stream=0):
        """Asynchronous decode on device pointers (ints); stream is a hipStream_t as int."""
        c = ctypes.c_void_p
        _check(lib().fpldpc_decode(self._h, c(llr_ptr), llr_type, batch, c(hard or None), c(iters or None),
                                   c(syn_ok or None), c(post or None), c(bit_errors or None), c(totals or None),
                                   c(stream or None)))

    def decode_torch(self, llr, post=False, bit_errors=False, totals=None, stream=None):
        """Decode a [B][n] int16/int32 CUDA tensor; returns a dict of output tensors.
        stream: None (torch's current stream), a torch.cuda.Stream, or a raw hipStream_t (int).
        On a stream other than the current one, the input and outputs are record_stream'ed so the
        caching allocator does not reuse them before the decode has run.  A decoder is single-stream
        (include/fpldpc.h): do not overlap two calls on it."""
        import torch
        assert llr.is_cuda and llr.dim() == 2 and llr.shape[1] == self.code.n and llr.is_contiguous()
        llr_type = FPLDPC_LLR_I16 if llr.dtype == torch.int16 else FPLDPC_LLR_I32
        assert llr.dtype in (torch.int16, torch.int32)
        B = llr.shape[0]
        dev = llr.device
        out = {
            "hard": torch.empty((B, self.hard_words), dtype=torch.int32, device=dev),
            "iters": torch.empty(B, dtype=torch.int32, device=dev),
            "syndrome_ok": torch.empty(B, dtype=torch.uint8, device=dev),
        }
        if post:
            out["post"] = torch.zeros((B, self.code.n), dtype=torch.int32, device=dev)
        if bit_errors:
            out["bit_errors"] = torch.empty(B, dtype=torch.int32, device=dev)
        cur = torch.cuda.current_stream(dev)
        if stream is None:
            s = cur
        elif isinstance(stream, torch.cuda.Stream):
            s = stream
        else:
            s = torch.cuda.ExternalStream(int(stream), device=dev)
        if s.cuda_stream != cur.cuda_stream:
            s.wait_stream(cur)  # outputs were allocated (and post zeroed) on the current stream
            for t in [llr, *out.values()] + ([totals] if totals is not None else []):
                t.record_stream(s)
        self.decode_ptrs(llr.data_ptr(), llr_type, B, out["hard"].data_ptr(), out["iters"].data_ptr(),
                         out["syndrome_ok"].data_ptr(), out["post"].data_ptr() if post else 0,
                         out["bit_errors"].data_ptr() if bit_errors else 0,
                         totals.data_ptr() if totals is not None else 0, s.cuda_stream)
        return out

    def decode_float_torch(self, llr, post=False, bit_errors=False, totals=None, stream=None):
        """Floating-point BP decode (fpldpc_decode_float) of a [B][n] float64 CUDA tensor."""
        import torch
        assert llr.is_cuda and llr.dim() == 2 and llr.shape[1] == self.code.n and llr.is_contiguous()
        assert llr.dtype == torch.float64
        B = llr.shape[0]
        dev = llr.device
        out = {
            "hard": torch.empty((B, self.hard_words), dtype=torch.int32, device=dev),
            "iters": torch.empty(B, dtype=torch.int32, device=dev),
            "syndrome_ok": torch.empty(B, dtype=torch.uint8, device=dev),
        }
        if post:
            out["post"] = torch.zeros((B, self.code.n), dtype=torch.float64, device=dev)
        if bit_errors:
            out["bit_errors"] = torch.empty(B, dtype=torch.int32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        _check(lib().fpldpc_decode_float(self._h, llr.data_ptr(), B, out["hard"].data_ptr(), out["iters"].data_ptr(),
                                         out["syndrome_ok"].data_ptr(), out["post"].data_ptr() if post else None,
                                         out["bit_errors"].data_ptr() if bit_errors else None,
                                         totals.data_ptr() if totals is not None else None, stream))
        return out

    def decode_float_host(self, llr, post=True, bit_errors=False):
        """Synchronous floating-point BP decode of a host [B][n] float64 array."""
        llr = np.ascontiguousarray(llr, np.float64)
        assert llr.ndim == 2 and llr.shape[1] == self.code.n
        B = llr.shape[0]
        hard = np.zeros((B, self.hard_words), np.uint32)
        iters = np.zeros(B, np.int32)
        ok = np.zeros(B, np.uint8)
        p = np.zeros((B, self.code.n), np.float64) if post else None
        be = np.zeros(B, np.int32) if bit_errors else None
        tot = np.zeros(4, np.int64)
        _check(lib().fpldpc_decode_float_host(self._h, _ptr(llr), B, _ptr(hard), _ptr(iters), _ptr(ok), _ptr(p),
                                              _ptr(be), _ptr(tot)))
        return {"hard": hard, "iters": iters, "syndrome_ok": ok, "post": p, "bit_errors": be, "totals": tot}

    def decode_host(self, llr, post=None, bit_errors=False, totals=None):
        """Synchronous decode of a host [B][n] int16/int32 array; returns numpy outputs."""
        llr = np.ascontiguousarray(llr)
        assert llr.ndim == 2 and llr.shape[1] == self.code.n and llr.dtype in (np.int16, np.int32)
        B = llr.shape[0]
        llr_type = FPLDPC_LLR_I16 if llr.dtype == np.int16 else FPLDPC_LLR_I32
        hard = np.zeros((B, self.hard_words), np.uint32)
        iters = np.zeros(B, np.int32)
        ok = np.zeros(B, np.uint8)
        post_arr = None
        if post is not None:
            post_arr = np.ascontiguousarray(post, np.int32) if not isinstance(post, bool) else np.zeros(
                (B, self.code.n), np.int32)
        be = np.zeros(B, np.int32) if bit_errors else None
        tot = None if totals is None else np.ascontiguousarray(totals, np.int64)
        _check(lib().fpldpc_decode_host(self._h, _ptr(llr), llr_type, B, _ptr(hard), _ptr(iters), _ptr(ok),
                                        _ptr(post_arr), _ptr(be), _ptr(tot)))
        out = {"hard": hard, "iters": iters, "syndrome_ok": ok}
        if post_arr is not None:
            out["post"] = post_arr
        if be is not None:
            out["bit_errors"] = be
        if tot is not None:
            out["totals"] = tot
        return out

    def ber_sim(self, snr, sigma, **kw):
        """Ordered BER/FER simulation (fpldpc_ber_sim): the reference harness's frame loop, batched.
        Keywords: see sim_params()."""
        p, keep = sim_params(snr, sigma, **kw)
        r = SimResult()
        _check(lib().fpldpc_ber_sim(self._h, ctypes.byref(p), ctypes.byref(r)))
        del keep
        return {k: getattr(r, k) for k, _ in SimResult._fields_}

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.fpldpc_decoder_destroy(self._h)
            self._h = None


class Encoder:
    """fpldpc_encoder_t: systematic encoder (reference G file, or derived natively from a Code)."""

    def __init__(self, handle):
        self._h = handle
        dims = np.zeros(3, np.int32)
        _check(lib().fpldpc_encoder_dims(self._h, _ptr(dims)))
        self.n, self.k, self.max_row_weight = (int(x) for x in dims)
        self.info_index = np.zeros(self.k, np.int32)
        self.parity_index = np.zeros(self.n - self.k, np.int32)
        _check(lib().fpldpc_encoder_info_index(self._h, _ptr(self.info_index), _ptr(self.parity_index)))

    @classmethod
    def from_code(cls, code):
        h = ctypes.c_void_p()
        _check(lib().fpldpc_encoder_from_code(code._h, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def load_g(cls, path):
        h = ctypes.c_void_p()
        _check(lib().fpldpc_encoder_load_g(os.fsencode(path), ctypes.byref(h)))
        return cls(h)

    def encode(self, info, nthreads=0):
        u = np.ascontiguousarray(np.atleast_2d(info), np.uint8)
        assert u.shape[1] == self.k
        cw = np.zeros((u.shape[0], self.n), np.uint8)
        _check(lib().fpldpc_encoder_encode_host(self._h, _ptr(u), u.shape[0], _ptr(cw), nthreads))
        return cw

    def encode_ptrs(self, info_ptr, batch, cw_ptr, stream=0):
        """Device encode (async on `stream`): uint8 info[batch][k] -> uint8 cw[batch][n], device pointers."""
        _check(lib().fpldpc_encoder_encode(self._h, info_ptr, batch, cw_ptr, stream))

    def encode_torch(self, info):
        """Device encode of a torch uint8 [B, k] CUDA tensor on torch's current stream -> [B, n]."""
        import torch
        assert info.is_cuda and info.dtype == torch.uint8 and info.dim() == 2 and info.shape[1] == self.k
        info = info.contiguous()
        cw = torch.empty((info.shape[0], self.n), dtype=torch.uint8, device=info.device)
        self.encode_ptrs(info.data_ptr(), info.shape[0], cw.data_ptr(), torch.cuda.current_stream(info.device).cuda_stream)
        return cw

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.fpldpc_encoder_free(self._h)
            self._h = None


def unpack_info_bytes(data, in_len, k):
    """setInfoBit's unpacking of a char stream (ArrayLDPC_Decoder.cpp:178-197)."""
    buf = bytes(data).ljust(in_len, b"\0")
    bits = np.zeros(k, np.uint8)
    _check(lib().fpldpc_unpack_info_bytes(buf, in_len, k, _ptr(bits)))
    return bits


def unpack_hard(hard_words, n):
    """[B][ceil(n/32)] packed words -> [B][n] uint8 bits (bit v%32 of word v//32)."""
    h = np.ascontiguousarray(hard_words).view(np.uint32)
    bits = np.unpackbits(h.view(np.uint8).reshape(h.shape[0], -1), axis=1, bitorder="little")
    return bits[:, :n]


def rng_skip(seed, draws):
    return int(lib().fpldpc_rng_skip(seed, draws))


def channel_llr(seed, first_frame, frames, n, snr, sigma, frac_bits=4, cw=None, dtype=np.int16, nthreads=0):
    """Reference-harness LLRs (PerfTest.cpp:108-120) for frames [first_frame, first_frame+frames)."""
    out = np.empty((frames, n), dtype)
    t = {np.dtype(np.int16): FPLDPC_LLR_I16, np.dtype(np.int32): FPLDPC_LLR_I32,
         np.dtype(np.float64): FPLDPC_LLR_F64}[np.dtype(dtype)]
    cwa = None if cw is None else np.ascontiguousarray(cw, np.uint8)
    _check(lib().fpldpc_channel_llr_host(seed, first_frame, frames, n, snr, sigma, frac_bits, _ptr(cwa), _ptr(out), t,
                                         nthreads))
    return out


def channel_llr_ptrs(seed, first_frame, frames, n, snr, sigma, frac_bits, cw_ptr, cw_per_frame, out_ptr, out_type,
                     overflow_ptr=0, stream=0):
    """Device channel (async on `stream`); every pointer is device memory (0 = NULL)."""
    _check(lib().fpldpc_channel_llr(seed, first_frame, frames, n, snr, sigma, frac_bits, cw_ptr or None, cw_per_frame,
                                    out_ptr, out_type, overflow_ptr or None, stream or None))


def channel_llr_torch(seed, first_frame, frames, n, snr, sigma, frac_bits=4, cw=None, dtype=None, device=None):
    """Device channel into a new torch [frames, n] tensor (int16 default) on torch's current stream.
    cw: None, a uint8 [n] tensor (shared) or [frames, n] (per frame).  Returns (llr, overflow) -- overflow: int32 [1] count of values outside int16."""
    import torch
    dtype = dtype or torch.int16
    device = torch.device(device if device is not None else (cw.device if cw is not None else "cuda"))
    out = torch.empty((frames, n), dtype=dtype, device=device)
    ovf = torch.zeros(1, dtype=torch.int32, device=device)
    per = 0
    if cw is not None:
        assert cw.dtype == torch.uint8 and cw.is_cuda
        cw = cw.contiguous()
        per = 1 if cw.dim() == 2 else 0
        assert cw.shape[-1] == n and (not per or cw.shape[0] == frames)
    t = {torch.int16: FPLDPC_LLR_I16, torch.int32: FPLDPC_LLR_I32, torch.float64: FPLDPC_LLR_F64}[dtype]
    channel_llr_ptrs(seed, first_frame, frames, n, snr, sigma, frac_bits, cw.data_ptr() if cw is not None else 0, per,
                     out.data_ptr(), t, ovf.data_ptr(), torch.cuda.current_stream(device).cuda_stream)
    return out, ovf


def snr_sigma(ebn0_db, rate):
    """snr = 2 * 10^(EbN0/10) * R, sigma = sqrt(1/snr)  (PerfTest.cpp:62-63, 252-254)."""
    import math
    snr = 2 * math.pow(10.0, ebn0_db / 10) * rate
    return snr, math.sqrt(1 / snr)


FPLDPC_COLL_AUTO, FPLDPC_COLL_RCCL, FPLDPC_COLL_HOST = 0, 1, 2


def sim_params(snr, sigma, info_index=None, info_bits=None, codeword=None, seed=123456789, first_frame=0, frac_bits=4,
               max_frame_errors=100, max_frames=0, count_mode=FPLDPC_COUNT_BITS, forced_index=None, forced_llr=0,
               chunk=0, host_threads=0, device_channel=False, on_frame=None):
    """fpldpc_sim_params for fpldpc_ber_sim / fpldpc_ber_sim_multi; returns (params, keep-alive list).
    on_frame(frame, iterations, blkerror) is called in frame order for every counted frame."""
    p = SimParams()
    lib().fpldpc_sim_params_default(ctypes.byref(p))
    keep = []

    def arr(a, dt):
        if a is None:
            return None, 0
        a = np.ascontiguousarray(a, dt)
        keep.append(a)
        return a.ctypes.data_as(ctypes.c_void_p), len(a)

    p.seed, p.first_frame, p.snr, p.sigma, p.frac_bits = seed, first_frame, snr, sigma, frac_bits
    p.codeword, _ = arr(codeword, np.uint8)
    p.info_index, p.k = arr(info_index, np.int32)
    p.info_bits, _ = arr(info_bits, np.uint8)
    p.forced_index, p.n_forced = arr(forced_index, np.int32)
    p.forced_llr = forced_llr
    p.max_frame_errors, p.max_frames, p.count_mode = max_frame_errors, max_frames, count_mode
    p.chunk, p.host_threads, p.device_channel = chunk, host_threads, int(bool(device_channel))
    if on_frame is not None:
        cb = OnFrame(lambda ctx, f, it, blk: on_frame(f, it, blk))
        keep.append(cb)
        p.on_frame = ctypes.cast(cb, ctypes.c_void_p).value
    return p, keep


def ber_sim_multi(decoders, snr, sigma, collective=FPLDPC_COLL_AUTO, **kw):
    """fpldpc_ber_sim_multi over several decoders (one host thread each; RCCL between distinct devices,
    host memory otherwise).  Returns the fpldpc_ber_sim result dict plus 'collective' (1 RCCL, 2 host)."""
    p, keep = sim_params(snr, sigma, **kw)
    hs = (ctypes.c_void_p * len(decoders))(*[d._h for d in decoders])
    r = SimResult()
    used = ctypes.c_int32(0)
    _check(lib().fpldpc_ber_sim_multi(hs, len(decoders), ctypes.byref(p), collective, ctypes.byref(r),
                                      ctypes.byref(used)))
    del keep
    out = {k: getattr(r, k) for k, _ in SimResult._fields_}
    out["collective"] = used.value
    return out
