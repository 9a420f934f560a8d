"""MI355X-native fixed-point LDPC decoder (drop-in for tyc85/FixedPointLDPC's decode path).

The product is libfpldpc.so: a C ABI (include/fpldpc.h) over hand-written gfx950 HIP kernels, plus
the C++ compatibility layer (include/fpldpc_compat.hpp).  This package only locates/builds that
library and binds it with ctypes for tests and bench.py.
"""
from ._lib import (FPLDPC_COLL_AUTO, FPLDPC_COLL_HOST, FPLDPC_COLL_RCCL, FPLDPC_LLR_F64, FPLDPC_LLR_I16, FPLDPC_LLR_I32, Code, Decoder, Encoder, FpldpcError, channel_llr, channel_llr_ptrs,
                   channel_llr_torch, lib, rng_skip, snr_sigma, unpack_hard, unpack_info_bytes, ber_sim_multi)

__all__ = ["ber_sim_multi", "FPLDPC_COLL_AUTO", "FPLDPC_COLL_RCCL", "FPLDPC_COLL_HOST", "Code", "Decoder", "Encoder", "unpack_info_bytes", "FpldpcError", "channel_llr", "channel_llr_ptrs", "channel_llr_torch", "lib", "rng_skip", "snr_sigma", "unpack_hard",
           "FPLDPC_LLR_I16", "FPLDPC_LLR_I32", "FPLDPC_LLR_F64"]
