// fpldpc_gen.hip -- gfx950 kernels on either side of the decoder: the reference harness's
// channel (Lehmer uniforms -> Odeh-Evans normals -> quantised BPSK/AWGN LLRs) and the systematic
// encoder, batched on the device so a BER simulation never leaves HBM.
//
// Channel: Random() rngs.cpp:52-69 (m = 2^31 - 1, a = 48271), Normal() rvgs.cpp:152-181,
// LLR_fp = (int)(2*snr*(1 - 2c + Normal(0, sigma)) * 2^frac) PerfTest.cpp:108-120.  Draw index
// D = frame*n + i (the reference's single stream, never re-seeded): a thread owns kChunk
// consecutive draws of one frame and jumps to its first one by a^D mod m (square-and-multiply
// over a table of a^(2^j)), then steps.  The Lehmer states are bit-identical to the host's; the
// normals use the device libm (log, sqrt in double), checked against the host channel
// (tests/test_gpu_gen.py).
// Encoder: ArrayLDPC_Encoder.cpp:160-225 -- info bits at the info positions, parity r = XOR of
// the info bits in row r, here as popcount(packed info & row mask) over 32-bit words.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "fpldpc_internal.hpp"

namespace fpldpc {
namespace {

constexpr uint64_t kMod = 2147483647ull;  // rngs.cpp:40
constexpr uint64_t kMul = 48271ull;       // rngs.cpp:41
constexpr int kChunk = 16;                // consecutive draws per thread
constexpr int kPowBits = 48;              // draw indices < 2^48

struct ChanArgs {
    uint64_t apow[kPowBits];  // a^(2^j) mod m
    uint64_t seed;
    int64_t first_frame;
    int frames, n, frac, out_type, cw_per_frame;
    double snr, sigma;
    const uint8_t *cw;
    void *out;
    int *overflow;
};

__device__ __forceinline__ uint64_t mulmod(uint64_t x, uint64_t y) {  // x, y < 2^31
    const uint64_t p = x * y;                                          // < 2^62
    uint64_t r = (p & kMod) + (p >> 31);                               // Mersenne fold
    r = (r & kMod) + (r >> 31);
    return r >= kMod ? r - kMod : r;
}

__global__ void __launch_bounds__(256) channel_kernel(ChanArgs a) {
    const int per_frame = (a.n + kChunk - 1) / kChunk;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (int64_t)a.frames * per_frame) return;
    const int f = (int)(tid / per_frame), i0 = (int)(tid % per_frame) * kChunk;
    // state after D draws = seed * a^D: the next Random() returns draw D + 1's state
    uint64_t D = (uint64_t)(a.first_frame + f) * (uint64_t)a.n + (uint64_t)i0;
    uint64_t s = a.seed;
#pragma unroll 1
    for (int j = 0; D; ++j, D >>= 1)
        if (D & 1) s = mulmod(s, a.apow[j]);
    const double scale = (double)(1 << a.frac);
    const uint8_t *cw = a.cw ? a.cw + (a.cw_per_frame ? (size_t)f * a.n : 0) : nullptr;
    const size_t base = (size_t)f * a.n;
    int ovf = 0;
    const int i1 = min(a.n, i0 + kChunk);
    for (int i = i0; i < i1; ++i) {
        s = mulmod(s, kMul);  // Random(): the same state sequence as Schrage's method
        const double u = (double)s / (double)kMod;
        // Normal(0, sigma): Odeh & Evans (rvgs.cpp:159-180), one uniform per variate
        const double p0 = 0.322232431088, q0 = 0.099348462606;
        const double p1 = 1.0, q1 = 0.588581570495;
        const double p2 = 0.342242088547, q2 = 0.531103462366;
        const double p3 = 0.204231210245e-1, q3 = 0.103537752850;
        const double p4 = 0.453642210148e-4, q4 = 0.385607006340e-2;
        const double t = u < 0.5 ? sqrt(-2.0 * log(u)) : sqrt(-2.0 * log(1.0 - u));
        const double p = __dadd_rn(p0, __dmul_rn(t, __dadd_rn(p1, __dmul_rn(t, __dadd_rn(p2, __dmul_rn(t, __dadd_rn(p3, __dmul_rn(t, p4))))))));
        const double q = __dadd_rn(q0, __dmul_rn(t, __dadd_rn(q1, __dmul_rn(t, __dadd_rn(q2, __dmul_rn(t, __dadd_rn(q3, __dmul_rn(t, q4))))))));
        const double z = u < 0.5 ? __dsub_rn(__ddiv_rn(p, q), t) : __dsub_rn(t, __ddiv_rn(p, q));
        const double nrm = __dadd_rn(0.0, __dmul_rn(a.sigma, z));
        const int c = cw ? (int)(cw[i] & 1) : 0;
        const double llr = __dmul_rn(__dmul_rn(2.0, a.snr), __dadd_rn((double)(1 - 2 * c), nrm));
        if (a.out_type == FPLDPC_LLR_F64) {
            static_cast<double *>(a.out)[base + i] = llr;
            continue;
        }
        const int x = (int)__dmul_rn(llr, scale);  // (int) truncation, no clipping
        if (a.out_type == FPLDPC_LLR_I16) {
            ovf += (x < -32768) | (x > 32767);
            static_cast<int16_t *>(a.out)[base + i] = (int16_t)x;
        } else {
            static_cast<int32_t *>(a.out)[base + i] = x;
        }
    }
    if (ovf && a.overflow) atomicAdd(a.overflow, ovf);
}

// info bits [B][k] (uint8) -> packed words [B][kw]
__global__ void __launch_bounds__(256) pack_info_kernel(const uint8_t *info, int batch, int k, int kw, uint32_t *out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)batch * kw) return;
    const int b = (int)(t / kw), w = (int)(t % kw);
    const uint8_t *u = info + (size_t)b * k + (size_t)w * 32;
    const int cnt = min(32, k - w * 32);
    uint32_t x = 0;
    for (int j = 0; j < cnt; ++j) x |= (uint32_t)(u[j] & 1u) << j;
    out[t] = x;
}

// codeword position v of frame b: info bit, or the parity of (packed info & row mask)
__global__ void __launch_bounds__(256) encode_kernel(const uint32_t *packed, const uint8_t *info, int batch, int n,
                                                     int k, int kw, const int32_t *pos, const uint32_t *rowmask,
                                                     uint8_t *cw) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)batch * n) return;
    const int b = (int)(t / n), v = (int)(t % n);
    const int p = pos[v];
    uint8_t bit;
    if (p >= 0) {
        bit = info[(size_t)b * k + p] & 1u;
    } else {
        const uint32_t *row = rowmask + (size_t)(-p - 1) * kw;
        const uint32_t *u = packed + (size_t)b * kw;
        uint32_t x = 0;
        for (int w = 0; w < kw; ++w) x ^= u[w] & row[w];
        bit = (uint8_t)(__popc(x) & 1);
    }
    cw[t] = bit;
}

__global__ void __launch_bounds__(256) force_llr_kernel(int16_t *llr, int frames, int n, const int32_t *idx, int n_idx,
                                                        int16_t value) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)frames * n_idx) return;
    llr[(t / n_idx) * n + idx[t % n_idx]] = value;
}

int hip_fail(hipError_t e, const char *what) { return fail_hip((int)e, what); }

}  // namespace

int launch_channel(int64_t seed, int64_t first_frame, int frames, int n, double snr, double sigma, int frac_bits,
                   const uint8_t *cw, int cw_per_frame, void *out, int out_type, int *overflow, void *stream) {
    if (frames <= 0) return FPLDPC_OK;
    ChanArgs a;
    uint64_t x = kMul;
    for (int j = 0; j < kPowBits; ++j) {
        a.apow[j] = x;
        x = (uint64_t)(((unsigned __int128)x * x) % kMod);
    }
    a.seed = (uint64_t)seed;
    a.first_frame = first_frame;
    a.frames = frames;
    a.n = n;
    a.frac = frac_bits;
    a.out_type = out_type;
    a.cw_per_frame = cw_per_frame;
    a.snr = snr;
    a.sigma = sigma;
    a.cw = cw;
    a.out = out;
    a.overflow = overflow;
    const int64_t threads = (int64_t)frames * ((n + kChunk - 1) / kChunk);
    hipLaunchKernelGGL(channel_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? FPLDPC_OK : hip_fail(e, "channel kernel launch");
}

int launch_force_llr(int16_t *llr, int frames, int n, const int32_t *idx, int n_idx, int16_t value, void *stream) {
    const int64_t t = (int64_t)frames * n_idx;
    if (t <= 0) return FPLDPC_OK;
    hipLaunchKernelGGL(force_llr_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, (hipStream_t)stream, llr, frames,
                       n, idx, n_idx, value);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? FPLDPC_OK : hip_fail(e, "force kernel launch");
}

int encoder_upload(fpldpc_encoder *e) {
    int dev = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err != hipSuccess) return hip_fail(err, "hipGetDevice");
    if (e->d_pos && e->device == dev) return FPLDPC_OK;
    if (e->d_pos) return fail(FPLDPC_ERR_ARG, "encoder already bound to another device");
    const int n = e->n, k = e->k, R = (int)e->row_ptr.size() - 1;
    e->kw = (k + 31) / 32;
    std::vector<int32_t> pos(n, 0);
    for (int i = 0; i < k; ++i) pos[e->info_index[i]] = i;
    for (int r = 0; r < R; ++r) pos[e->parity_index[r]] = -(r + 1);
    std::vector<uint32_t> mask((size_t)std::max(R, 1) * e->kw, 0);
    for (int r = 0; r < R; ++r)
        for (int j = e->row_ptr[r]; j < e->row_ptr[r + 1]; ++j) {
            const int s = e->info_slot[e->row_var[j]];
            mask[(size_t)r * e->kw + s / 32] ^= 1u << (s % 32);  // repeated entries cancel, as XOR does
        }
    if ((err = hipMalloc(&e->d_pos, sizeof(int32_t) * n)) != hipSuccess) return hip_fail(err, "hipMalloc");
    if ((err = hipMalloc(&e->d_rowmask, sizeof(uint32_t) * mask.size())) != hipSuccess) return hip_fail(err, "hipMalloc");
    if ((err = hipMemcpy(e->d_pos, pos.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(err, "hipMemcpy");
    if ((err = hipMemcpy(e->d_rowmask, mask.data(), sizeof(uint32_t) * mask.size(), hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(err, "hipMemcpy");
    e->device = dev;
    return FPLDPC_OK;
}

int launch_encode(fpldpc_encoder *e, const uint8_t *info, int batch, uint8_t *cw, void *stream) {
    if (batch <= 0) return FPLDPC_OK;
    int st = encoder_upload(e);
    if (st) return st;
    if (batch > e->cap) {  // grows to the largest batch seen (not inside graph capture)
        (void)hipFree(e->d_packed);
        e->d_packed = nullptr;
        e->cap = 0;
        const hipError_t err = hipMalloc(&e->d_packed, sizeof(uint32_t) * (size_t)batch * e->kw);
        if (err != hipSuccess) return hip_fail(err, "hipMalloc");
        e->cap = batch;
    }
    hipStream_t s = (hipStream_t)stream;
    const int64_t t1 = (int64_t)batch * e->kw, t2 = (int64_t)batch * e->n;
    hipLaunchKernelGGL(pack_info_kernel, dim3((unsigned)((t1 + 255) / 256)), dim3(256), 0, s, info, batch, e->k, e->kw,
                       e->d_packed);
    hipLaunchKernelGGL(encode_kernel, dim3((unsigned)((t2 + 255) / 256)), dim3(256), 0, s, e->d_packed, info, batch, e->n,
                       e->k, e->kw, e->d_pos, e->d_rowmask, cw);
    const hipError_t err = hipGetLastError();
    return err == hipSuccess ? FPLDPC_OK : hip_fail(err, "encode kernel launch");
}

}  // namespace fpldpc

extern "C" {

int fpldpc_encoder_encode(fpldpc_encoder_t enc, const uint8_t *info, int32_t batch, uint8_t *cw, void *stream) {
    if (!enc || batch < 0 || (batch > 0 && (!info || !cw))) return fpldpc::fail(FPLDPC_ERR_ARG, "bad argument");
    return fpldpc::launch_encode(enc, info, batch, cw, stream);
}

int fpldpc_channel_llr(int64_t seed, int64_t first_frame, int32_t frames, int32_t n, double snr, double sigma,
                       int32_t frac_bits, const uint8_t *cw, int32_t cw_per_frame, void *out, int32_t out_type,
                       int32_t *overflow, void *stream) {
    if (!out || frames < 0 || n <= 0 || first_frame < 0 || frac_bits < 0 || frac_bits > 24 || seed <= 0 ||
        seed >= 2147483647 || (uint64_t)(first_frame + frames) * (uint64_t)n >= (1ull << fpldpc::kPowBits))
        return fpldpc::fail(FPLDPC_ERR_ARG, "bad channel arguments");
    if (out_type != FPLDPC_LLR_I32 && out_type != FPLDPC_LLR_I16 && out_type != FPLDPC_LLR_F64)
        return fpldpc::fail(FPLDPC_ERR_ARG, "bad out_type");
    return fpldpc::launch_channel(seed, first_frame, frames, n, snr, sigma, frac_bits, cw, cw_per_frame, out, out_type,
                                  overflow, stream);
}

}  // extern "C"
