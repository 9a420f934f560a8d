// fpldpc_channel.cpp -- the reference harness's channel model on the host: Lehmer uniforms with
// O(log k) skip-ahead, Odeh-Evans normals, BPSK/AWGN LLR quantisation.  Frames are independent
// given the skip-ahead, so generation is split over threads by frame range.
//
// Reference: Random() rngs.cpp:52-69 (m = 2^31-1, a = 48271, Schrage), Normal() rvgs.cpp:152-181,
// LLR quantisation PerfTest.cpp:108-120 / 168-169 / 287-297.
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "fpldpc_internal.hpp"

// Bit parity with the gcc/glibc-built reference needs the exact operation sequence: no FMA
// contraction of the Odeh-Evans polynomials or the LLR scaling.
#pragma clang fp contract(off)

namespace {

constexpr int64_t kModulus = 2147483647;  // rngs.cpp:40
constexpr int64_t kMultiplier = 48271;    // rngs.cpp:41

inline double lehmer_next(int64_t *state) {
    const int64_t Q = kModulus / kMultiplier, R = kModulus % kMultiplier;
    const int64_t s = *state;
    const int64_t t = kMultiplier * (s % Q) - R * (s / Q);
    *state = t > 0 ? t : t + kModulus;
    return (double)*state / kModulus;
}

inline double odeh_evans_normal(int64_t *state, double sigma) {
    const double p0 = 0.322232431088, q0 = 0.099348462606;
    const double p1 = 1.0, q1 = 0.588581570495;
    const double p2 = 0.342242088547, q2 = 0.531103462366;
    const double p3 = 0.204231210245e-1, q3 = 0.103537752850;
    const double p4 = 0.453642210148e-4, q4 = 0.385607006340e-2;
    const double u = lehmer_next(state);
    const double t = u < 0.5 ? sqrt(-2.0 * log(u)) : sqrt(-2.0 * log(1.0 - u));
    const double p = p0 + t * (p1 + t * (p2 + t * (p3 + t * p4)));
    const double q = q0 + t * (q1 + t * (q2 + t * (q3 + t * q4)));
    const double z = u < 0.5 ? (p / q) - t : t - (p / q);
    return 0.0 + sigma * z;  // Normal(m = 0, s = sigma)
}

inline int64_t mulmod(int64_t a, int64_t b) { return (int64_t)(((__int128)a * b) % kModulus); }

}  // namespace

extern "C" {

int64_t fpldpc_rng_skip(int64_t seed, uint64_t draws) {
    int64_t r = 1, b = kMultiplier;
    while (draws) {
        if (draws & 1) r = mulmod(r, b);
        b = mulmod(b, b);
        draws >>= 1;
    }
    return mulmod(seed, r);
}

int fpldpc_channel_llr_host(int64_t seed, int64_t first_frame, int32_t frames, int32_t n, double snr,
                            double sigma, int32_t frac_bits, const uint8_t *cw, void *out, int32_t out_type,
                            int32_t nthreads) {
    if (!out || frames < 0 || n <= 0 || first_frame < 0 || frac_bits < 0 || frac_bits > 24 || seed <= 0 ||
        seed >= kModulus)
        return fpldpc::fail(FPLDPC_ERR_ARG, "bad channel arguments");
    if (out_type != FPLDPC_LLR_I32 && out_type != FPLDPC_LLR_I16 && out_type != FPLDPC_LLR_F64)
        return fpldpc::fail(FPLDPC_ERR_ARG, "bad out_type");
    if (frames == 0) return FPLDPC_OK;
    unsigned hw = std::thread::hardware_concurrency();
    int T = nthreads > 0 ? nthreads : (int)(hw ? hw : 1);
    T = std::max(1, std::min(T, frames));
    std::vector<int> overflow(T, 0);
    auto work = [&](int t) {
        const int64_t f_lo = (int64_t)frames * t / T, f_hi = (int64_t)frames * (t + 1) / T;
        int64_t state = fpldpc_rng_skip(seed, (uint64_t)(first_frame + f_lo) * (uint64_t)n);
        const double scale = (double)(1 << frac_bits);
        for (int64_t f = f_lo; f < f_hi; f++)
            for (int i = 0; i < n; i++) {
                const double llr = 2 * snr * (1 - 2 * (cw ? (int)(cw[i] & 1) : 0) + odeh_evans_normal(&state, sigma));
                const size_t at = (size_t)f * n + i;
                if (out_type == FPLDPC_LLR_F64) {
                    static_cast<double *>(out)[at] = llr;
                    continue;
                }
                const int32_t q = (int32_t)(llr * scale);  // int() truncation, no clipping
                if (out_type == FPLDPC_LLR_I32) {
                    static_cast<int32_t *>(out)[at] = q;
                } else {
                    if (q < -32768 || q > 32767) overflow[t] = 1;
                    static_cast<int16_t *>(out)[at] = (int16_t)q;
                }
            }
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++) th.emplace_back(work, t);
        for (auto &x : th) x.join();
    }
    for (int t = 0; t < T; t++)
        if (overflow[t]) return fpldpc::fail(FPLDPC_ERR_ARG, "LLR does not fit int16");
    return FPLDPC_OK;
}

}  // extern "C"
