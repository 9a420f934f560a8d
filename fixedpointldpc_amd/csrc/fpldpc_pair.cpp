// fpldpc_pair.cpp -- one batch as two launches in flight: frames [0, h) on decoder a, [h, batch) on
// decoder b (same code and parameters), each on its own stream, joined to the caller's.  A single
// persistent launch ends with a tail in which few CUs still hold frames (a frame pulled late that
// runs all iterations, or the youngest workgroup of a CU finishing alone); the second
// launch's workgroups take those CUs as the first's leave.  The same frames, the same kernels, so
// the outputs are those of fpldpc_decode on the whole batch (GPU tests compare them); only the
// schedule differs.  Host orchestration only: no kernel or launch argument changes here.
#include <hip/hip_runtime.h>

#include <cstring>

#include "fpldpc.h"
#include "fpldpc_internal.hpp"

using namespace fpldpc;

namespace {

#define PAIR_TRY(expr)                                         \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return fail_hip((int)_e, #expr); \
    } while (0)

struct Guard {
    int prev = -1;
    bool ok = true;
    explicit Guard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~Guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int check_pair(fpldpc_decoder_t a, fpldpc_decoder_t b, int32_t batch, const void *llr, int32_t llr_type) {
    if (!a || !b) return fail(FPLDPC_ERR_ARG, "null decoder");
    if (a == b) return fail(FPLDPC_ERR_ARG, "decode_pair: the two decoders must be distinct (one stream each)");
    if (a->device != b->device) return fail(FPLDPC_ERR_ARG, "decode_pair: decoders on different devices");
    if (a->code.n != b->code.n || a->code.m != b->code.m || a->code.clist != b->code.clist)
        return fail(FPLDPC_ERR_ARG, "decode_pair: decoders of different codes");
    if (std::memcmp(&a->params, &b->params, sizeof(fpldpc_params)) != 0)
        return fail(FPLDPC_ERR_ARG, "decode_pair: decoders with different parameters");
    if (batch < 0) return fail(FPLDPC_ERR_ARG, "negative batch");
    if (batch > 0 && !llr) return fail(FPLDPC_ERR_ARG, "null llr");
    if (llr_type != FPLDPC_LLR_I32 && llr_type != FPLDPC_LLR_I16) return fail(FPLDPC_ERR_ARG, "bad llr_type");
    return FPLDPC_OK;
}

template <class T>
T *at(T *p, size_t off) {
    return p ? p + off : nullptr;
}

}  // namespace

extern "C" {

int fpldpc_decode_pair(fpldpc_decoder_t a, fpldpc_decoder_t b, const void *llr, int32_t llr_type, int32_t batch,
                       uint32_t *hard, int32_t *iters, uint8_t *syndrome_ok, int32_t *post, int32_t *bit_errors,
                       int64_t *totals, void *stream, void *stream_b) {
    int st = check_pair(a, b, batch, llr, llr_type);
    if (st) return st;
    if (batch < 2) return fpldpc_decode(a, llr, llr_type, batch, hard, iters, syndrome_ok, post, bit_errors, totals, stream);
    if (stream_b == stream) return fail(FPLDPC_ERR_ARG, "decode_pair: the second stream must differ from the first");
    Guard g(a->device);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    hipStream_t sa = (hipStream_t)stream, sb = (hipStream_t)stream_b;
    const size_t n = a->code.n, hw = (n + 31) / 32, h = (size_t)batch / 2, es = llr_type == FPLDPC_LLR_I16 ? 2 : 4;
    hipEvent_t fork = nullptr, join = nullptr;
    PAIR_TRY(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    hipError_t e = hipEventCreateWithFlags(&join, hipEventDisableTiming);
    if (e != hipSuccess) {
        (void)hipEventDestroy(fork);
        return fail_hip((int)e, "hipEventCreateWithFlags");
    }
    // b's half starts after everything the caller queued on stream (inputs, zeroed totals ...)
    e = hipEventRecord(fork, sa);
    if (e == hipSuccess) e = hipStreamWaitEvent(sb, fork, 0);
    if (e == hipSuccess) {
        st = fpldpc_decode(a, llr, llr_type, (int32_t)h, hard, iters, syndrome_ok, post, bit_errors, totals, stream);
        if (!st)
            st = fpldpc_decode(b, static_cast<const char *>(llr) + h * n * es, llr_type, (int32_t)(batch - h),
                               at(hard, h * hw), at(iters, h), at(syndrome_ok, h), at(post, h * n), at(bit_errors, h),
                               totals, stream_b);
        // the caller's stream continues after both halves
        if (!st) e = hipEventRecord(join, sb);
        if (!st && e == hipSuccess) e = hipStreamWaitEvent(sa, join, 0);
    }
    (void)hipEventDestroy(fork);
    (void)hipEventDestroy(join);
    if (st) return st;
    if (e != hipSuccess) return fail_hip((int)e, "decode_pair: stream join");
    return FPLDPC_OK;
}

int fpldpc_decode_pair_host(fpldpc_decoder_t a, fpldpc_decoder_t b, const void *llr, int32_t llr_type, int32_t batch,
                            uint32_t *hard, int32_t *iters, uint8_t *syndrome_ok, int32_t *post, int32_t *bit_errors,
                            int64_t *totals) {
    int st = check_pair(a, b, batch, llr, llr_type);
    if (st) return st;
    if (batch < 2) return fpldpc_decode_host(a, llr, llr_type, batch, hard, iters, syndrome_ok, post, bit_errors, totals);
    Guard g(a->device);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    const size_t n = a->code.n, hw = (n + 31) / 32, es = llr_type == FPLDPC_LLR_I16 ? 2 : 4;
    const size_t half[2] = {(size_t)batch / 2, (size_t)batch - (size_t)batch / 2}, first[2] = {0, half[0]};
    fpldpc_decoder_t dec[2] = {a, b};
    int64_t tot[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    if (totals) std::memcpy(tot[0], totals, sizeof(tot[0]));
    // each half staged through its own decoder's device buffer, on its own stream (as fpldpc_decode_host)
    for (int i = 0; i < 2; ++i) {
        fpldpc_decoder_t d = dec[i];
        const size_t B = half[i], f0 = first[i];
        auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t llr_b = align(B * n * es), hard_b = align(B * hw * 4), it_b = align(B * 4), ok_b = align(B),
                     post_b = align(B * n * 4), be_b = align(B * 4), tot_b = align(32);
        const size_t need = llr_b + hard_b + it_b + ok_b + post_b + be_b + tot_b;
        if (need > d->stage_bytes) {
            PAIR_TRY(hipStreamSynchronize(d->stream));
            (void)hipFree(d->d_stage);
            d->d_stage = nullptr;
            d->stage_bytes = 0;
            PAIR_TRY(hipMalloc(&d->d_stage, need));
            d->stage_bytes = need;
        }
        char *p = static_cast<char *>(d->d_stage);
        void *d_llr = p;
        uint32_t *d_hard = hard ? reinterpret_cast<uint32_t *>(p + llr_b) : nullptr;
        int32_t *d_it = iters ? reinterpret_cast<int32_t *>(p + llr_b + hard_b) : nullptr;
        uint8_t *d_ok = syndrome_ok ? reinterpret_cast<uint8_t *>(p + llr_b + hard_b + it_b) : nullptr;
        int32_t *d_post = post ? reinterpret_cast<int32_t *>(p + llr_b + hard_b + it_b + ok_b) : nullptr;
        int32_t *d_be = bit_errors ? reinterpret_cast<int32_t *>(p + llr_b + hard_b + it_b + ok_b + post_b) : nullptr;
        int64_t *d_tot = totals ? reinterpret_cast<int64_t *>(p + llr_b + hard_b + it_b + ok_b + post_b + be_b) : nullptr;
        hipStream_t s = d->stream;
        PAIR_TRY(hipMemcpyAsync(d_llr, static_cast<const char *>(llr) + f0 * n * es, B * n * es, hipMemcpyHostToDevice, s));
        // posteriors left untouched on a pre-check pass: seed each half with the caller's buffer
        if (d_post) PAIR_TRY(hipMemcpyAsync(d_post, post + f0 * n, B * n * 4, hipMemcpyHostToDevice, s));
        if (d_tot) PAIR_TRY(hipMemcpyAsync(d_tot, tot[i], 32, hipMemcpyHostToDevice, s));
        st = fpldpc_decode(d, d_llr, llr_type, (int32_t)B, d_hard, d_it, d_ok, d_post, d_be, d_tot, s);
        if (st) return st;
        if (d_hard) PAIR_TRY(hipMemcpyAsync(hard + f0 * hw, d_hard, B * hw * 4, hipMemcpyDeviceToHost, s));
        if (d_it) PAIR_TRY(hipMemcpyAsync(iters + f0, d_it, B * 4, hipMemcpyDeviceToHost, s));
        if (d_ok) PAIR_TRY(hipMemcpyAsync(syndrome_ok + f0, d_ok, B, hipMemcpyDeviceToHost, s));
        if (d_post) PAIR_TRY(hipMemcpyAsync(post + f0 * n, d_post, B * n * 4, hipMemcpyDeviceToHost, s));
        if (d_be) PAIR_TRY(hipMemcpyAsync(bit_errors + f0, d_be, B * 4, hipMemcpyDeviceToHost, s));
        if (d_tot) PAIR_TRY(hipMemcpyAsync(tot[i], d_tot, 32, hipMemcpyDeviceToHost, s));
    }
    PAIR_TRY(hipStreamSynchronize(a->stream));
    PAIR_TRY(hipStreamSynchronize(b->stream));
    if (totals)
        for (int c = 0; c < 4; ++c) totals[c] = tot[0][c] + tot[1][c];
    return FPLDPC_OK;
}

}  // extern "C"
