// fpldpc_sim.cpp -- ordered BER/FER simulation around one GPU decoder (fpldpc_ber_sim).
//
// The reference harness decodes one frame at a time and stops at the frame whose decode brings the
// frame-error count to 100 (PerfTest.cpp:97-135, 275-311, 385-426, 485-511, 574-600).  Here frames
// are decoded in chunks on the GPU while the host generates the next chunk's LLRs (two pinned /
// device buffer pairs, one stream, one event per chunk); per-frame error counts come back and are
// accumulated in frame order on the host, so the stop frame and every counter equal the serial
// loop's.  Frames of the last chunk past the stop frame are decoded but not counted.
// With device_channel the LLRs are generated on the device in the decoder's stream instead
// (fpldpc_gen.hip), two chunks in flight, and the host only does the ordered accounting.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "fpldpc_internal.hpp"

using namespace fpldpc;

namespace {

#define SIM_TRY(expr)                                          \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return fail_hip((int)_e, #expr); \
    } while (0)

struct Slot {
    int16_t *h_llr = nullptr;
    int32_t *h_out = nullptr;  // [chunk] bit errors, then [chunk] iterations
    int16_t *d_llr = nullptr;
    int32_t *d_out = nullptr;
    hipEvent_t done = nullptr;
    int frames = 0;
    int64_t first = 0;
};

struct SimBuffers {
    Slot s[2];
    int32_t *d_forced = nullptr;
    ~SimBuffers() {
        (void)hipFree(d_forced);
        for (auto &x : s) {
            (void)hipHostFree(x.h_llr);
            (void)hipHostFree(x.h_out);
            (void)hipFree(x.d_llr);
            (void)hipFree(x.d_out);
            if (x.done) (void)hipEventDestroy(x.done);
        }
    }
};

}  // namespace

extern "C" {

void fpldpc_sim_params_default(fpldpc_sim_params *p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->seed = 123456789;  // rngs.cpp:45
    p->frac_bits = 4;     // ArrayLDPCMacro.h:36
    p->max_frame_errors = 100;  // PerfTest.cpp:97
    p->count_mode = FPLDPC_COUNT_BITS;
}

int fpldpc_ber_sim(fpldpc_decoder_t dec, const fpldpc_sim_params *sp, fpldpc_sim_result *out) {
    if (!dec || !sp || !out) return fail(FPLDPC_ERR_ARG, "null argument");
    const int n = dec->code.n;
    if (sp->max_frame_errors <= 0 && sp->max_frames <= 0)
        return fail(FPLDPC_ERR_ARG, "ber_sim needs max_frame_errors or max_frames");
    if (sp->count_mode != FPLDPC_COUNT_BITS && sp->count_mode != FPLDPC_COUNT_ITERS)
        return fail(FPLDPC_ERR_ARG, "bad count_mode");
    if (sp->count_mode == FPLDPC_COUNT_BITS && (sp->k <= 0 || !sp->info_index || !sp->info_bits))
        return fail(FPLDPC_ERR_ARG, "FPLDPC_COUNT_BITS needs info_index / info_bits");
    if (sp->n_forced < 0 || (sp->n_forced > 0 && !sp->forced_index)) return fail(FPLDPC_ERR_ARG, "bad forced list");
    for (int i = 0; i < sp->n_forced; i++)
        if (sp->forced_index[i] < 0 || sp->forced_index[i] >= n) return fail(FPLDPC_ERR_ARG, "forced index out of range");
    if (sp->forced_llr < -32768 || sp->forced_llr > 32767) return fail(FPLDPC_ERR_ARG, "forced_llr must fit int16");
    int st = FPLDPC_OK;
    if (sp->count_mode == FPLDPC_COUNT_BITS) {
        st = fpldpc_set_reference(dec, sp->info_index, sp->info_bits, sp->k);
        if (st) return st;
    }
    const auto t0 = std::chrono::steady_clock::now();
    int chunk = sp->chunk > 0 ? sp->chunk : 16384;
    if (sp->max_frames > 0) chunk = (int)std::min<int64_t>(chunk, sp->max_frames);

    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(dec->device) != hipSuccess) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    struct Restore {
        int d;
        ~Restore() {
            if (d >= 0) (void)hipSetDevice(d);
        }
    } restore{prev};

    SimBuffers b;
    const size_t llr_bytes = (size_t)chunk * n * sizeof(int16_t);
    for (auto &x : b.s) {
        if (!sp->device_channel) SIM_TRY(hipHostMalloc((void **)&x.h_llr, llr_bytes, hipHostMallocDefault));
        // [chunk] bit errors, [chunk] iterations, [1] int16 overflow count (device channel)
        SIM_TRY(hipHostMalloc((void **)&x.h_out, ((size_t)chunk * 2 + 1) * sizeof(int32_t), hipHostMallocDefault));
        SIM_TRY(hipMalloc((void **)&x.d_llr, llr_bytes));
        SIM_TRY(hipMalloc((void **)&x.d_out, ((size_t)chunk * 2 + 1) * sizeof(int32_t)));
        SIM_TRY(hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
    }
    hipStream_t s = dec->stream;
    const uint8_t *d_cw = nullptr;
    if (sp->device_channel) {
        if (sp->codeword) {
            SIM_TRY(hipMalloc((void **)&b.d_forced, sizeof(int32_t) * std::max(sp->n_forced, 0) + n));
            d_cw = reinterpret_cast<const uint8_t *>(b.d_forced + std::max(sp->n_forced, 0));
            SIM_TRY(hipMemcpy((void *)d_cw, sp->codeword, n, hipMemcpyHostToDevice));
        } else if (sp->n_forced > 0) {
            SIM_TRY(hipMalloc((void **)&b.d_forced, sizeof(int32_t) * sp->n_forced));
        }
        if (sp->n_forced > 0)
            SIM_TRY(hipMemcpy(b.d_forced, sp->forced_index, sizeof(int32_t) * sp->n_forced, hipMemcpyHostToDevice));
    }

    int64_t next_frame = sp->first_frame;  // next frame to generate
    const int64_t frame_end = sp->max_frames > 0 ? sp->first_frame + sp->max_frames : INT64_MAX;
    auto generate = [&](Slot &x) -> int {
        const int64_t left = frame_end - next_frame;
        x.frames = (int)std::min<int64_t>(chunk, left);
        if (x.frames <= 0) return FPLDPC_OK;
        x.first = next_frame;
        if (sp->device_channel) {  // generated on the device by submit()
            next_frame += x.frames;
            return FPLDPC_OK;
        }
        int r = fpldpc_channel_llr_host(sp->seed, next_frame, x.frames, n, sp->snr, sp->sigma, sp->frac_bits,
                                        sp->codeword, x.h_llr, FPLDPC_LLR_I16, sp->host_threads);
        if (r) return r;
        for (int f = 0; f < x.frames; f++)
            for (int i = 0; i < sp->n_forced; i++) x.h_llr[(size_t)f * n + sp->forced_index[i]] = (int16_t)sp->forced_llr;
        next_frame += x.frames;
        return FPLDPC_OK;
    };
    auto submit = [&](Slot &x) -> int {
        if (x.frames <= 0) return FPLDPC_OK;
        int r;
        if (sp->device_channel) {
            int32_t *ovf = x.d_out + 2 * (size_t)chunk;
            SIM_TRY(hipMemsetAsync(ovf, 0, sizeof(int32_t), s));
            if ((r = launch_channel(sp->seed, x.first, x.frames, n, sp->snr, sp->sigma, sp->frac_bits, d_cw, 0, x.d_llr,
                                    FPLDPC_LLR_I16, ovf, s)))
                return r;
            if (sp->n_forced > 0 &&
                (r = launch_force_llr(x.d_llr, x.frames, n, b.d_forced, sp->n_forced, (int16_t)sp->forced_llr, s)))
                return r;
            SIM_TRY(hipMemcpyAsync(x.h_out + 2 * (size_t)chunk, ovf, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        } else {
            SIM_TRY(hipMemcpyAsync(x.d_llr, x.h_llr, (size_t)x.frames * n * sizeof(int16_t), hipMemcpyHostToDevice, s));
        }
        r = fpldpc_decode(dec, x.d_llr, FPLDPC_LLR_I16, x.frames, nullptr, x.d_out + chunk, nullptr, nullptr,
                              sp->count_mode == FPLDPC_COUNT_BITS ? x.d_out : nullptr, nullptr, s);
        if (r) return r;
        if (sp->count_mode == FPLDPC_COUNT_BITS)
            SIM_TRY(hipMemcpyAsync(x.h_out, x.d_out, (size_t)x.frames * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        SIM_TRY(hipMemcpyAsync(x.h_out + chunk, x.d_out + chunk, (size_t)x.frames * sizeof(int32_t),
                               hipMemcpyDeviceToHost, s));
        SIM_TRY(hipEventRecord(x.done, s));
        return FPLDPC_OK;
    };

    fpldpc_sim_result r{};
    bool stop = false;
    int cur = 0;
    if ((st = generate(b.s[0]))) return st;
    if ((st = submit(b.s[0]))) return st;
    while (b.s[cur].frames > 0) {
        Slot &x = b.s[cur], &y = b.s[cur ^ 1];
        // overlap: next chunk's channel on the host while the GPU decodes this one
        y.frames = 0;
        if (!stop && next_frame < frame_end) {
            if ((st = generate(y))) return st;
        }
        SIM_TRY(hipEventSynchronize(x.done));
        if (sp->device_channel && x.h_out[2 * (size_t)chunk] != 0)
            return fail(FPLDPC_ERR_ARG, "LLR does not fit int16");  // as the host channel
        r.frames_decoded += x.frames;
        for (int f = 0; f < x.frames && !stop; f++) {
            const int it = x.h_out[chunk + f];
            const int64_t blk = sp->count_mode == FPLDPC_COUNT_BITS ? x.h_out[f] : it;
            if (sp->on_frame) sp->on_frame(sp->on_frame_ctx, sp->first_frame + r.frames, it, blk);
            r.frames++;
            r.iter_sum += it;
            r.bit_errors += blk;
            if (blk > 0) r.frame_errors++;
            if (sp->max_frame_errors > 0 && r.frame_errors >= sp->max_frame_errors) stop = true;
        }
        if (stop) {
            if (y.frames > 0) y.frames = 0;  // generated but not needed
            break;
        }
        if ((st = submit(y))) return st;
        cur ^= 1;
    }
    SIM_TRY(hipStreamSynchronize(s));
    r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = r;
    return FPLDPC_OK;
}

}  // extern "C"
