// fpldpc_decoder.cpp -- decoder objects and the decode entry points of the C ABI (include/fpldpc.h).
//
// Replaces the reference's FP_Decoder state (ArrayLDPCMacro.h:121-176) by a device-resident
// description of the code (slot-major var-index table, check degrees) plus the kernel choice.
// There is no CPU decode path here: without a usable HIP device every decode call fails loudly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "fpldpc_internal.hpp"

using namespace fpldpc;


namespace {

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

#define HIP_TRY(expr)                                             \
    do {                                                          \
        hipError_t _e = (expr);                                   \
        if (_e != hipSuccess) return fail_hip((int)_e, #expr);    \
    } while (0)

void free_decoder(fpldpc_decoder *d) {
    if (!d) return;
    DeviceGuard g(d->device);
    (void)hipFree(d->d_vidx);
    (void)hipFree(d->d_cdeg);
    (void)hipFree(d->d_counter);
    (void)hipFree(d->d_scratch);
    (void)hipFree(d->d_fb_list);
    if (d->h_probe) (void)hipHostFree(d->h_probe);
    if (d->h_wgtrace) (void)hipHostFree(d->h_wgtrace);
    (void)hipFree(d->d_info_idx);
    (void)hipFree(d->d_info_bits);
    (void)hipFree(d->d_info_mask);
    (void)hipFree(d->d_stage);
    (void)hipFree(d->edges.vidx);
    (void)hipFree(d->edges.cdeg);
    (void)hipFree(d->edges.c2v);
    (void)hipFree(d->d_edge_stage);
    if (d->h_edge_stage) (void)hipHostFree(d->h_edge_stage);
    free_float_state(d->fl);
    if (d->last_done) (void)hipEventDestroy(d->last_done);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

// fpldpc_decode_frame's index table in the code's own check order (clist order per check), built on
// first use: slot k of check c -> var, [dc_max][m]; c2v scratch [2][edge_kernel_dc][m].
int edge_tables(fpldpc_decoder *d) {
    fpldpc::EdgeTables &t = d->edges;
    if (t.vidx) return FPLDPC_OK;
    const fpldpc_code &c = d->code;
    const int dc = edge_kernel_dc(c.dc_max);
    if (!dc) return fail(FPLDPC_ERR_UNSUPPORTED, "check degree above 64");
    std::vector<uint16_t> vidx((size_t)c.dc_max * c.m, 0);
    std::vector<uint8_t> cdeg(c.m);
    for (int r = 0; r < c.m; r++) {
        cdeg[r] = (uint8_t)c.cdeg[r];
        for (int k = 0; k < c.cdeg[r]; k++) vidx[(size_t)k * c.m + r] = (uint16_t)c.clist[(size_t)r * c.dc_max + k];
    }
    fpldpc::EdgeTables n;
    n.n = c.n;
    n.m = c.m;
    n.dc = dc;
    n.dc_max = c.dc_max;
    hipError_t e = hipMalloc(&n.vidx, vidx.size() * sizeof(uint16_t));
    if (e == hipSuccess) e = hipMemcpy(n.vidx, vidx.data(), vidx.size() * sizeof(uint16_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&n.cdeg, cdeg.size());
    if (e == hipSuccess) e = hipMemcpy(n.cdeg, cdeg.data(), cdeg.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&n.c2v, sizeof(int32_t) * 2 * (size_t)dc * c.m);
    if (e != hipSuccess) {
        (void)hipFree(n.vidx);
        (void)hipFree(n.cdeg);
        (void)hipFree(n.c2v);
        return fail_hip((int)e, "edge tables");
    }
    t = n;
    return FPLDPC_OK;
}

// Constant = int((5.0/8.0) * (1 << FRAC_WIDTH)) (ArrayLDPCMacro.h:175)
int constant_c(int frac_bits) { return (int)((5.0 / 8.0) * (1 << frac_bits)); }

int check_params(const fpldpc_params &p) {
    if (p.max_iter < 1 || p.max_iter > 100000) return fail(FPLDPC_ERR_ARG, "max_iter out of range (1..100000)");
    if (p.frac_bits < 0 || p.frac_bits > 16) return fail(FPLDPC_ERR_ARG, "frac_bits out of range");
    if (p.width_mask <= 0) return fail(FPLDPC_ERR_ARG, "width_mask must be positive");
    return FPLDPC_OK;
}

}  // namespace

extern "C" {

void fpldpc_params_default(fpldpc_params *p) {
    if (!p) return;
    p->max_iter = 30;     // ArrayLDPCMacro.h:17
    p->frac_bits = 4;     // ArrayLDPCMacro.h:36
    p->width_mask = 0xff; // ArrayLDPCMacro.h:29
    p->early_term = 1;    // ArrayLDPC_Decoder.cpp:164-167
    p->precheck = 0;
    p->device = -1;
}

}  // extern "C"

namespace {

// kc: the kernel choice to use (a twin takes its source's), or null to choose one for the code and
// device (FPLDPC_KERNEL may force it); diag: read the diagnostic switches from the environment.
int create_decoder(const fpldpc_code *code, const fpldpc_params *params, const KernelChoice *kc, bool diag,
                   fpldpc_decoder_t *out) {
    if (!code || !out) return fail(FPLDPC_ERR_ARG, "null argument");
    fpldpc_params p;
    fpldpc_params_default(&p);
    if (params) p = *params;
    int st = check_params(p);
    if (st) return st;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(FPLDPC_ERR_HIP, "no HIP device available (the decoder has no CPU path)");
    int dev = p.device;
    if (dev < 0) HIP_TRY(hipGetDevice(&dev));
    if (dev >= ndev) return fail(FPLDPC_ERR_ARG, "device ordinal out of range");
    DeviceGuard g(dev);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");

    std::unique_ptr<fpldpc_decoder, void (*)(fpldpc_decoder *)> d(new fpldpc_decoder(), free_decoder);
    d->code = *code;
    d->params = p;
    d->device = dev;
    if (kc) {
        d->kc = *kc;
    } else {
        st = choose_kernel(d->code, dev, p.width_mask, constant_c(p.frac_bits), &d->kc);
        if (st) return st;
    }

    const fpldpc_code &c = d->code;
    const int DC = kernel_dc(d->kc.v);
    const int m_pad = (c.m + 63) / 64 * 64;
    // Slot-major var-index table: vidx[k][j] = clist[c][k] (fold order) for the check c in column j,
    // 0 in unused slots so that every gather stays in bounds.  Columns are the checks in code order,
    // or by ascending degree (stable) for variants whose first passes fold a fixed degree: the
    // decode does not depend on check order (each check folds its own edges; posterior sums are
    // integer adds).
    std::vector<int> order(c.m);
    for (int r = 0; r < c.m; r++) order[r] = r;
    if (d->kc.sort_checks)
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return c.cdeg[x] < c.cdeg[y]; });
    std::vector<uint16_t> vidx((size_t)DC * m_pad, 0);
    std::vector<uint8_t> cdeg(c.m);
    for (int j = 0; j < c.m; j++) {
        const int r = order[j];
        cdeg[j] = (uint8_t)c.cdeg[r];
        for (int k = 0; k < c.cdeg[r]; k++) vidx[(size_t)k * m_pad + j] = (uint16_t)c.clist[(size_t)r * c.dc_max + k];
    }
    HIP_TRY(hipMalloc(&d->d_vidx, vidx.size() * sizeof(uint16_t)));
    HIP_TRY(hipMemcpy(d->d_vidx, vidx.data(), vidx.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&d->d_cdeg, cdeg.size()));
    HIP_TRY(hipMemcpy(d->d_cdeg, cdeg.data(), cdeg.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&d->d_counter, kCounterInts * sizeof(int32_t)));  // zero between calls (chain_exit)
    HIP_TRY(hipMemset(d->d_counter, 0, kCounterInts * sizeof(int32_t)));
    if (d->kc.scratch_ints) HIP_TRY(hipMalloc(&d->d_scratch, d->kc.scratch_ints * sizeof(int32_t)));
    HIP_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&d->last_done, hipEventDisableTiming));
    d->dcode.n = c.n;
    d->dcode.m = c.m;
    d->dcode.dc = DC;
    d->dcode.m_pad = m_pad;
    d->dcode.vidx = d->d_vidx;
    d->dcode.cdeg = d->d_cdeg;
    // Diagnostics, read once here rather than on every decode call (see fpldpc_decode)
    if (const char *sp = getenv("FPLDPC_SPLIT_TAIL")) d->split_tail = *sp != '0';
    if (diag) {
        const char *probe_env = getenv("FPLDPC_CLOCK_PROBE");
        d->diag_probe = probe_env && *probe_env == '1';
        if (const char *t = getenv("FPLDPC_WG_TRACE")) d->diag_trace_path = t;
    }
    *out = d.release();
    return FPLDPC_OK;
}

}  // namespace

namespace fpldpc {
int decoder_create_twin(fpldpc_decoder_t src, fpldpc_decoder_t *out) {
    if (!src) return fail(FPLDPC_ERR_ARG, "null decoder");
    fpldpc_params p = src->params;
    p.device = src->device;
    return create_decoder(&src->code, &p, &src->kc, false, out);
}
}  // namespace fpldpc

extern "C" {

int fpldpc_decoder_create(fpldpc_code_t code, const fpldpc_params *params, fpldpc_decoder_t *out) {
    return create_decoder(code, params, nullptr, true, out);
}

int fpldpc_decoder_destroy(fpldpc_decoder_t dec) {
    free_decoder(dec);
    return FPLDPC_OK;
}

int fpldpc_decoder_describe(fpldpc_decoder_t dec, char *buf, size_t cap) {
    if (!dec || !buf || cap == 0) return fail(FPLDPC_ERR_ARG, "null argument");
    snprintf(buf, cap, "%s grid=%d threads=%d lds=%zu device=%d", dec->kc.name, dec->kc.grid, dec->kc.threads,
             dec->kc.lds_bytes, dec->device);
    return FPLDPC_OK;
}

int fpldpc_decoder_hard_words(fpldpc_decoder_t dec) {
    if (!dec) return fail(FPLDPC_ERR_ARG, "null argument");
    return (dec->code.n + 31) / 32;
}

int fpldpc_decoder_fallback_counts(fpldpc_decoder_t dec, int32_t counts[2]) {
    if (!dec || !counts) return fail(FPLDPC_ERR_ARG, "null argument");
    counts[0] = counts[1] = 0;
    if (dec->kc.fallback == Variant::kNone) return FPLDPC_OK;
    DeviceGuard g(dec->device);
    // the last call's counts are final once its kernels are done, on whichever stream they ran
    HIP_TRY(hipEventSynchronize(dec->last_done));
    int32_t c[kCounterInts];
    HIP_TRY(hipMemcpy(c, dec->d_counter, sizeof c, hipMemcpyDeviceToHost));
    counts[0] = c[kCountFb0Last];
    counts[1] = c[kCountFb1Last];
    return FPLDPC_OK;
}

int fpldpc_set_reference(fpldpc_decoder_t dec, const int32_t *info_index, const uint8_t *info_bits, int32_t k) {
    if (!dec || k < 0 || (k > 0 && (!info_index || !info_bits))) return fail(FPLDPC_ERR_ARG, "bad reference");
    for (int i = 0; i < k; i++)
        if (info_index[i] < 0 || info_index[i] >= dec->code.n) return fail(FPLDPC_ERR_ARG, "info index out of range");
    DeviceGuard g(dec->device);
    (void)hipFree(dec->d_info_idx);
    (void)hipFree(dec->d_info_bits);
    (void)hipFree(dec->d_info_mask);
    dec->d_info_idx = nullptr;
    dec->d_info_bits = nullptr;
    dec->d_info_mask = nullptr;
    dec->k_info = 0;
    if (k == 0) return FPLDPC_OK;
    std::vector<uint8_t> bits(info_bits, info_bits + k);
    for (auto &b : bits) b &= 1;
    HIP_TRY(hipMalloc(&dec->d_info_idx, sizeof(int32_t) * k));
    HIP_TRY(hipMalloc(&dec->d_info_bits, k));
    HIP_TRY(hipMemcpy(dec->d_info_idx, info_index, sizeof(int32_t) * k, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dec->d_info_bits, bits.data(), k, hipMemcpyHostToDevice));
    // distinct positions: the packed form the packed kernels count from their hard-decision words
    const int hw = (dec->code.n + 31) / 32;
    std::vector<uint32_t> mk(2 * (size_t)hw, 0);
    bool distinct = true;
    for (int i = 0; i < k && distinct; i++) {
        const int v = info_index[i];
        if (mk[v / 32] >> (v % 32) & 1) distinct = false;
        mk[v / 32] |= 1u << (v % 32);
        mk[hw + v / 32] |= (uint32_t)bits[i] << (v % 32);
    }
    if (distinct) {
        HIP_TRY(hipMalloc(&dec->d_info_mask, mk.size() * sizeof(uint32_t)));
        HIP_TRY(hipMemcpy(dec->d_info_mask, mk.data(), mk.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    dec->k_info = k;
    return FPLDPC_OK;
}

int fpldpc_decode(fpldpc_decoder_t dec, const void *llr, int32_t llr_type, int32_t batch, uint32_t *hard,
                  int32_t *iters, uint8_t *syndrome_ok, int32_t *post, int32_t *bit_errors, int64_t *totals,
                  void *stream) {
    if (!dec) return fail(FPLDPC_ERR_ARG, "null decoder");
    if (batch < 0) return fail(FPLDPC_ERR_ARG, "negative batch");
    if (batch == 0) return FPLDPC_OK;
    if (!llr) return fail(FPLDPC_ERR_ARG, "null llr");
    if (llr_type != FPLDPC_LLR_I32 && llr_type != FPLDPC_LLR_I16) return fail(FPLDPC_ERR_ARG, "bad llr_type");
    if (bit_errors && dec->k_info == 0) return fail(FPLDPC_ERR_ARG, "bit_errors requested without fpldpc_set_reference");
    DeviceGuard g(dec->device);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    LaunchArgs a;
    a.llr = llr;
    a.llr_i16 = llr_type == FPLDPC_LLR_I16;
    a.batch = batch;
    a.max_iter = dec->params.max_iter;
    a.C = constant_c(dec->params.frac_bits);
    a.mask = dec->params.width_mask;
    a.early_term = dec->params.early_term;
    a.precheck = dec->params.precheck;
    a.hard = hard;
    a.hard_words = (dec->code.n + 31) / 32;
    a.iters = iters;
    a.syn_ok = syndrome_ok;
    a.post = post;
    a.bit_errors = bit_errors;
    a.totals = reinterpret_cast<unsigned long long *>(totals);
    a.info_idx = dec->d_info_idx;
    a.info_bits = dec->d_info_bits;
    a.k_info = dec->k_info;
    a.info_mask = dec->d_info_mask;
    a.work_counter = dec->d_counter;
    a.c2v_scratch = dec->d_scratch;
    a.bfe_w = (uint32_t)std::max(0, __builtin_popcount((unsigned)a.mask) - 2);
    a.split_tail = dec->split_tail ? 1 : 0;
    if (dec->kc.fallback != Variant::kNone) {
        if (batch > dec->fb_cap) {  // grows to the largest batch seen (not inside graph capture)
            (void)hipFree(dec->d_fb_list);
            dec->d_fb_list = nullptr;
            dec->fb_cap = 0;
            HIP_TRY(hipMalloc(&dec->d_fb_list, sizeof(int) * (size_t)batch * dec->kc.lists()));
            dec->fb_cap = batch;
        }
        a.fb_list = dec->d_fb_list;
    }
    // Diagnostic: FPLDPC_CLOCK_PROBE=1 (at decoder creation) stamps workgroup 0's shader clock
    // (s_memtime) against the 100 MHz s_memrealtime around the kernel and prints the in-kernel clock
    // (synchronises).
    const bool probe = dec->diag_probe;
    if (probe && !dec->h_probe) HIP_TRY(hipHostMalloc((void **)&dec->h_probe, 64, hipHostMallocMapped));
    if (probe) {
        memset(dec->h_probe, 0, 64);
        a.probe = dec->h_probe;
    }
    // Diagnostic: FPLDPC_WG_TRACE=<file> (at decoder creation) writes, after each call, every
    // workgroup's {xcc<<32 | HW_ID, start, end (100 MHz s_memrealtime), frames pulled, 4 reserved
    // words} of the packed kernels as raw uint64 [grid][8].
    const char *trace_path = dec->diag_trace_path.empty() ? nullptr : dec->diag_trace_path.c_str();
    if (trace_path) {
        // [grid][8] per workgroup, then [grid][64] per wave (the FPLDPC_WAIT_TRACE diagnostic build)
        if (!dec->h_wgtrace)
            HIP_TRY(hipHostMalloc((void **)&dec->h_wgtrace, sizeof(unsigned long long) * 72 * dec->kc.grid, hipHostMallocMapped));
        memset(dec->h_wgtrace, 0, sizeof(unsigned long long) * 72 * dec->kc.grid);
        a.wgtrace = dec->h_wgtrace;
    }
    int st = launch_decode(dec->kc, dec->dcode, a, stream);
    if (!st && dec->kc.fallback != Variant::kNone) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIP_TRY(hipStreamIsCapturing((hipStream_t)stream, &cs));
        if (cs == hipStreamCaptureStatusNone) HIP_TRY(hipEventRecord(dec->last_done, (hipStream_t)stream));
    }
    if (!st && a.wgtrace) {
        HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
        if (FILE *f = fopen(trace_path, "wb")) {
            fwrite(dec->h_wgtrace, sizeof(unsigned long long), 8 * (size_t)dec->kc.grid, f);
            fclose(f);
        }
        const unsigned long long *w = dec->h_wgtrace + 8 * (size_t)dec->kc.grid;
        if (std::any_of(w, w + 64 * (size_t)dec->kc.grid, [](unsigned long long x) { return x != 0; }))
            if (FILE *f = fopen((dec->diag_trace_path + ".waves").c_str(), "wb")) {
                fwrite(w, sizeof(unsigned long long), 64 * (size_t)dec->kc.grid, f);
                fclose(f);
            }
    }
    if (st || !probe) return st;
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    const unsigned long long *q = dec->h_probe;
    if (q[2] > q[0] && q[3] > q[1])
        fprintf(stderr, "fpldpc clock probe: %.0f MHz (workgroup 0: %llu cycles in %.3f ms)\n",
                (double)(q[2] - q[0]) / (double)(q[3] - q[1]) * 100.0, q[2] - q[0], (q[3] - q[1]) * 1e-5);
    return st;
}

int fpldpc_decode_host(fpldpc_decoder_t dec, const void *llr, int32_t llr_type, int32_t batch, uint32_t *hard,
                       int32_t *iters, uint8_t *syndrome_ok, int32_t *post, int32_t *bit_errors, int64_t *totals) {
    if (!dec) return fail(FPLDPC_ERR_ARG, "null decoder");
    if (batch < 0) return fail(FPLDPC_ERR_ARG, "negative batch");
    if (batch == 0) return FPLDPC_OK;  // (as fpldpc_decode: an empty batch needs no buffers)
    if (!llr) return fail(FPLDPC_ERR_ARG, "null llr");
    if (llr_type != FPLDPC_LLR_I32 && llr_type != FPLDPC_LLR_I16) return fail(FPLDPC_ERR_ARG, "bad llr_type");
    DeviceGuard g(dec->device);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    const size_t n = dec->code.n, hw = (n + 31) / 32, B = batch;
    auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t llr_b = align(B * n * (llr_type == FPLDPC_LLR_I16 ? 2 : 4));
    const size_t hard_b = align(B * hw * 4), it_b = align(B * 4), ok_b = align(B), post_b = align(B * n * 4),
                 be_b = align(B * 4), tot_b = align(32);
    const size_t need = llr_b + hard_b + it_b + ok_b + post_b + be_b + tot_b;
    if (need > dec->stage_bytes) {
        (void)hipFree(dec->d_stage);
        dec->d_stage = nullptr;
        dec->stage_bytes = 0;
        HIP_TRY(hipMalloc(&dec->d_stage, need));
        dec->stage_bytes = need;
    }
    char *p = static_cast<char *>(dec->d_stage);
    void *d_llr = p;
    p += llr_b;
    uint32_t *d_hard = hard ? reinterpret_cast<uint32_t *>(p) : nullptr;
    p += hard_b;
    int32_t *d_it = iters ? reinterpret_cast<int32_t *>(p) : nullptr;
    p += it_b;
    uint8_t *d_ok = syndrome_ok ? reinterpret_cast<uint8_t *>(p) : nullptr;
    p += ok_b;
    int32_t *d_post = post ? reinterpret_cast<int32_t *>(p) : nullptr;
    p += post_b;
    int32_t *d_be = bit_errors ? reinterpret_cast<int32_t *>(p) : nullptr;
    p += be_b;
    int64_t *d_tot = totals ? reinterpret_cast<int64_t *>(p) : nullptr;
    hipStream_t s = dec->stream;
    HIP_TRY(hipMemcpyAsync(d_llr, llr, B * n * (llr_type == FPLDPC_LLR_I16 ? 2 : 4), hipMemcpyHostToDevice, s));
    // Posteriors are left untouched on a pre-check pass (the reference keeps the previous frame's
    // Posteriori_fp, ArrayLDPC_Decoder.cpp:443-450): seed the device copy with the caller's buffer.
    if (d_post) HIP_TRY(hipMemcpyAsync(d_post, post, B * n * 4, hipMemcpyHostToDevice, s));
    if (d_tot) HIP_TRY(hipMemcpyAsync(d_tot, totals, 32, hipMemcpyHostToDevice, s));
    int st = fpldpc_decode(dec, d_llr, llr_type, batch, d_hard, d_it, d_ok, d_post, d_be, d_tot, s);
    if (st) return st;
    if (d_hard) HIP_TRY(hipMemcpyAsync(hard, d_hard, B * hw * 4, hipMemcpyDeviceToHost, s));
    if (d_it) HIP_TRY(hipMemcpyAsync(iters, d_it, B * 4, hipMemcpyDeviceToHost, s));
    if (d_ok) HIP_TRY(hipMemcpyAsync(syndrome_ok, d_ok, B, hipMemcpyDeviceToHost, s));
    if (d_post) HIP_TRY(hipMemcpyAsync(post, d_post, B * n * 4, hipMemcpyDeviceToHost, s));
    if (d_be) HIP_TRY(hipMemcpyAsync(bit_errors, d_be, B * 4, hipMemcpyDeviceToHost, s));
    if (d_tot) HIP_TRY(hipMemcpyAsync(totals, d_tot, 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FPLDPC_OK;
}

int fpldpc_edge_ram_words(fpldpc_decoder_t dec, int64_t *words) {
    if (!dec || !words) return fail(FPLDPC_ERR_ARG, "null argument");
    *words = (int64_t)dec->code.dc_max * dec->code.m;
    return FPLDPC_OK;
}

int fpldpc_decode_frame(fpldpc_decoder_t dec, const void *llr, int32_t llr_type, int32_t keep_edges, int32_t *edge_ram,
                        uint32_t *hard, int32_t *iters, uint8_t *syndrome_ok, int32_t *post, void *stream) {
    if (!dec) return fail(FPLDPC_ERR_ARG, "null decoder");
    if (!llr || !edge_ram) return fail(FPLDPC_ERR_ARG, "null llr or edge RAM");
    if (llr_type != FPLDPC_LLR_I32 && llr_type != FPLDPC_LLR_I16) return fail(FPLDPC_ERR_ARG, "bad llr_type");
    DeviceGuard g(dec->device);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    int st = edge_tables(dec);
    if (st) return st;
    LaunchArgs a;
    a.llr = llr;
    a.llr_i16 = llr_type == FPLDPC_LLR_I16;
    a.batch = 1;
    a.max_iter = dec->params.max_iter;
    a.C = constant_c(dec->params.frac_bits);
    a.mask = dec->params.width_mask;
    a.early_term = dec->params.early_term;
    a.precheck = dec->params.precheck;
    a.hard = hard;
    a.hard_words = (dec->code.n + 31) / 32;
    a.iters = iters;
    a.syn_ok = syndrome_ok;
    a.post = post;
    return launch_decode_frame(a, dec->edges, edge_ram, keep_edges != 0, stream);
}

int fpldpc_decode_frame_host(fpldpc_decoder_t dec, const int32_t *llr, int32_t keep_edges, int32_t *edge_ram,
                             uint32_t *hard, int32_t *iters, uint8_t *syndrome_ok, int32_t *post) {
    if (!dec) return fail(FPLDPC_ERR_ARG, "null decoder");
    if (!llr || !edge_ram) return fail(FPLDPC_ERR_ARG, "null llr or edge RAM");
    DeviceGuard g(dec->device);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    const size_t n = dec->code.n, hw = (n + 31) / 32, ew = (size_t)dec->code.dc_max * dec->code.m;
    // One staging block, the same layout in pinned host memory and on the device: llr [n], edge RAM
    // [ew], post [n], hard [hw], iters, syndrome flag.  The reference's callers decode one frame per
    // call (PerfTest.cpp:121-128), so a call is one host-to-device copy of the inputs, the kernel and
    // one copy back of the outputs (3 submissions), not one pageable copy per buffer.
    const size_t in_words = 2 * n + ew, words = in_words + hw + 2;
    if (!dec->d_edge_stage) HIP_TRY(hipMalloc(&dec->d_edge_stage, sizeof(int32_t) * words));
    if (!dec->h_edge_stage) HIP_TRY(hipHostMalloc((void **)&dec->h_edge_stage, sizeof(int32_t) * words, hipHostMallocDefault));
    int32_t *h = dec->h_edge_stage;
    memcpy(h, llr, n * 4);
    memcpy(h + n, edge_ram, ew * 4);  // kept as is by a pre-check pass
    if (post) memcpy(h + n + ew, post, n * 4);  // likewise (:443-450)
    int32_t *d_llr = dec->d_edge_stage, *d_edge = d_llr + n, *d_post = d_edge + ew;
    uint32_t *d_hard = reinterpret_cast<uint32_t *>(d_post + n);
    int32_t *d_it = reinterpret_cast<int32_t *>(d_hard + hw);
    uint8_t *d_ok = reinterpret_cast<uint8_t *>(d_it + 1);
    hipStream_t s = dec->stream;
    HIP_TRY(hipMemcpyAsync(d_llr, h, (post ? in_words : n + ew) * 4, hipMemcpyHostToDevice, s));
    int st = fpldpc_decode_frame(dec, d_llr, FPLDPC_LLR_I32, keep_edges, d_edge, d_hard, d_it, d_ok,
                                 post ? d_post : nullptr, s);
    if (st) return st;
    HIP_TRY(hipMemcpyAsync(h + n, d_edge, (words - n) * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    memcpy(edge_ram, h + n, ew * 4);
    if (post) memcpy(post, h + n + ew, n * 4);
    if (hard) memcpy(hard, h + in_words, hw * 4);
    if (iters) memcpy(iters, h + in_words + hw, 4);
    if (syndrome_ok) *syndrome_ok = *reinterpret_cast<const uint8_t *>(h + in_words + hw + 1);
    return FPLDPC_OK;
}

}  // extern "C"
