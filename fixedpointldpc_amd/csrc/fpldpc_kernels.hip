// fpldpc_kernels.hip -- gfx950 (CDNA4) flooding decoder for the reference's fixed-point LDPC path.
//
// Reference semantics (tyc85/FixedPointLDPC): FP_Decoder::decode_general_fp
// (ArrayLDPC_Decoder.cpp:18-171) with the box-plus FP_Decoder::sxor (:677-694), the syndrome
// test checkPost_fp_general (:296-333), and decode_fixpoint's channel pre-check (:443-450).
//
// Design (DESIGN.md "Kernels"):
//   * One workgroup decodes one frame at a time and pulls the next frame from a device work
//     counter (persistent grid, per-frame early termination, no frozen lanes).
//   * One lane per check node.  The check's c2v messages live in VGPRs across iterations (or in a
//     per-workgroup global scratch for codes too large for registers); the posterior vector lives
//     in LDS.  The reference's variable-node phase (:121-156) is folded into the check pass:
//     v2c = post - c2v (:143-152), and the next posterior post' = LLR + sum(c2v') is accumulated
//     with LDS integer atomics (order-free, exact).  Three rotating posterior buffers give one
//     barrier per iteration.
//   * The check update keeps the reference's SERIAL forward/backward fold (:83-116): box-plus is
//     not associative, so no tree/shuffle reduction is used for it.
//   * The syndrome of iteration t is computed while gathering the posteriors of iteration t+1
//     (hard = post > 0 ? 0 : 1, :305-308); the pre-check is the same test on the channel LLRs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>

#include "fpldpc_internal.hpp"


namespace fpldpc {
namespace {

constexpr int kNT = 256;  // threads per workgroup (4 waves)
// per-workgroup control words after the posterior buffers in LDS (flood_pk's misc[])
constexpr int kTotW = 16;  // flood_pk: the workgroup's 4 totals counters misc[kTotW..+3]
constexpr int kMiscInts = kTotW + 4;

struct KArgs {
    const void *llr;
    int llr_i16;
    int n, m, m_pad, batch, max_iter, C, mask, early_term, precheck;
    const uint16_t *vidx;
    const uint8_t *cdeg;
    uint32_t *hard;
    int hard_words;
    int32_t *iters;
    uint8_t *syn_ok;
    int32_t *post;
    int32_t *bit_errors;
    unsigned long long *totals;
    const int32_t *info_idx;
    const uint8_t *info_bits;
    int k_info;
    const uint32_t *info_mask;  // [2][hard_words] packed: info positions, reference bits (distinct indices) or null
    int *work_counter;
    int32_t *c2v_scratch;
    uint32_t bfe_w;  // width_mask = 2^(bfe_w + 2) - 1 (contiguous-mask kernels only)
    // frame-list mode (fallback pass): work item i decodes frame frame_list[i], i < *frame_count
    const int *frame_list;
    const int *frame_count;
    // packed kernels: frames whose int16 range check failed are appended here for the int32 pass
    int *fb_list;
    int *fb_count;
    uint32_t cmax;  // largest c2v magnitude for which int16 posteriors / v2c cannot overflow
    unsigned long long *probe;  // diagnostic (FPLDPC_CLOCK_PROBE): workgroup 0's s_memtime/s_memrealtime
    unsigned long long *wgtrace;  // diagnostic (FPLDPC_WG_TRACE): per workgroup {xcc<<32 | hw_id, start, end, frames, stamps[4]}
    int *counters;       // the decoder's counter block (fpldpc_internal.hpp kCounterInts)
    int last_in_chain;   // 1: this launch is the call's last kernel and resets the counter block
    int split_tail;      // packed array kernels: a lone frame continues in the split form (flood_pk)
};

__device__ __forceinline__ void clock_probe(const KArgs &a, int slot) {
    if (a.probe && blockIdx.x == 0 && threadIdx.x == 0) {
        a.probe[slot] = __builtin_amdgcn_s_memtime();
        a.probe[slot + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// Next frame for this workgroup (thread 0 only): the work counter indexes the batch, or the
// fallback list in frame-list mode.  Returns -1 when the work is exhausted.
// Every workgroup calls this as it exits (all threads, uniform).  The last workgroup out of the
// call's LAST kernel resets the decoder's counter block for the next call: every workgroup of this
// kernel has made its last counter access before counting itself out, and the chain's earlier
// kernels have completed (stream order).  So no hipMemsetAsync precedes a decode call; the block
// is zeroed once at decoder creation.  The fallback-list sizes are kept for
// fpldpc_decoder_fallback_counts.
// (No fences: every counter access a workgroup makes before counting itself out is a returning
// atomic or a load whose value it has used, so it has been performed; the next call's kernels see
// the reset at the kernel boundary.)
__device__ __forceinline__ void chain_reset(int *c) {
    c[kCountFb0Last] = __hip_atomic_load(&c[kCountFb0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    c[kCountFb1Last] = __hip_atomic_load(&c[kCountFb1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = 0; i <= kCountExit; ++i) c[i] = 0;
}
__device__ __forceinline__ void chain_exit(const KArgs &a) {
    if (!a.last_in_chain || threadIdx.x != 0) return;
    if (atomicAdd(&a.counters[kCountExit], 1) == (int)gridDim.x - 1) chain_reset(a.counters);
}
// A fallback kernel whose frame list came out empty (the common case) leaves at once, uncounted:
// no workgroup of it touches a counter, and the list size it reads is already 0, so workgroup 0
// alone can reset the block (the last kernel of the chain) without waiting for the others --
// counting 256 workgroups out through one atomic cost ~7 us per call.
__device__ __forceinline__ bool empty_list(const KArgs &a) {
    if (!a.frame_list || *a.frame_count != 0) return false;
    if (a.last_in_chain && blockIdx.x == 0 && threadIdx.x == 0) chain_reset(a.counters);
    return true;
}

__device__ __forceinline__ int pull_frame(const KArgs &a, int *counter) {
    const int wi = atomicAdd(counter, 1);
    if (a.frame_list) return wi < *a.frame_count ? a.frame_list[wi] : -1;
    return wi < a.batch ? wi : -1;
}

// x [+] y = sgn(x) sgn(y) (min(|x|,|y|) + max(0, C - ((|x|+|y|) & mask) >> 2)
//                                      - max(0, C - (||x|-|y|| & mask) >> 2)),  sgn(0) = -1.
// ArrayLDPC_Decoder.cpp:677-694, ArrayLDPCMacro.h:222-224.  The magnitude term r is never
// negative (tests/test_oracle.py::test_sign_split: exhaustively wherever min(|x|,|y|) < C, for
// every mask 2^w - 1, w = 2..16, FRAC 3/4/6), so the sign of the result is + iff
// (x > 0) == (y > 0), and r == 0 gives 0 either way.
__device__ __forceinline__ int boxplus(int x, int y, int C, int mask) {
    const int a = x < 0 ? -x : x;
    const int b = y < 0 ? -y : y;
    const int s = ((a + b) & mask) >> 2;
    const int d = ((a > b ? a - b : b - a) & mask) >> 2;
    const int p1 = max(C - s, 0);
    const int p2 = max(C - d, 0);
    const int r = min(a, b) + p1 - p2;
    return ((x > 0) == (y > 0)) ? r : -r;
}

__device__ __forceinline__ void lds_add(int *p, int v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int DC>
__device__ __forceinline__ int slot_var(const uint32_t (&vpk)[(DC + 1) / 2], int k) {
    return (k & 1) ? (int)(vpk[k >> 1] >> 16) : (int)(vpk[k >> 1] & 0xffffu);
}

// One check: gather posteriors, syndrome parity, serial forward/backward fold, scatter-add.
// c2v: in = previous c2v (0 before the first iteration), out = new c2v.  Returns the parity of
// the hard decisions of pc over the check (1 = unsatisfied).
template <int DC, bool REGULAR>
__device__ __forceinline__ int check_update(int (&c2v)[DC], const uint32_t (&vpk)[(DC + 1) / 2], int deg,
                                            const int *pc, int *pn, bool update, int C, int mask) {
    int m[DC];
    int par = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const int p = pc[slot_var<DC>(vpk, k)];
        if (REGULAR || k < deg) par ^= (p <= 0) ? 1 : 0;
        m[k] = p - c2v[k];  // v2c = post - c2v (ArrayLDPC_Decoder.cpp:143-152)
    }
    if (!update) return par;
    // Backward[k] = Backward[k+1] [+] m[k], Backward[deg-1] = m[deg-1]   (:84-89)
    int B[DC];
    B[DC - 1] = m[DC - 1];
#pragma unroll
    for (int k = DC - 2; k >= 1; --k) {
        const int bk = boxplus(B[k + 1], m[k], C, mask);
        B[k] = (REGULAR || k < deg - 1) ? bk : m[k];
    }
    // Forward[k] = Forward[k-1] [+] m[k]; out[0] = B[1], out[k] = F[k-1] [+] B[k+1],
    // out[deg-1] = F[deg-2]   (:83-116)
    int F = m[0];
    c2v[0] = B[1];
#pragma unroll
    for (int k = 1; k <= DC - 2; ++k) {
        const int o = boxplus(F, B[k + 1], C, mask);
        c2v[k] = (REGULAR || k < deg - 1) ? o : F;
        F = boxplus(F, m[k], C, mask);
    }
    c2v[DC - 1] = F;
    // post' = LLR + sum c2v' (:131-144), accumulated order-free in LDS.
#pragma unroll
    for (int k = 0; k < DC; ++k)
        if (REGULAR || k < deg) lds_add(pn + slot_var<DC>(vpk, k), c2v[k]);
    return par;
}

__device__ __forceinline__ int load_llr(const KArgs &a, size_t i) {
    return a.llr_i16 ? (int)static_cast<const int16_t *>(a.llr)[i] : static_cast<const int32_t *>(a.llr)[i];
}

// Frame prologue: LLR -> LDS (int32) and the first two posterior buffers.
template <int NT = kNT>
__device__ __forceinline__ void frame_load(const KArgs &a, int cw, int *bufs, int *llr_s) {
    const int n = a.n;
    const size_t base = (size_t)cw * n;
    for (int v = threadIdx.x; v < n; v += NT) {
        const int x = load_llr(a, base + v);
        llr_s[v] = x;
        bufs[v] = x;
        bufs[n + v] = x;
    }
}

// Frame epilogue: posteriors, packed hard decisions, per-frame BER and totals.
template <int NT = kNT>
__device__ __forceinline__ void frame_store(const KArgs &a, int cw, const int *pf, bool write_post, int iters,
                                            int ok, int *misc) {
    const int n = a.n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (a.post && write_post)
        for (int v = tid; v < n; v += NT) a.post[(size_t)cw * n + v] = pf[v];
    if (a.hard) {
        uint32_t *h = a.hard + (size_t)cw * a.hard_words;
        for (int base = wave * 64; base < n; base += NT) {
            const int v = base + lane;
            const unsigned long long b = __ballot(v < n && pf[v] <= 0);
            if (lane == 0) {
                const int w = base >> 5;
                h[w] = (uint32_t)b;
                if (w + 1 < a.hard_words) h[w + 1] = (uint32_t)(b >> 32);
            }
        }
    }
    int errors = 0;
    if (a.k_info > 0) {
        int e = 0;
        for (int i = tid; i < a.k_info; i += NT) e += ((pf[a.info_idx[i]] <= 0) ? 1 : 0) != a.info_bits[i];
        if (e) atomicAdd(&misc[1], e);
        __syncthreads();
        errors = misc[1];
    }
    if (tid == 0) {
        if (a.iters) a.iters[cw] = iters;
        if (a.syn_ok) a.syn_ok[cw] = (uint8_t)ok;
        if (a.bit_errors) a.bit_errors[cw] = errors;
        if (a.totals) {
            atomicAdd(&a.totals[0], (unsigned long long)errors);
            atomicAdd(&a.totals[1], (unsigned long long)(errors > 0));
            atomicAdd(&a.totals[2], 1ull);
            atomicAdd(&a.totals[3], (unsigned long long)iters);
        }
    }
}

// Register-resident variant: CPL checks per lane (check c = tid + q*kNT), c2v and the packed
// var indices of each check held in VGPRs for the lifetime of the workgroup.
template <int DC, int CPL, bool REGULAR>
__global__ void __launch_bounds__(kNT) flood_reg(KArgs a) {
    if (empty_list(a)) return;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    const int n = a.n;
    int *const bufs = smem;          // 3 x n posterior buffers
    int *const llr_s = smem + 3 * n; // n
    int *const misc = smem + 4 * n;  // [0] frame slot, [1] bit-error accumulator
    const int tid = threadIdx.x;

    constexpr int DP = (DC + 1) / 2;
    uint32_t vpk[CPL][DP];
    int deg[CPL];
    bool act[CPL];
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
        const int c = tid + q * kNT;
        act[q] = c < a.m;
        deg[q] = act[q] ? (REGULAR ? DC : (int)a.cdeg[c]) : 0;
#pragma unroll
        for (int j = 0; j < DP; ++j) {
            uint32_t lo = 0, hi = 0;
            if (act[q]) {
                lo = a.vidx[(size_t)(2 * j) * a.m_pad + c];
                if (2 * j + 1 < DC) hi = a.vidx[(size_t)(2 * j + 1) * a.m_pad + c];
            }
            vpk[q][j] = lo | (hi << 16);
        }
    }

    for (;;) {
        __syncthreads();
        if (tid == 0) {
            misc[0] = pull_frame(a, a.work_counter);
            misc[1] = 0;
        }
        __syncthreads();
        const int cw = misc[0];
        if (cw < 0) break;
        frame_load(a, cw, bufs, llr_s);
        int c2v[CPL][DC];
#pragma unroll
        for (int q = 0; q < CPL; ++q)
#pragma unroll
            for (int k = 0; k < DC; ++k) c2v[q][k] = 0;
        __syncthreads();

        int cur = 0;
        const int *pf = nullptr;
        bool pre = false;
        int iters = 0, ok = 0;
        for (int it = 1;; ++it) {
            const bool update = it <= a.max_iter;
            const int *pc = bufs + cur * n;
            int *pn = bufs + ((cur + 1) % 3) * n;
            int *pr = bufs + ((cur + 2) % 3) * n;
            if (update)
                for (int v = tid; v < n; v += kNT) pr[v] = llr_s[v];
            int fail = 0;
#pragma unroll
            for (int q = 0; q < CPL; ++q)
                if (act[q]) fail |= check_update<DC, REGULAR>(c2v[q], vpk[q], deg[q], pc, pn, update, a.C, a.mask);
            fail = __syncthreads_or(fail);
            const int done = it - 1;
            if (done == 0 && a.precheck && !fail) {
                pf = llr_s;
                pre = true;
                iters = 0;
                ok = 1;
                break;
            }
            if ((done >= 1 && a.early_term && !fail) || done >= a.max_iter) {
                pf = pc;
                iters = done;
                ok = !fail;
                break;
            }
            cur = (cur + 1) % 3;
        }
        frame_store(a, cw, pf, !pre, iters, ok, misc);
    }
    chain_exit(a);
}

// Global-scratch variant for codes whose c2v state does not fit the register budget: checks
// strided over the lanes, c2v in a per-workgroup scratch [DC][m_pad] (coalesced per slot), var
// indices read from the [DC][m_pad] table (L1/L2 resident).
template <int DC>
__device__ __forceinline__ int check_update_gmem(int c, int deg, int m_pad, const uint16_t *vidx, int32_t *c2vs,
                                                 bool first, const int *pc, int *pn, bool update, int C, int mask) {
    int m[DC];
    int vi[DC];
    int par = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        vi[k] = vidx[(size_t)k * m_pad + c];
        const int p = pc[vi[k]];
        if (k < deg) par ^= (p <= 0) ? 1 : 0;
        m[k] = first ? p : p - c2vs[(size_t)k * m_pad + c];
    }
    if (!update) return par;
    int B[DC];
    B[DC - 1] = m[DC - 1];
#pragma unroll
    for (int k = DC - 2; k >= 1; --k) {
        const int bk = boxplus(B[k + 1], m[k], C, mask);
        B[k] = (k < deg - 1) ? bk : m[k];
    }
    int F = m[0];
    int out[DC];
    out[0] = B[1];
#pragma unroll
    for (int k = 1; k <= DC - 2; ++k) {
        const int o = boxplus(F, B[k + 1], C, mask);
        out[k] = (k < deg - 1) ? o : F;
        F = boxplus(F, m[k], C, mask);
    }
    out[DC - 1] = F;
#pragma unroll
    for (int k = 0; k < DC; ++k)
        if (k < deg) {
            c2vs[(size_t)k * m_pad + c] = out[k];
            lds_add(pn + vi[k], out[k]);
        }
    return par;
}

template <int DC>
__global__ void __launch_bounds__(kNT) flood_gmem(KArgs a) {
    if (empty_list(a)) return;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    const int n = a.n;
    int *const bufs = smem;
    int *const llr_s = smem + 3 * n;
    int *const misc = smem + 4 * n;
    const int tid = threadIdx.x;
    int32_t *const c2vs = a.c2v_scratch + (size_t)blockIdx.x * DC * a.m_pad;

    for (;;) {
        __syncthreads();
        if (tid == 0) {
            misc[0] = pull_frame(a, a.work_counter);
            misc[1] = 0;
        }
        __syncthreads();
        const int cw = misc[0];
        if (cw < 0) break;
        frame_load(a, cw, bufs, llr_s);
        __syncthreads();

        int cur = 0;
        const int *pf = nullptr;
        bool pre = false;
        int iters = 0, ok = 0;
        for (int it = 1;; ++it) {
            const bool update = it <= a.max_iter;
            const int *pc = bufs + cur * n;
            int *pn = bufs + ((cur + 1) % 3) * n;
            int *pr = bufs + ((cur + 2) % 3) * n;
            if (update)
                for (int v = tid; v < n; v += kNT) pr[v] = llr_s[v];
            int fail = 0;
            for (int c = tid; c < a.m; c += kNT)
                fail |= check_update_gmem<DC>(c, a.cdeg[c], a.m_pad, a.vidx, c2vs, it == 1, pc, pn, update, a.C, a.mask);
            fail = __syncthreads_or(fail);
            const int done = it - 1;
            if (done == 0 && a.precheck && !fail) {
                pf = llr_s;
                pre = true;
                iters = 0;
                ok = 1;
                break;
            }
            if ((done >= 1 && a.early_term && !fail) || done >= a.max_iter) {
                pf = pc;
                iters = done;
                ok = !fail;
                break;
            }
            cur = (cur + 1) % 3;
        }
        frame_store(a, cw, pf, !pre, iters, ok, misc);
    }
    chain_exit(a);
}

// ------------------------------------------------------------------------------------------
// Stateful single-frame decode: the reference's edge RAM kept across calls.  Between calls
// FP_Decoder's EdgeRAM (ArrayLDPCMacro.h:162) holds the v2c message of every edge as the last
// variable-node phase wrote it (accum - c2v, ArrayLDPC_Decoder.cpp:152, :615).  decode_general_fp,
// and decode_fixpoint in state PCV, first overwrite it with the channel values (:45-61, :462-485);
// decode_fixpoint in state C2V skips that and iterates from what the previous frame left (:488-618),
// the new LLRs entering in the variable-node phase.  `edge` is that RAM, edge[k * m + c] = slot k of
// check c (clist order, the code's own check order), owned by the caller; the first update reads its
// v2c from it (keep = 1) or from the LLRs (keep = 0), later updates from post - c2v.  The c2v of the
// last two updates sit in a global double buffer, so the RAM written back at the end is the one that
// belongs to the returned posteriors: pf[var] - c2v of update `done`.  The pre-check (:443-450) runs
// before anything touches the RAM and leaves it as it was.  One workgroup, one frame: this is the
// per-frame drop-in path (include/fpldpc_compat.hpp), not the batch kernels.
struct EdgeArgs {
    const uint16_t *vidx;  // [DC][m] var of slot k of check c (clist order)
    const uint8_t *cdeg;   // [m]
    int32_t *edge;         // [dc_max][m] edge RAM (v2c), in/out
    int32_t *c2v;          // [2][DC][m] scratch
    int keep;              // 1: iterate from `edge` (state C2V); 0: edge init from the channel values
    int dc_max;            // rows of vidx / edge (the code's largest check degree)
};

// LDS = true (when it fits, edge_lds_bytes): the c2v double buffer and the index table live in LDS
// after the posteriors instead of global memory -- A and W (R's 1128 x 47 edges do not fit).
template <int DC, bool LDS>
__global__ void __launch_bounds__(kNT) flood_edges(KArgs a, EdgeArgs e) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    const int n = a.n, m = a.m;
    int *const bufs = smem;
    int *const llr_s = smem + 3 * n;
    int *const misc = smem + 4 * n;
    const int tid = threadIdx.x;
    int32_t *const c2v = LDS ? smem + 4 * n + kMiscInts : e.c2v;
    const uint16_t *vidx = e.vidx;
    if constexpr (LDS) {
        uint16_t *const lv = reinterpret_cast<uint16_t *>(smem + 4 * n + kMiscInts + 2 * DC * m);
        for (int i = tid; i < e.dc_max * m; i += kNT) lv[i] = e.vidx[i];
        vidx = lv;
    }
    for (int v = tid; v < n; v += kNT) {
        const int x = load_llr(a, v);
        llr_s[v] = x;
        bufs[n + v] = x;  // posteriors of update 1: LLR + sum c2v
    }
    if (tid == 0) misc[1] = 0;
    __syncthreads();
    if (a.precheck) {  // hardDecision(LLR) (:270-294): a passing channel syndrome returns 0
        int fail = 0;
        for (int c = tid; c < m; c += kNT) {
            int par = 0;
            for (int k = 0; k < e.cdeg[c]; ++k) par ^= llr_s[vidx[(size_t)k * m + c]] <= 0;
            fail |= par;
        }
        if (!__syncthreads_or(fail)) {
            frame_store(a, 0, llr_s, false, 0, 1, misc);
            return;
        }
    }
    int cur = 0, iters = 0, ok = 0;
    const int *pf = nullptr;
    for (int it = 1;; ++it) {
        const bool update = it <= a.max_iter;
        const int *pc = bufs + cur * n;
        int *pn = bufs + ((cur + 1) % 3) * n;
        int *pr = bufs + ((cur + 2) % 3) * n;
        if (update)
            for (int v = tid; v < n; v += kNT) pr[v] = llr_s[v];
        const int32_t *c2r = c2v + (size_t)((it - 1) & 1) * DC * m;  // c2v of update it - 1
        int32_t *c2w = c2v + (size_t)(it & 1) * DC * m;               // c2v of update it
        int fail = 0;
        for (int c = tid; c < m; c += kNT) {
            const int deg = e.cdeg[c];
            int mv[DC], vi[DC];
            int par = 0;
#pragma unroll
            for (int k = 0; k < DC; ++k) {
                vi[k] = 0;
                mv[k] = 0;
                if (k < deg) {
                    vi[k] = vidx[(size_t)k * m + c];
                    const int p = pc[vi[k]];
                    par ^= p <= 0;
                    mv[k] = it > 1 ? p - c2r[(size_t)k * m + c] : e.keep ? e.edge[(size_t)k * m + c] : llr_s[vi[k]];
                }
            }
            if (it > 1) fail |= par;  // syndrome of the posteriors after it - 1 updates (:164, :621)
            if (!update) continue;
            // forward / backward fold (:83-116), the reference's order
            int B[DC];
            B[DC - 1] = mv[DC - 1];
#pragma unroll
            for (int k = DC - 2; k >= 1; --k) B[k] = k < deg - 1 ? boxplus(B[k + 1], mv[k], a.C, a.mask) : mv[k];
            int F = mv[0];
#pragma unroll
            for (int k = 0; k < DC; ++k) {
                if (k >= deg) continue;
                const int o = k == 0 ? B[1] : k == deg - 1 ? F : boxplus(F, B[k + 1], a.C, a.mask);
                if (k > 0) F = boxplus(F, mv[k], a.C, a.mask);
                c2w[(size_t)k * m + c] = o;
                lds_add(pn + vi[k], o);  // post' = LLR + sum c2v' (:131-144)
            }
        }
        fail = __syncthreads_or(fail);
        const int done = it - 1;
        if ((done >= 1 && a.early_term && !fail) || done >= a.max_iter) {
            pf = pc;
            iters = done;
            ok = !fail;
            break;
        }
        cur = (cur + 1) % 3;
    }
    // the edge RAM after the last variable-node phase: v2c = post - c2v of update `done`
    const int32_t *c2d = c2v + (size_t)(iters & 1) * DC * m;
    for (int c = tid; c < m; c += kNT)
        for (int k = 0; k < e.cdeg[c]; ++k)
            e.edge[(size_t)k * m + c] = pf[vidx[(size_t)k * m + c]] - c2d[(size_t)k * m + c];
    frame_store(a, 0, pf, true, iters, ok, misc);
}

// ------------------------------------------------------------------------------------------
// Sign/magnitude kernels.  Box-plus splits exactly into a magnitude chain and a sign parity:
//   |x [+] y| = bp_mag(|x|, |y|), sign = XOR of the (v <= 0) flags,
// because a zero magnitude absorbs (bp_mag(0, b) = 0, so the sgn(0) = -1 rule of
// ArrayLDPCMacro.h:222-224 can only ever multiply a zero).  The serial fold ORDER of the
// magnitudes is kept exactly as the reference's (ArrayLDPC_Decoder.cpp:83-116); only the sign
// bookkeeping leaves the chain: one parity S per check, c2v_k sign = S ^ neg(m_k).
// tests/test_oracle.py::test_sign_split checks this against the reference's sxor fold: pairs
// exhaustively on [-1024, 1024]^2, whole checks of degree 47 and 8 on random v2c, bp_mag2's packed
// arithmetic per half, for every mask 2^w - 1 (w = 2..16) the packed kernels accept.
__device__ __forceinline__ uint32_t bp_mag(uint32_t a, uint32_t b, uint32_t C, uint32_t w) {
    const uint32_t mn = min(a, b);
    const uint32_t mx = max(a, b);
    const uint32_t t1 = __builtin_amdgcn_ubfe(a + b, 2, w);   // ((a+b) & mask) >> 2
    const uint32_t t2 = __builtin_amdgcn_ubfe(mx - mn, 2, w);  // (|a-b| & mask) >> 2
    // min + max(0, C - t1) - max(0, C - t2) = min + min(C, t2) - min(C, t1)
    return mn + min(C, t2) - min(C, t1);
}

__device__ __forceinline__ uint32_t iabs(int x) { return (uint32_t)(x < 0 ? -x : x); }

// Array codes (ROM::CirShift = (i*k) mod p, ArrayLDPCMacro.h:57; H_array_p*_forward.txt): check
// (i, j) = i*P + j connects var k*P + (j + i*k) mod P, k = 0..P-1, so the gather address is
// computed (one add + one min per edge, the k*P part folds into the LDS instruction offset) and no
// index table is read.  One lane per check (m = r*P <= 256), c2v state in VGPRs.
template <int P>
__global__ void __launch_bounds__(kNT, 4) flood_array(KArgs a) {
    if (empty_list(a)) return;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    const int n = a.n;
    int *const bufs = smem;
    int *const llr_s = smem + 3 * n;
    int *const misc = smem + 4 * n;
    const int tid = threadIdx.x;
    const bool act = tid < a.m;
    const uint32_t row = act ? (uint32_t)(tid / P) : 0u, col = act ? (uint32_t)(tid % P) : 0u;
    const uint32_t C = (uint32_t)a.C, w = a.bfe_w;

    for (;;) {
        __syncthreads();
        if (tid == 0) {
            misc[0] = pull_frame(a, a.work_counter);
            misc[1] = 0;
        }
        __syncthreads();
        const int cw = misc[0];
        if (cw < 0) break;
        frame_load(a, cw, bufs, llr_s);
        int st[P];  // c2v between iterations; v2c (m) inside the update
#pragma unroll
        for (int k = 0; k < P; ++k) st[k] = 0;
        __syncthreads();

        int cur = 0;
        const int *pf = nullptr;
        bool pre = false;
        int iters = 0, ok = 0;
        for (int it = 1;; ++it) {
            const bool update = it <= a.max_iter;
            const int *pc = bufs + cur * n;
            int *pn = bufs + ((cur + 1) % 3) * n;
            int *pr = bufs + ((cur + 2) % 3) * n;
            if (update)
                for (int v = tid; v < n; v += kNT) pr[v] = llr_s[v];
            int fail = 0;
            if (act) {
                // gather posteriors; v2c = post - c2v (ArrayLDPC_Decoder.cpp:143-152); syndrome
                // parity of the hard decisions post > 0 ? 0 : 1 (:305-308); sign parity S
                // (opaque start: the compiler would otherwise hoist all P loop-invariant
                // addresses out of the iteration loop and keep them in registers)
                uint32_t t = col;
                asm volatile("" : "+v"(t));
                bool par = false, S = false;
#pragma unroll
                for (int k = 0; k < P; ++k) {
                    const int p = pc[k * P + t];
                    par ^= p <= 0;
                    st[k] = p - st[k];
                    S ^= st[k] <= 0;
                    t += row;
                    t = min(t, t - (uint32_t)P);
                }
                fail = par;
                if (update) {
                    // backward magnitudes B[k] = B[k+1] [+] m[k] (:84-89)
                    uint32_t B[P];
                    B[P - 1] = iabs(st[P - 1]);
#pragma unroll
                    for (int k = P - 2; k >= 1; --k) B[k] = bp_mag(B[k + 1], iabs(st[k]), C, w);
                    // Recompute |m| and neg(m) below instead of keeping 2 x 47 values live across
                    // the passes (the opaque moves stop the compiler from CSE-ing them).
#pragma unroll
                    for (int k = 0; k < P; ++k) asm volatile("" : "+v"(st[k]));
                    // forward pass fused with the extrinsic outputs (:83-116)
                    uint32_t F = iabs(st[0]);
                    st[0] = (S ^ (st[0] <= 0)) ? -(int)B[1] : (int)B[1];
#pragma unroll
                    for (int k = 1; k <= P - 2; ++k) {
                        const bool nk = st[k] <= 0;
                        const uint32_t ak = iabs(st[k]);
                        const uint32_t o = bp_mag(F, B[k + 1], C, w);
                        st[k] = (S ^ nk) ? -(int)o : (int)o;
                        F = bp_mag(F, ak, C, w);
                    }
                    st[P - 1] = (S ^ (st[P - 1] <= 0)) ? -(int)F : (int)F;
                    // post' = LLR + sum c2v' (:131-144), order-free integer adds in LDS
                    t = col;
                    asm volatile("" : "+v"(t));
#pragma unroll
                    for (int k = 0; k < P; ++k) {
                        lds_add(pn + k * P + t, st[k]);
                        t += row;
                        t = min(t, t - (uint32_t)P);
                    }
                } else {
                    // restore the c2v state (unused after the final syndrome, kept for clarity)
                }
            }
            fail = __syncthreads_or(fail);
            const int done = it - 1;
            if (done == 0 && a.precheck && !fail) {
                pf = llr_s;
                pre = true;
                iters = 0;
                ok = 1;
                break;
            }
            if ((done >= 1 && a.early_term && !fail) || done >= a.max_iter) {
                pf = pc;
                iters = done;
                ok = !fail;
                break;
            }
            cur = (cur + 1) % 3;
        }
        frame_store(a, cw, pf, !pre, iters, ok, misc);
    }
    chain_exit(a);
}

// ------------------------------------------------------------------------------------------
// Packed kernel: two frames per lane, one in each 16-bit half (v_pk_* ops), so every VALU op,
// LDS access and address computation serves two frames.  Exact while every value fits int16:
// with |LLR| <= kLlrMax and every c2v magnitude <= a.cmax = (32767 - kLlrMax) / (dv_max + 1),
// |post| and |v2c| stay below 32768 and the u16 magnitude chain (a + b <= 65534) never wraps.
// A frame that leaves that range (or overlaps in time with a partner that does) is not written:
// it is appended to a.fb_list and decoded again by flood_array<P> (int32) in a second pass, so
// outputs are bit-exact for every input.
//
// Posteriors live in LDS as *biased* pairs V = (lo + 0x7fff) | (hi + 0x7fff) << 16: c2v
// messages are added in carry form (lo + 65536*hi, a plain int32), so the next posterior is still
// accumulated with one ds_add_u32 per edge, and since LLR + bias + sum(c2v) is exact modulo 2^32
// the final word has both biased halves in place while |post| <= 32767, whatever the order of the
// adds.  Bits 15 / 31 are then (post >= 1) = NOT hard (:305-308), and v2c = V - c2v is again a
// biased pair (one subtraction).  The two halves run independent frames: when one finishes (own
// iteration count, early termination, pre-check) its outputs are written and the half is refilled
// with the next frame at the next step while the other half carries on.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
constexpr int kLlrMax = 8000;

__device__ __forceinline__ u16x2 U2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ i16x2 I2(uint32_t x) { return __builtin_bit_cast(i16x2, x); }
__device__ __forceinline__ uint32_t W(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t W(i16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// low half of a carry-form word lo + 65536*hi (the c2v state): the high half is (v - lo) >> 16
__device__ __forceinline__ int carry_lo(uint32_t v) { return (int)(short)(v & 0xffffu); }

// bp_mag on both halves: min(a,b) + min(C, ((|a-b| & M) >> 2)) - min(C, ((a+b) & M) >> 2).
// The halves are magnitudes below 2^15, so a + b and max - min never cross into the other half, a
// 32-bit right shift only pollutes bits 14-15 of the low half (cleared by M2, at most 14 bits per
// half), and mn + q2 - q1 >= 0 per half: full-rate 32-bit add/sub/shift/and give exact per-half
// results, and only the three min/max steps need the (half-rate) packed instructions.
// 2*x written as x + x: hipcc turns it into v_lshlrev_b32, which issues at half the rate of
// v_add_u32 on gfx950 (profiles/r1/ubench_valu_rate.txt)
__device__ __forceinline__ uint32_t sub2x(uint32_t a, uint32_t x) {  // a - 2x
    uint32_t r;
    asm("v_sub_u32 %0, %1, %2\n\tv_sub_u32 %0, %0, %2" : "=&v"(r) : "v"(a), "v"(x));
    return r;
}

// (The packed kernels hold C2 / M2 in VGPRs, see flood_pk: as SGPR operands, hipcc's choice for
// uniform values, the 270 v_and_b32 / v_pk_min_u16 per check-step that read them cost A 0.5-1.9 %
// and W 0.7 % (profiles/r2/ab/bp_form.txt); C = 10 / mask 0xff as immediates measured 4.6 % slower.)
// FORM 0 leaves the order to hipcc; FORM 1 is one asm block (no pk_min result read by the next
// instruction).  Measured per kernel (profiles/r5/ab/post_ra.txt): the asm block is +2.7 % on R and
// +1.3 % on W but -4 % on A, whatever its order (two other orders of the block were measured the
// same), so each check policy picks its own (kBp).  (Also measured and not kept: two independent
// box-pluses interleaved in one block with their six v_pk_min_u16 four instructions apart -- W and R
// unchanged, R's kernel spilling when its whole checks used it; W's output-range ORs kept out of
// v_or3_b32 -- W -2.7 %.)
constexpr int kBpArray1 = 0;  // A: compiler order
constexpr int kBpMany = 1;    // R (two checks per lane, split units) and W: the asm block
template <int FORM>
__device__ __forceinline__ uint32_t bp_mag2(uint32_t a, uint32_t b, u16x2 C2, uint32_t M2) {
    if constexpr (FORM == 0) {
        const uint32_t mn = W(__builtin_elementwise_min(U2(a), U2(b)));
        const uint32_t s = a + b;          // per half a + b < 2^16
        const uint32_t d = sub2x(s, mn);   // per half max - min = a + b - 2 min >= 0
        const uint32_t q1 = W(__builtin_elementwise_min(U2((s >> 2) & M2), C2));
        const uint32_t q2 = W(__builtin_elementwise_min(U2((d >> 2) & M2), C2));
        return mn + q2 - q1;
    } else {
        uint32_t mn, s, t;
        static_assert(FORM == 1, "bp_mag2: FORM 0 (compiler order) or 1 (one asm block)");
        asm("v_pk_min_u16 %0, %3, %4\n\tv_add_u32 %1, %3, %4\n\tv_lshrrev_b32 %2, 2, %1\n\t"
            "v_sub_u32 %1, %1, %0\n\tv_sub_u32 %1, %1, %0\n\tv_and_b32 %2, %2, %6\n\t"
            "v_lshrrev_b32 %1, 2, %1\n\tv_pk_min_u16 %2, %2, %5\n\tv_and_b32 %1, %1, %6\n\t"
            "v_pk_min_u16 %1, %1, %5\n\tv_sub_u32 %0, %0, %2\n\tv_add_u32 %0, %0, %1"
            : "=&v"(mn), "=&v"(s), "=&v"(t) : "v"(a), "v"(b), "v"(W(C2)), "v"(M2));
        return mn;
    }
}

// Biased pairs (posteriors, LLRs, v2c): half h holds x + 0x7fff, in [0, 0xfffe] for |x| <= 32767.
__device__ __forceinline__ int bias_half(uint32_t v, int h) { return (int)((v >> (16 * h)) & 0xffffu) - 0x7fff; }
__device__ __forceinline__ uint32_t bias_set(uint32_t v, int h, int x) {
    const uint32_t u = (uint32_t)(x + 0x7fff) & 0xffffu;
    return h ? (v & 0xffffu) | (u << 16) : (v & 0xffff0000u) | u;
}
// biased v2c pair u -> sign-magnitude halves (|x| in bits 0-14, x <= 0 in bit 15; the flag of a
// zero is irrelevant: a zero magnitude absorbs every chain through it, and output k's sign never
// uses flag k).  Per half: t = 0x8000 iff x >= 1, c = its bit-0 copy, w = t - c = 0x7fff iff
// x >= 1; ~(u ^ w) is then x - 1 (x >= 1) or 0x8000 | -x (x <= 0), and + c gives |x| without a
// carry out of the half, so the whole word is c - (u ^ w) - 1 in plain 32-bit arithmetic.  Six
// full-rate VOP2 ops: v_xnor_b32, though VOP2, issues at the slow rate in a mix
// (profiles/r1/ubench/mix_rate.txt), as hipcc's v_xad_u32 fusion would.
__device__ __forceinline__ uint32_t sign_mag_b(uint32_t u, uint32_t sgn = 0x80008000u) {
    const uint32_t t = u & sgn, c = t >> 15;
    uint32_t x = u ^ (t - c), r;
    asm("v_sub_u32 %0, %1, %2\n\tv_add_u32 %0, -1, %0" : "=&v"(r) : "v"(c), "v"(x));
    return r;
}
// sign_mag_b on 8 values with the final c - x - 1 as v_subb_co_u32 (c - x - VCC): VCC is set to all
// ones once and stays so, because c <= x in every lane and half combination (c = 1 in a half only
// when that half's x is >= 0x8000; c = 0 borrows from 0 - x - 1), so every subtraction borrows out
// again: 5 full-rate ops per value instead of 6.
template <int G>
__device__ __forceinline__ void sign_mag_b_x(uint32_t (&u)[G]) {
    static_assert(G == 8, "batch of 8");
    uint32_t t[8], c[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        t[g] = u[g] & 0x80008000u;
        c[g] = t[g] >> 15;
        u[g] ^= t[g] - c[g];
    }
    asm("s_mov_b64 vcc, -1\n\t"
        "v_subb_co_u32_e32 %0, vcc, %8, %0, vcc\n\t"
        "v_subb_co_u32_e32 %1, vcc, %9, %1, vcc\n\t"
        "v_subb_co_u32_e32 %2, vcc, %10, %2, vcc\n\t"
        "v_subb_co_u32_e32 %3, vcc, %11, %3, vcc\n\t"
        "v_subb_co_u32_e32 %4, vcc, %12, %4, vcc\n\t"
        "v_subb_co_u32_e32 %5, vcc, %13, %5, vcc\n\t"
        "v_subb_co_u32_e32 %6, vcc, %14, %6, vcc\n\t"
        "v_subb_co_u32_e32 %7, vcc, %15, %7, vcc"
        : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7])
        : "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6]), "v"(c[7])
        : "vcc");
}
// The same on G = 4, 6 or 7 values (the pipelined gather, the table policy), one asm block (split
// into blocks of two it measured 1 % slower: the block boundaries constrain the scheduler)
template <int G>
__device__ __forceinline__ void sign_mag_b_xg(uint32_t (&u)[G]) {
    static_assert(G == 4 || G == 6 || G == 7, "batch of 4, 6 or 7");
    uint32_t t[G], c[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        t[g] = u[g] & 0x80008000u;
        c[g] = t[g] >> 15;
        u[g] ^= t[g] - c[g];
    }
    if constexpr (G == 4)
        asm("s_mov_b64 vcc, -1\n\t"
            "v_subb_co_u32_e32 %0, vcc, %4, %0, vcc\n\t"
            "v_subb_co_u32_e32 %1, vcc, %5, %1, vcc\n\t"
            "v_subb_co_u32_e32 %2, vcc, %6, %2, vcc\n\t"
            "v_subb_co_u32_e32 %3, vcc, %7, %3, vcc"
            : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3])
            : "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3])
            : "vcc");
    else if constexpr (G == 7)
        asm("s_mov_b64 vcc, -1\n\t"
            "v_subb_co_u32_e32 %0, vcc, %7, %0, vcc\n\t"
            "v_subb_co_u32_e32 %1, vcc, %8, %1, vcc\n\t"
            "v_subb_co_u32_e32 %2, vcc, %9, %2, vcc\n\t"
            "v_subb_co_u32_e32 %3, vcc, %10, %3, vcc\n\t"
            "v_subb_co_u32_e32 %4, vcc, %11, %4, vcc\n\t"
            "v_subb_co_u32_e32 %5, vcc, %12, %5, vcc\n\t"
            "v_subb_co_u32_e32 %6, vcc, %13, %6, vcc"
            : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6])
            : "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6])
            : "vcc");
    else
        asm("s_mov_b64 vcc, -1\n\t"
            "v_subb_co_u32_e32 %0, vcc, %6, %0, vcc\n\t"
            "v_subb_co_u32_e32 %1, vcc, %7, %1, vcc\n\t"
            "v_subb_co_u32_e32 %2, vcc, %8, %2, vcc\n\t"
            "v_subb_co_u32_e32 %3, vcc, %9, %3, vcc\n\t"
            "v_subb_co_u32_e32 %4, vcc, %10, %4, vcc\n\t"
            "v_subb_co_u32_e32 %5, vcc, %11, %5, vcc"
            : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5])
            : "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5])
            : "vcc");
}
// LDS addressing of the packed kernels: buffers are addressed by their 32-bit LDS byte address
// (< 64 KiB within a workgroup's allocation); a slot's 16-bit byte offset, kept two per VGPR,
// plus the buffer's (wave-uniform) address costs one v_add_u16 for the low half (the result's
// high half is zeroed on gfx9) or a shift and an add for the high half, all full-rate VOP2.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) int lds_i32;
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(size_t)(const __attribute__((address_space(3))) void *)p;
}
// (base in a VGPR: a 16-bit VOP2 op with an SGPR operand issues at the slow rate)
// LDS byte address of a slot: base + the low (hi = 0) or high 16-bit offset of a packed pair.
// SDWA: one 32-bit add with a word select for either half, any LDS address -- the stored-offset
// policy (A) and the split checks (A +1.15 %; R's LDS-table policy -1.2 %, profiles/r3/ab/sdwa.txt).
// Otherwise a 16-bit add for the low half (LDS byte addresses below 64 KiB, as in flood_pk's
// one-frame-pair layouts) and shift + add for the high one.
template <bool SDWA>
__device__ __forceinline__ uint32_t lds_at(uint32_t offs2, int hi, uint32_t base) {
    uint32_t r;
    if constexpr (SDWA) {
    if (hi)
        asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
            : "=v"(r) : "v"(base), "v"(offs2));
    else
        asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
            : "=v"(r) : "v"(base), "v"(offs2));
    } else {
    if (hi)
        asm("v_lshrrev_b32 %0, 16, %1\n\tv_add_u32 %0, %2, %0" : "=&v"(r) : "v"(offs2), "v"(base));
    else
        asm("v_add_u16 %0, %1, %2" : "=v"(r) : "v"(base), "v"(offs2));
    }
    return r;
}
__device__ __forceinline__ void lds_add_at(uint32_t addr, int v) {
    __hip_atomic_fetch_add(reinterpret_cast<lds_i32 *>((size_t)addr), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Output k of a check: magnitude o, sign = parity of the other inputs' flags = (S ^ flag_k) in bits
// 15 / 31; st (the v2c in sign-magnitude) is overwritten with the carry-form c2v (o ^ neg) - neg.
template <bool ASM_OR = false>
__device__ __forceinline__ void emit_c2v(uint32_t &st, uint32_t o, uint32_t S, uint32_t &ovor) {
    if (ASM_OR)
        asm("v_or_b32 %0, %0, %1" : "+v"(ovor) : "v"(o));  // not fused into v_or3_b32 (VOP3)
    else
        ovor |= o;
    const uint32_t neg = W((i16x2)(I2(S ^ st) >> (i16x2)15));
    // per half neg ? -o : o, as one 32-bit word in carry form: (o ^ m) - m with m = 0xffff in a
    // negative half is (+-hi)*65536 + (+-lo) exactly (the low half's borrow is the carry form's)
    asm("v_xor_b32 %0, %1, %2\n\tv_sub_u32 %0, %0, %2" : "=&v"(st) : "v"(o), "v"(neg));
}

// Check side of the packed kernel, array codes: c2v state (carry form) in VGPRs; CPL checks per
// lane (c = tid + q*NT).  Slot k of check (row i, column j) reads variable k*P + (j + i*k) mod P.
// With one check per lane (A) the 16-bit byte offsets 4*((j + i*k) mod P) are computed once and
// kept two per VGPR (P/2 VGPRs), so a gather or scatter address costs one SDWA add with a word
// select (lds_at; round 2: v_add_u16 for the low half, shift + add for the high one); with several
// checks per lane (R: no VGPRs to spare) they come from an LDS table or are walked per step.
// With several checks per lane (R) the offsets do not fit VGPRs; LDS_OFFS keeps them in an LDS
// table instead (kTabW words per check, the same packing as `offs`, a word = two slots), so a
// slot costs one table read per two slots plus the same one or two address ops as with VGPR
// offsets -- against three walk ops per slot and pass.  The table's row pitch kTabW is odd, so each
// 32-lane half of a wave (consecutive checks) reads 32 different banks (ds_read_b32: dword mod 32).
template <int P, int CPL = 1, int NT = kNT, bool STORE_OFFS = true, bool LDS_OFFS = false>
struct ArrayChecks {
    static constexpr int kN = P * P;  // code length, known at compile time
    static constexpr bool kStoreOffs = CPL == 1 && STORE_OFFS;
    static constexpr bool kLdsOffs = LDS_OFFS && !kStoreOffs;
    static constexpr bool kSdwa = kStoreOffs;  // slot-address form (lds_at)
    static constexpr int kOW = kStoreOffs ? (P + 1) / 2 : 1;
    static constexpr int kBp = CPL == 1 ? kBpArray1 : kBpMany;  // bp_mag2 form
    // flood_pk's refill batch and LDS-staged stores (two checks per lane: none, R's kernel spills
    // with the batch; its frames run 50 iterations, so the per-frame work weighs 1 %)
    static constexpr int kRefillBatch = CPL == 1 ? 4 : 0;
    static constexpr int kTabW = ((P + 1) / 2) | 1;  // LDS table words per check (odd pitch)
    static constexpr int kTabWords = kLdsOffs ? kTabW : 0;  // per check, for variant_lds
    uint32_t st[CPL][P];
    uint32_t row[CPL], col[CPL];
    uint32_t offs[kOW];  // kStoreOffs: slot 2w's byte offset in bits 0-15, slot 2w+1's in bits 16-31
    uint32_t tabq[kLdsOffs ? CPL : 1];  // kLdsOffs: LDS byte address of check q's table row
    bool act[CPL];
    // LDS byte address of stored-offset slot k in the buffer at base
    __device__ __forceinline__ uint32_t soff(int k, uint32_t base) const {
        return lds_at<kSdwa>(offs[kStoreOffs ? k >> 1 : 0], k & 1, base);
    }
    // table word w of check q (slots 2w, 2w+1)
    __device__ __forceinline__ uint32_t tword(int q, int w) const {
        return reinterpret_cast<const lds_u32 *>((size_t)tabq[q])[w];
    }
    __device__ __forceinline__ void init(const KArgs &a, int tid, uint32_t *tab = nullptr) {
        if (kLdsOffs) {
            // the table: every check's kTabW words, built once per workgroup (a barrier follows init)
            for (int c = tid; c < a.m; c += NT) {
                const uint32_t r = (uint32_t)(c / P);
                uint32_t x = (uint32_t)(c % P);
                for (int w = 0; w < (P + 1) / 2; ++w) {
                    uint32_t word = 4u * x;
                    x += r;
                    x = x >= (uint32_t)P ? x - P : x;
                    if (2 * w + 1 < P) {
                        word |= (4u * x) << 16;
                        x += r;
                        x = x >= (uint32_t)P ? x - P : x;
                    }
                    tab[c * kTabW + w] = word;
                }
            }
#pragma unroll
            for (int q = 0; q < (kLdsOffs ? CPL : 1); ++q) tabq[q] = lds_addr(tab + (tid + q * NT) * kTabW);
        }
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            const int c = tid + q * NT;  // this lane's checks
            act[q] = c < a.m;
            row[q] = act[q] ? (uint32_t)(c / P) : 0u;
            col[q] = act[q] ? (uint32_t)(c % P) : 0u;
#pragma unroll
            for (int k = 0; k < P; ++k) st[q][k] = 0;
        }
        if (kStoreOffs) {
#pragma unroll
            for (int w = 0; w < kOW; ++w) offs[w] = 0;
            uint32_t x = col[0];
#pragma unroll
            for (int k = 0; k < P; ++k) {
                offs[k >> 1] |= (4u * x) << (16 * (k & 1));
                x += row[0];
                x = x >= (uint32_t)P ? x - P : x;
            }
        }
    }
    // One flooding step for this lane's checks: gather from buffer pc, update, scatter-add into
    // buffer pn (LDS byte addresses).  par: bit 15 / 31 = OR over the lane's checks
    // of each check's syndrome parity for the low / high frame; ovor |= every c2v magnitude.
    __device__ __forceinline__ void step(const KArgs &a, const uint32_t *, uint32_t *, uint32_t pc, uint32_t pn, u16x2 C2,
                                         uint32_t M2, uint32_t &par, uint32_t &ovor) {
        uint32_t fail = 0;  // OR over the lane's checks of each check's parity (not their XOR)
        // (literal operands: the same mask constants in VGPRs measured the same, profiles/r2/ab/bp_form.txt)
        constexpr uint32_t SGN = 0x80008000u, MAG = 0x7fff7fffu;
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            if (!act[q]) continue;
            uint32_t(&stq)[P] = st[q];
            // Gather.  State stq[k] = c2v of the previous step in carry form; becomes the v2c
            // message in sign-magnitude halves (|m| in bits 0-14, m <= 0 in bit 15).
            unsigned short t4 = (unsigned short)(4 * col[q]);  // walked offset (!kStoreOffs)
            if (!kStoreOffs && !kLdsOffs) asm volatile("" : "+v"(t4));
            const unsigned short step4 = (unsigned short)(4 * row[q]), wrap4 = (unsigned short)(4 * P);
            uint32_t px = 0, S = 0;
            [[maybe_unused]] unsigned short tL = 0;  // walked offset of slot L
            // loads in batches of G, issued back to back, so G LDS reads are in flight per wave
            // instead of the compiler's one or two (each waited on a few instructions later)
            constexpr int G = 8;
            if constexpr (kLdsOffs) {
                // software-pipelined like the VGPR-offset gather: batches of 4 slots (2 table
                // words); batch b+1's 4 reads are issued before batch b is processed, and the table
                // words two batches ahead are read before that
                constexpr int G4 = 4, NB = (P + G4 - 1) / G4, NW = (P + 1) / 2;
                uint32_t ow[3][2], Vb[2][G4];
                auto words = [&](int b) {
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        if (2 * b + i < NW) ow[b % 3][i] = tword(q, 2 * b + i);
                };
                auto issue = [&](int b) {
#pragma unroll
                    for (int g = 0; g < G4; ++g) {
                        const int k = b * G4 + g;
                        if (k >= P) break;
                        const uint32_t o = lds_at<kSdwa>(ow[b % 3][g >> 1], k & 1, pc);
                        Vb[b & 1][g] = reinterpret_cast<const lds_u32 *>((size_t)o)[k * P];
                    }
                };
                words(0);
                words(1);
                issue(0);
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    if (b + 2 < NB) words(b + 2);
                    if (b + 1 < NB) issue(b + 1);
                    __builtin_amdgcn_sched_barrier(0);
                    const int k0 = b * G4;
                    if (k0 + G4 <= P) {
                        uint32_t u[G4];
#pragma unroll
                        for (int g = 0; g < G4; ++g) {
                            px ^= Vb[b & 1][g];
                            u[g] = Vb[b & 1][g] - stq[k0 + g];
                        }
                        sign_mag_b_xg<G4>(u);
#pragma unroll
                        for (int g = 0; g < G4; ++g) {
                            S ^= u[g];
                            stq[k0 + g] = u[g];
                        }
                    } else {
#pragma unroll
                        for (int g = 0; g < G4; ++g) {
                            const int k = k0 + g;
                            if (k >= P) break;
                            px ^= Vb[b & 1][g];
                            const uint32_t sm = sign_mag_b(Vb[b & 1][g] - stq[k], SGN);
                            S ^= sm;
                            stq[k] = sm;
                        }
                    }
                }
            } else if constexpr (kStoreOffs) {
                // slots per gather batch: 4, 6, 7 and 8 measured the same; without the batch's
                // scheduling barrier the kernel spills (profiles/r5/ab/post_ra.txt run 9)
                constexpr int G4 = 4, NB = (P + G4 - 1) / G4;
                uint32_t Vb[2][G4];
                auto issue = [&](int b) {
#pragma unroll
                    for (int g = 0; g < G4; ++g) {
                        const int k = b * G4 + g;
                        if (k >= P) break;
                        if (!kStoreOffs && k == (P - 1) / 2) tL = t4;
                        const uint32_t o = kStoreOffs ? soff(k, pc) : pc + t4;
                        Vb[b & 1][g] = reinterpret_cast<const lds_u32 *>((size_t)o)[k * P];
                        if (!kStoreOffs) {
                            t4 = (unsigned short)(t4 + step4);
                            t4 = __builtin_elementwise_min(t4, (unsigned short)(t4 - wrap4));
                        }
                    }
                };
                issue(0);
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    if (b + 1 < NB) issue(b + 1);
                    __builtin_amdgcn_sched_barrier(0);
                    const int k0 = b * G4;
                    if (k0 + G4 <= P) {
                        uint32_t u[G4];
#pragma unroll
                        for (int g = 0; g < G4; ++g) {
                            px ^= Vb[b & 1][g];
                            u[g] = Vb[b & 1][g] - stq[k0 + g];
                        }
                        if constexpr (G4 == 8) sign_mag_b_x(u); else sign_mag_b_xg<G4>(u);
#pragma unroll
                        for (int g = 0; g < G4; ++g) {
                            S ^= u[g];
                            stq[k0 + g] = u[g];
                        }
                    } else {
#pragma unroll
                        for (int g = 0; g < G4; ++g) {
                            const int k = k0 + g;
                            if (k >= P) break;
                            px ^= Vb[b & 1][g];
                            const uint32_t sm = sign_mag_b(Vb[b & 1][g] - stq[k], SGN);
                            S ^= sm;
                            stq[k] = sm;
                        }
                    }
                }
            } else
#pragma unroll
            for (int k0 = 0; k0 < P; k0 += G) {
                uint32_t V[G];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int k = k0 + g;
                    if (k >= P) break;
                    if (!kStoreOffs && k == (P - 1) / 2) tL = t4;
                    const uint32_t o = kStoreOffs ? soff(k, pc) : pc + t4;
                    V[g] = reinterpret_cast<const lds_u32 *>((size_t)o)[k * P];
                    if (!kStoreOffs) {
                        t4 = (unsigned short)(t4 + step4);
                        t4 = __builtin_elementwise_min(t4, (unsigned short)(t4 - wrap4));
                    }
                }
                if (G > 1) __builtin_amdgcn_sched_barrier(0);
                if (k0 + G <= P) {  // whole batch: the last step of sign_mag_b as a borrow chain
                    uint32_t u[G];
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        px ^= V[g];
                        u[g] = V[g] - stq[k0 + g];
                    }
                    sign_mag_b_x(u);
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        S ^= u[g];
                        stq[k0 + g] = u[g];
                    }
                    continue;
                }
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int k = k0 + g;
                    if (k >= P) break;
                    px ^= V[g];                                      // bits 15 / 31: NOT hard (:305-308)
                    const uint32_t sm = sign_mag_b(V[g] - stq[k], SGN);  // v2c = post - c2v (:143-152)
                    S ^= sm;
                    stq[k] = sm;
                }
            }
            // parity of the hard bits = parity of the NOT-hard bits, inverted for an odd degree
            fail |= (px ^ ((P & 1) ? 0x80008000u : 0u)) & 0x80008000u;
            // Middle-out schedule of the reference's fold (:83-116): the forward chain F and the
            // backward chain B run side by side (two independent dependency chains per lane):
            // phase 1 builds F_0..F_{L-1} and B_{L+1}..B_{P-1}; phase 2 extends F rightwards and B
            // leftwards from the middle, emitting c2v_k = F_{k-1} [+] B_{k+1} on both sides.  Every
            // chain and every output is the same fold, in the same order, as the serial schedule.
            constexpr int L = (P - 1) / 2;
            uint32_t FB[P];  // FB[k] = F_k for k < L, B_k for k > L
            FB[0] = stq[0] & MAG;
            FB[P - 1] = stq[P - 1] & MAG;
#pragma unroll
            for (int j = 1; j < P - 1 - L; ++j) {
                if (j < L) FB[j] = bp_mag2<kBp>(FB[j - 1], stq[j] & MAG, C2, M2);
                FB[P - 1 - j] = bp_mag2<kBp>(FB[P - j], stq[P - 1 - j] & MAG, C2, M2);
            }
            // opaque: recompute st & MAG below instead of keeping 46 masked copies live
#pragma unroll
            for (int k = 0; k < P; ++k) asm volatile("" : "+v"(stq[k]));
            // output k: magnitude o, sign = parity of the other inputs' flags = (S ^ flag_k);
            // written back as carry-form c2v o - 2*(o & signmask) (state and scatter value), and
            // scattered into pn as soon as it is emitted (spreads the LDS atomics over phase 2)
            uint32_t F, B;  // running F_{kf-1}, B_{kb+1}
            {
                const uint32_t aL = stq[L] & MAG;
                const uint32_t o = bp_mag2<kBp>(FB[L - 1], FB[L + 1], C2, M2);
                F = bp_mag2<kBp>(FB[L - 1], aL, C2, M2);
                B = bp_mag2<kBp>(FB[L + 1], aL, C2, M2);
                emit_c2v<true>(stq[L], o, S, ovor);
            }
            unsigned short uf = tL, ub = tL;
            if (!kStoreOffs && !kLdsOffs) asm volatile("" : "+v"(uf), "+v"(ub));
            // kLdsOffs: the table words of the forward / backward side's current slot pair, read one
            // pair ahead (wf_n / wb_n) so the read has a whole emission to complete
            uint32_t wf = 0, wb = 0, wf_n = 0, wb_n = 0;
            if (kLdsOffs) {  // the pair holding slot L, and the next pair on each side
                wf = wb = tword(q, L >> 1);
                if ((L >> 1) + 1 < (P + 1) / 2) wf_n = tword(q, (L >> 1) + 1);
                if ((L >> 1) >= 1) wb_n = tword(q, (L >> 1) - 1);
            }
            auto addr = [&](int k, uint32_t w, unsigned short t, uint32_t base) -> uint32_t {
                if (kStoreOffs) return soff(k, base);
                if (kLdsOffs) return lds_at<kSdwa>(w, k & 1, base);
                return base + t;
            };
            lds_add_at(addr(L, wf, tL, pn) + L * P * 4, (int)stq[L]);
#pragma unroll
            for (int j = 1; j <= (L > P - 1 - L ? L : P - 1 - L); ++j) {
                const int kf = L + j, kb = L - j;
                if (kf <= P - 1) {
                    uint32_t o = F;  // c2v_{P-1} = F_{P-2}
                    if (kf <= P - 2) {
                        o = bp_mag2<kBp>(F, FB[kf + 1], C2, M2);
                        F = bp_mag2<kBp>(F, stq[kf] & MAG, C2, M2);
                    }
                    emit_c2v<true>(stq[kf], o, S, ovor);
                    if (!kStoreOffs && !kLdsOffs) {
                        uf = (unsigned short)(uf + step4);
                        uf = __builtin_elementwise_min(uf, (unsigned short)(uf - wrap4));
                    }
                    if (kLdsOffs && (kf >> 1) != ((kf - 1) >> 1)) {  // a new slot pair on this side
                        wf = wf_n;
                        if ((kf >> 1) + 1 < (P + 1) / 2) wf_n = tword(q, (kf >> 1) + 1);
                    }
                    lds_add_at(addr(kf, wf, uf, pn) + kf * P * 4, (int)stq[kf]);
                }
                if (kb >= 0) {
                    uint32_t o = B;  // c2v_0 = B_1
                    if (kb >= 1) {
                        o = bp_mag2<kBp>(FB[kb - 1], B, C2, M2);
                        B = bp_mag2<kBp>(B, stq[kb] & MAG, C2, M2);
                    }
                    emit_c2v<true>(stq[kb], o, S, ovor);
                    if (!kStoreOffs && !kLdsOffs) {
                        ub = (unsigned short)(ub - step4);
                        ub = __builtin_elementwise_min(ub, (unsigned short)(ub + wrap4));
                    }
                    if (kLdsOffs && (kb >> 1) != ((kb + 1) >> 1)) {  // a new slot pair on this side
                        wb = wb_n;
                        if ((kb >> 1) >= 1) wb_n = tword(q, (kb >> 1) - 1);
                    }
                    lds_add_at(addr(kb, wb, ub, pn) + kb * P * 4, (int)stq[kb]);
                }
            }
        }
        par = fail;
    }
    // Syndrome of buffer pc only (no update): bits 15 / 31 of par as in step().  The c2v state is
    // left as it is; every frame in flight ends at this step and is refilled (state cleared) or idle.
    __device__ __forceinline__ uint32_t syndrome(const uint32_t *, uint32_t pc) const {
        uint32_t fail = 0;
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            if (!act[q]) continue;
            uint32_t px = 0;
            if (kStoreOffs) {
#pragma unroll
                for (int k = 0; k < P; ++k)
                    px ^= reinterpret_cast<const lds_u32 *>((size_t)soff(k, pc))[k * P];
            } else if (kLdsOffs) {
#pragma unroll
                for (int w = 0; w < (P + 1) / 2; ++w) {
                    const uint32_t ow = tword(q, w);
                    px ^= reinterpret_cast<const lds_u32 *>((size_t)lds_at<kSdwa>(ow, 0, pc))[2 * w * P];
                    if (2 * w + 1 < P) px ^= reinterpret_cast<const lds_u32 *>((size_t)lds_at<kSdwa>(ow, 1, pc))[(2 * w + 1) * P];
                }
            } else {  // walked offsets, as in step()
                unsigned short t4 = (unsigned short)(4 * col[q]);
                const unsigned short step4 = (unsigned short)(4 * row[q]), wrap4 = (unsigned short)(4 * P);
#pragma nounroll
                for (int k = 0; k < P; ++k) {
                    px ^= reinterpret_cast<const lds_u32 *>((size_t)(pc + t4))[k * P];
                    t4 = (unsigned short)(t4 + step4);
                    t4 = __builtin_elementwise_min(t4, (unsigned short)(t4 - wrap4));
                }
            }
            fail |= (px ^ ((P & 1) ? 0x80008000u : 0u)) & 0x80008000u;
        }
        return fail;
    }
    // zero the refilled half(s) of the carry-form c2v state
    __device__ __forceinline__ void clear(int finished) {
#pragma unroll
        for (int q = 0; q < CPL; ++q)
#pragma unroll
            for (int k = 0; k < P; ++k) {
                if (finished & 1) st[q][k] -= (uint32_t)carry_lo(st[q][k]);
                if (finished & 2) st[q][k] = (uint32_t)carry_lo(st[q][k]);
            }
    }

    // ---- The tail: one frame, its check split over the lane's two halves (flood_pk) ----
    // Once the work queue is empty a workgroup whose partner half has gone idle carries ONE frame,
    // and its packed lanes would spend every instruction's second half on nothing -- the launch then
    // waits on such frames, each at a lone workgroup's step latency.  In the split form the frame sits
    // in half 0 of the LDS words and lane halves fold the two ends of the same check: the low half
    // owns slots j = 0..L-1 (the forward chain F_0..F_{L-1}), the high half slots P-1-j (the backward
    // chain B_{P-1}..B_{L+1}), both the middle slot L -- SplitCore's middle-out schedule with the two
    // sides in the halves of one lane instead of in lanes l and l + 32, the exchange a 16-bit rotate.
    // The same chains and outputs in the same order (:83-116); L + 1 state words per lane, and about
    // 55 % of the packed step's instructions for the one frame.
    static constexpr bool kSplit = CPL == 1 && kStoreOffs;
    static constexpr int SL = (P - 1) / 2;
    static __device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
    // state of the frame in half h (the other half's c2v is zero) -> split pairs (c2v_j, c2v_{P-1-j})
    __device__ __forceinline__ void split_enter(int h) {
        uint32_t(&S)[P] = st[0];
#pragma unroll
        for (int j = 0; j <= SL; ++j) {
            const uint32_t a = S[j], b = S[P - 1 - j];
            const int ca = h ? (int)(a - (uint32_t)carry_lo(a)) >> 16 : carry_lo(a);
            const int cb = h ? (int)(b - (uint32_t)carry_lo(b)) >> 16 : carry_lo(b);
            S[j] = (uint32_t)ca + ((uint32_t)cb << 16);  // carry form lo + 65536 hi (j = L: both c2v_L)
        }
#pragma unroll
        for (int j = SL + 1; j < P; ++j) S[j] = 0;
    }
    __device__ __forceinline__ void split_step(const uint32_t *, uint32_t *, uint32_t pc, uint32_t pn, u16x2 C2,
                                               uint32_t M2, uint32_t &par, uint32_t &ovor) {
        constexpr uint32_t SGN = 0x80008000u, MAG = 0x7fff7fffu;
        constexpr int L = SL, J = L + 1;
        par = 0;
        if (!act[0]) return;
        uint32_t(&S)[P] = st[0];
        // Gather, software-pipelined in batches of 4 pairs as the packed step: own slot j's posterior
        // word and slot P-1-j's, combined into (half 0 of j, half 0 of P-1-j); v2c = that - c2v.
        constexpr int G4 = 4, NB = (J + G4 - 1) / G4;
        uint32_t Va[2][G4], Vc[2][G4];
        auto issue = [&](int b) {
#pragma unroll
            for (int g = 0; g < G4; ++g) {
                const int j = b * G4 + g;
                if (j >= J) break;
                Va[b & 1][g] = reinterpret_cast<const lds_u32 *>((size_t)soff(j, pc))[j * P];
                if (j < L) Vc[b & 1][g] = reinterpret_cast<const lds_u32 *>((size_t)soff(P - 1 - j, pc))[(P - 1 - j) * P];
            }
        };
        uint32_t px = 0, Sg = 0, VL = 0;
        issue(0);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (b + 1 < NB) issue(b + 1);
            __builtin_amdgcn_sched_barrier(0);
            const int j0 = b * G4;
            uint32_t u[G4];
#pragma unroll
            for (int g = 0; g < G4; ++g) {
                const int j = j0 + g;
                if (j >= J) break;
                const uint32_t a = Va[b & 1][g];
                const uint32_t V = __builtin_amdgcn_perm(j < L ? Vc[b & 1][g] : a, a, 0x05040100u);
                if (j < L) px ^= V;  // bits 15 / 31: NOT hard of slots j / P-1-j (:305-308)
                else VL = a;
                u[g] = V - S[j];
            }
            if (j0 + G4 <= J) {
                sign_mag_b_xg<G4>(u);
            } else {
#pragma unroll
                for (int g = 0; g < G4; ++g)
                    if (j0 + g < J) u[g] = sign_mag_b(u[g], SGN);
            }
#pragma unroll
            for (int g = 0; g < G4; ++g) {
                const int j = j0 + g;
                if (j >= J) break;
                if (j < L) Sg ^= u[g];
                S[j] = u[g];
            }
        }
        // the whole check's sign and syndrome parities (each half holds one side's), in both halves
        Sg ^= rot16(Sg) ^ S[L];
        px ^= rot16(px) ^ VL;
        par = (px ^ ((P & 1) ? 0x80008000u : 0u)) & 0x8000u;
        // phase 1: each half's chain over its own slots
        uint32_t X[L];
        X[0] = S[0] & MAG;
#pragma unroll
        for (int j = 1; j < L; ++j) X[j] = bp_mag2<kBp>(X[j - 1], S[j] & MAG, C2, M2);
#pragma unroll
        for (int j = 0; j < J; ++j) asm volatile("" : "+v"(S[j]));  // recompute S & MAG below
        // phase 2: the other half's chain end, the middle output, then that chain extended outwards
        // through own slots (low half: B_L..B_1, high half: F_L..F_{P-2}), emitting as it goes
        const uint32_t R = rot16(X[L - 1]);
        {
            const uint32_t o = bp_mag2<kBp>(X[L - 1], R, C2, M2);
            uint32_t Y = bp_mag2<kBp>(R, S[L] & MAG, C2, M2);
            emit_c2v<true>(S[L], o, Sg, ovor);
            lds_add_at(soff(L, pn) + L * P * 4, carry_lo(S[L]));
#pragma unroll
            for (int j = L - 1; j >= 0; --j) {
                uint32_t oj = Y;  // own slot 0 / P-1: the extended chain itself
                if (j >= 1) {
                    oj = bp_mag2<kBp>(X[j - 1], Y, C2, M2);
                    Y = bp_mag2<kBp>(Y, S[j] & MAG, C2, M2);
                }
                emit_c2v<true>(S[j], oj, Sg, ovor);
                const int lo = carry_lo(S[j]);
                lds_add_at(soff(j, pn) + j * P * 4, lo);
                lds_add_at(soff(P - 1 - j, pn) + (P - 1 - j) * P * 4, (int)(S[j] - (uint32_t)lo) >> 16);
            }
        }
    }
};

// Exchange of one value between lanes l and l + 32 of a wave (gfx950 v_permlane32_swap): the
// builtin swaps the upper half of its first operand with the lower half of its second, so with both
// operands x, r[0] ^ r[1] ^ x is the partner's x in every lane (two full-rate XORs, no select).
__device__ __forceinline__ uint32_t partner32(uint32_t x) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return r[0] ^ r[1] ^ x;
}

// Check side of the packed kernel, array codes, TWO lanes per check: lanes l and l + 32 of a wave
// hold check c = 32 * wave + (l & 31).  Side 0 (l < 32) owns slots 0..L-1, side 1 slots P-1..L+1
// (stored in that order, so both sides run the same instruction stream), and both hold the middle
// slot L (P = 2L + 1).  Each side folds its own slots into its chain (side 0 the forward chain
// F_0..F_{L-1}, side 1 the backward chain B_{P-1}..B_{L+1}), the two chain ends are exchanged once
// (v_permlane32_swap), and each side then extends the OTHER side's chain through its own slots --
// from the middle outwards -- emitting c2v_k = F_{k-1} [+] B_{k+1} for its own k.  These are the
// middle-out schedule's chains and outputs (ArrayChecks, :83-116) split between two lanes: the same
// box-plus operations in the same order per chain, L + 1 fold steps per lane instead of 2L + 1, so a
// frame pair's check step has half the latency on a lone workgroup and twice the waves per frame.
// (sxor is commutative -- min, |x|+|y| and ||x|-|y|| are symmetric -- though not associative, so a
// side 1 operand order such as B_{L+1} [+] F_{L-1} gives the reference's F_{L-1} [+] B_{L+1}.)
// The middle output is computed by both sides (identical) and scattered by side 0 only; the sign
// parity S and the syndrome parity are combined over both sides with one exchange each.
// Offsets: own slot j of side s is slot k = s ? P-1-j : j, at byte offset 4 * (P*k + (col + row*k)
// mod P) (< 64 KiB), two per VGPR.
template <int P>
struct SplitCore {
    static_assert(P % 2 == 1, "odd P");
    static constexpr int L = (P - 1) / 2;  // the middle slot; own slots j = 0..L-1, the middle at j = L
    static constexpr int J = L + 1;        // state words S[0..J)
    static constexpr int OW = (J + 1) / 2; // offset words S[J..J+OW), two 16-bit slot offsets each
    static constexpr int NS = J + OW;
    static constexpr bool kSdwa = true;
    template <int N>
    static __device__ __forceinline__ uint32_t soff(const uint32_t (&S)[N], int j, uint32_t base) {
        return lds_at<kSdwa>(S[J + (j >> 1)], j & 1, base);
    }
    // state zero, offsets of check (row, col) on this side
    template <int N>
    static __device__ __forceinline__ void init(uint32_t (&S)[N], bool act, uint32_t row, uint32_t col, int side) {
        static_assert(N >= NS, "state array too small");
#pragma unroll
        for (int i = 0; i < NS; ++i) S[i] = 0;
        if (act) {
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const uint32_t k = side ? (uint32_t)(P - 1 - j) : (uint32_t)j;
                const uint32_t o = 4u * (P * k + (col + row * k) % P);
                S[J + (j >> 1)] |= o << (16 * (j & 1));
            }
        }
    }
    template <int N>
    static __device__ __forceinline__ void step(uint32_t (&S)[N], bool act, uint32_t keepL, uint32_t pc, uint32_t pn, u16x2 C2,
                                                uint32_t M2, uint32_t &par, uint32_t &ovor) {
        constexpr uint32_t SGN = 0x80008000u, MAG = 0x7fff7fffu;
        par = 0;
        if (!act) return;
        // Gather (software-pipelined in batches of 4, as ArrayChecks): S[j] = v2c in sign-magnitude
        constexpr int G4 = 4, NB = (J + G4 - 1) / G4;
        uint32_t Vb[2][G4];
        uint32_t px = 0, Sg = 0, VL = 0;
        auto issue = [&](int b) {
#pragma unroll
            for (int g = 0; g < G4; ++g) {
                const int j = b * G4 + g;
                if (j >= J) break;
                Vb[b & 1][g] = *reinterpret_cast<const lds_u32 *>((size_t)soff(S, j, pc));
            }
        };
        issue(0);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (b + 1 < NB) issue(b + 1);
            __builtin_amdgcn_sched_barrier(0);
            const int j0 = b * G4;
            if (j0 + G4 <= J) {
                uint32_t u[G4];
#pragma unroll
                for (int g = 0; g < G4; ++g) u[g] = Vb[b & 1][g] - S[j0 + g];
                sign_mag_b_xg<G4>(u);
#pragma unroll
                for (int g = 0; g < G4; ++g) S[j0 + g] = u[g];
            } else {
#pragma unroll
                for (int g = 0; g < G4; ++g) {
                    const int j = j0 + g;
                    if (j >= J) break;
                    S[j] = sign_mag_b(Vb[b & 1][g] - S[j], SGN);
                }
            }
#pragma unroll
            for (int g = 0; g < G4; ++g) {
                const int j = j0 + g;
                if (j >= J) break;
                if (j < L) {
                    px ^= Vb[b & 1][g];  // bits 15 / 31: NOT hard (:305-308)
                    Sg ^= S[j];
                } else {
                    VL = Vb[b & 1][g];
                }
            }
        }
        // Phase 1: this side's chain over its own slots
        uint32_t X[L];
        X[0] = S[0] & MAG;
#pragma unroll
        for (int j = 1; j < L; ++j) X[j] = bp_mag2<kBpMany>(X[j - 1], S[j] & MAG, C2, M2);
#pragma unroll
        for (int j = 0; j < J; ++j) asm volatile("" : "+v"(S[j]));  // recompute S & MAG below
        // the exchange: the partner's chain end, sign parity and syndrome parity
        const uint32_t R = partner32(X[L - 1]);
        Sg ^= partner32(Sg) ^ S[L];
        px ^= partner32(px) ^ VL;
        par = (px ^ ((P & 1) ? 0x80008000u : 0u)) & 0x80008000u;
        // Phase 2: the middle output, then the partner's chain extended outwards through own slots
        {
            const uint32_t o = bp_mag2<kBpMany>(X[L - 1], R, C2, M2);
            const uint32_t aL = S[L] & MAG;
            uint32_t Y = bp_mag2<kBpMany>(R, aL, C2, M2);
            emit_c2v<true>(S[L], o, Sg, ovor);
            lds_add_at(soff(S, L, pn), (int)(S[L] & keepL));
#pragma unroll
            for (int j = L - 1; j >= 0; --j) {
                uint32_t oj = Y;  // own slot 0's output: the extended chain itself
                if (j >= 1) {
                    oj = bp_mag2<kBpMany>(X[j - 1], Y, C2, M2);
                    Y = bp_mag2<kBpMany>(Y, S[j] & MAG, C2, M2);
                }
                emit_c2v<true>(S[j], oj, Sg, ovor);
                lds_add_at(soff(S, j, pn), (int)S[j]);
            }
        }
    }
    // Syndrome of buffer pc only (no update), bits 15 / 31 as in step()
    template <int N>
    static __device__ __forceinline__ uint32_t syndrome(const uint32_t (&S)[N], bool act, uint32_t pc) {
        if (!act) return 0;
        uint32_t px = 0;
#pragma unroll
        for (int j = 0; j < L; ++j) px ^= *reinterpret_cast<const lds_u32 *>((size_t)soff(S, j, pc));
        const uint32_t VL = *reinterpret_cast<const lds_u32 *>((size_t)soff(S, L, pc));
        px ^= partner32(px) ^ VL;
        return (px ^ ((P & 1) ? 0x80008000u : 0u)) & 0x80008000u;
    }
    // zero the refilled half(s) of the state words (the offset words are left alone)
    template <int N>
    static __device__ __forceinline__ void clear(uint32_t (&S)[N], int finished) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (finished & 1) S[j] -= (uint32_t)carry_lo(S[j]);
            if (finished & 2) S[j] = (uint32_t)carry_lo(S[j]);
        }
    }
};

// R-sized array codes (1024 < m <= NT + 256 + 128): the LDS-offset-table policy with 2 checks per lane
// for checks [0, NT + 256) -- the second check on threads [0, 256) only -- and the remaining checks
// (R: 104) two lanes per check (SplitCore) on threads [256, 512), their state and offsets in the
// words of the second-check state those lanes do not use.  R's 1128 checks are 17.6 wave-units of
// one check per lane: as 2 checks per lane they load the SIMDs 5 / 5 / 4 / 4 per step (some SIMD
// carries two second-pass units); here every SIMD carries 3 + 1 whole units and one split unit of
// half the work, 4.5.
template <int P, int NT = 768>
struct MixChecks {
    static constexpr bool kSplit = false;
    static constexpr int kRefillBatch = 0;
    using Reg = ArrayChecks<P, 2, NT, true, true>;
    using Sp = SplitCore<P>;
    static_assert(Sp::NS <= P, "split state must fit a check's state words");
    static constexpr int kN = P * P;
    static constexpr int kTabWords = Reg::kTabWords;
    static constexpr int kSplitBase = NT + 256;  // first split check
    Reg reg;
    uint32_t keepL;
    bool split_lane, sact;
    __device__ __forceinline__ void init(const KArgs &a, int tid_in, uint32_t *tab) {
        // Roles of the three 256-thread blocks of waves (one wave of each per SIMD): the oldest block
        // (threads 0..255) takes one whole check + the split units, the middle block the two whole
        // checks, the youngest one whole check.  Round 6's per-wave stamps (FPLDPC_WAIT_TRACE) showed
        // the hardware's age-ordered issue finishing the oldest, heaviest waves first and parking them
        // at the step barrier for 36 % of their time; of the six role orders measured
        // (profiles/r6/ab/r_roles.txt) this one ran fastest, and with wave priorities 1 / 0 / 2 on top
        // R went 666 -> 677 Mb/s (r_prio.txt, r_prio2.txt).  Since the quick exit between steps the
        // priorities cost 0.3-0.4 % (profiles/r6/ab/r_prio_quick.txt) and are gone.  `u` is the lane's
        // check index as before (the same 32-lane pairs for the split units: u & 63 == tid & 63).
        // (roles as hex digits, block b in digit b)
        constexpr int kRoles = 0x201;
        const int tid = ((kRoles >> (4 * (tid_in >> 8))) & 0xf) * 256 + (tid_in & 255);
        reg.init(a, tid, tab);
        reg.act[1] = reg.act[1] && tid < 256;
        split_lane = tid >= 256 && tid < 512;
        const int l = tid & 63, side = l >> 5;
        const int c = kSplitBase + ((tid - 256) >> 6) * 32 + (l & 31);
        sact = split_lane && c < a.m;
        keepL = side ? 0u : ~0u;
        if (split_lane) Sp::init(reg.st[1], sact, sact ? (uint32_t)(c / P) : 0u, sact ? (uint32_t)(c % P) : 0u, side);
    }
    __device__ __forceinline__ void step(const KArgs &a, const uint32_t *pcp, uint32_t *pnp, uint32_t pc, uint32_t pn, u16x2 C2,
                                         uint32_t M2, uint32_t &par, uint32_t &ovor) {
        reg.step(a, pcp, pnp, pc, pn, C2, M2, par, ovor);
        if (split_lane) {
            uint32_t p2 = 0;
            Sp::step(reg.st[1], sact, keepL, pc, pn, C2, M2, p2, ovor);
            par |= p2;
        }
    }
    __device__ __forceinline__ uint32_t syndrome(const uint32_t *pcp, uint32_t pc) const {
        uint32_t f = reg.syndrome(pcp, pc);
        if (split_lane) f |= Sp::syndrome(reg.st[1], sact, pc);
        return f;
    }
    __device__ __forceinline__ void clear(int finished) {
        // the second check's words beyond the split state hold the split offsets on split lanes
        uint32_t keep[Sp::OW];
#pragma unroll
        for (int w = 0; w < Sp::OW; ++w) keep[w] = reg.st[1][Sp::J + w];
        reg.clear(finished);
        if (split_lane) {
#pragma unroll
            for (int w = 0; w < Sp::OW; ++w) reg.st[1][Sp::J + w] = keep[w];
        }
    }
};

// Check side of the packed kernel, any code with check degree <= DC (irregular allowed, e.g. the
// 802.11n code: degrees 7 and 8): CPL checks per lane (check c = tid + q*256), per-slot gather
// byte offsets packed two per VGPR (from the [DC][m_pad] var-index table), c2v state (carry form)
// in VGPRs.  The fold follows the reference's serial schedule; slots k >= deg are masked (DMIN:
// the smallest check degree the variant accepts, so slots below it need no masks).
// QLO > 0: the decoder's table lists the checks by ascending degree and the first QLO passes
// (checks [0, QLO*256)) all have degree DMIN exactly (choose_kernel checks it), so those passes fold
// DMIN slots with no masks and no gather, box-plus or emission for slot DMIN..DC-1 -- W: 768 of its
// 972 checks are degree 7, and a degree-7 check in an 8-slot pass pays for the 8th slot.  Check
// order is free: each check's fold is its own, and the posterior sums are integer adds (atomics
// from many waves already arrive in any order).
template <int DC, int CPL, int DMIN, int QLO = 0, int TNT = kNT>
struct TableChecks {
    static_assert(QLO >= 0 && QLO <= CPL && DMIN <= DC, "bad pass split");
    // The tail's split form (round 6): one frame in half 0 of the LDS words, and a lane's four checks
    // fold two at a time -- q0 in the low half with q2 in the high half, then q1 with q3 -- so a lone
    // frame's step is two passes instead of four.  Needs the degree-sorted layout with QLO = 3 (q0..q2
    // all of degree DMIN; q3 DMIN..DC or absent).  W @ 2 dB +4.5 %, W at 30 iterations +0.3 %, with W's
    // translation unit compiled without the post-RA scheduler (profiles/r6/ab/w_split_options.txt;
    // round 5's version in the shared unit: +3 % / -2 to -5 %, the packed loop's registers reallocated).
    static constexpr bool kSplit = CPL == 4 && QLO == 3 && DC == DMIN + 1;
    static __device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
    static constexpr int kRefillBatch = 4;
    static constexpr int kTabWords = 0;
    static constexpr int kN = 0;  // code length at run time
    // posteriors as biased pairs with the array policy's borrow-chain sign/magnitude (W +1.0 % over
    // carry form, profiles/r2/ab/tab_biased.txt; round 1's biased variant without the borrow chain
    // measured the same, profiles/r1/ab/w_biased.jsonl)
    static constexpr int DP = (DC + 1) / 2;
    uint32_t st[CPL][DC];
    uint32_t off[CPL][DP];  // byte offsets 4*var of slots 2j (low 16 bits) and 2j+1 (high)
    int deg[CPL];
    // slots folded by pass Q, and its degree (a compile-time DMIN in the QLO passes)
    template <int Q>
    static constexpr int slots() { return Q < QLO ? DMIN : DC; }
    template <int Q>
    __device__ __forceinline__ int degree() const { return Q < QLO ? DMIN : deg[Q]; }
    __device__ __forceinline__ void init(const KArgs &a, int tid, uint32_t * = nullptr) {
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            const int c = tid + q * TNT;
            const bool act = c < a.m;
            deg[q] = act ? (int)a.cdeg[c] : 0;
#pragma unroll
            for (int j = 0; j < DP; ++j) {
                uint32_t lo = 0, hi = 0;
                if (act) {
                    lo = 4u * a.vidx[(size_t)(2 * j) * a.m_pad + c];
                    if (2 * j + 1 < DC) hi = 4u * a.vidx[(size_t)(2 * j + 1) * a.m_pad + c];
                }
                off[q][j] = lo | (hi << 16);
            }
#pragma unroll
            for (int k = 0; k < DC; ++k) st[q][k] = 0;
        }
    }
    __device__ __forceinline__ uint32_t o16(int q, int k) const {
        return (k & 1) ? off[q][k >> 1] >> 16 : off[q][k >> 1] & 0xffffu;
    }
    template <int Q>
    __device__ __forceinline__ void step_q(const char *pcb, char *pnb, u16x2 C2, uint32_t M2, uint32_t &fail,
                                           uint32_t &ovor) {
        constexpr uint32_t MAG = 0x7fff7fffu;
        constexpr int D = slots<Q>();
        const int d = degree<Q>();
        if (Q >= QLO && d == 0) return;
        uint32_t sm[D];
        uint32_t S = 0, px = 0;
        // bits 15 / 31 of a biased pair: NOT hard (:305-308)
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const uint32_t V = *reinterpret_cast<const uint32_t *>(pcb + o16(Q, k));
            px ^= (k < DMIN || k < d) ? V : 0u;
            sm[k] = V - st[Q][k];  // biased v2c = post - c2v (:143-152)
        }
        if constexpr (D == 8) {
            sign_mag_b_x(sm);
        } else if constexpr (D == 7 || D == 6 || D == 4) {
            sign_mag_b_xg<D>(sm);
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) sm[k] = sign_mag_b(sm[k]);
        }
#pragma unroll
        for (int k = 0; k < D; ++k) S ^= (k < DMIN || k < d) ? sm[k] : 0u;
        fail |= (px ^ ((d & 1) ? 0x80008000u : 0u)) & 0x80008000u;
        // serial forward/backward fold (:83-116) over the first d slots
        uint32_t B[D];
        B[D - 1] = sm[D - 1] & MAG;
#pragma unroll
        for (int k = D - 2; k >= 1; --k) {
            const uint32_t b = bp_mag2<kBpMany>(B[k + 1], sm[k] & MAG, C2, M2);
            B[k] = (k < DMIN - 1 || k < d - 1) ? b : sm[k] & MAG;
        }
        uint32_t F = sm[0] & MAG;
        uint32_t o0 = B[1];
        ovor |= o0;
        emit_c2v(sm[0], o0, S, ovor);
#pragma unroll
        for (int k = 1; k <= D - 2; ++k) {
            const uint32_t ak = sm[k] & MAG;
            const uint32_t ob = bp_mag2<kBpMany>(F, B[k + 1], C2, M2);
            const uint32_t o = (k < DMIN - 1 || k < d - 1) ? ob : F;
            if (k < DMIN || k < d) ovor |= o;
            uint32_t t = sm[k];
            emit_c2v(t, o, S, dummy_);
            sm[k] = t;
            F = bp_mag2<kBpMany>(F, ak, C2, M2);
        }
        if (d == D) ovor |= F;
        emit_c2v(sm[D - 1], F, S, dummy_);
#pragma unroll
        for (int k = 0; k < D; ++k) {
            if (k < DMIN || k < d) {
                st[Q][k] = sm[k];
                lds_add(reinterpret_cast<int *>(pnb + o16(Q, k)), (int)sm[k]);
            }
        }
    }
    template <int... Qs>
    __device__ __forceinline__ void step_all(std::integer_sequence<int, Qs...>, const char *pcb, char *pnb, u16x2 C2,
                                             uint32_t M2, uint32_t &fail, uint32_t &ovor) {
        (step_q<Qs>(pcb, pnb, C2, M2, fail, ovor), ...);
    }
    __device__ __forceinline__ void step(const KArgs &a, const uint32_t *pc, uint32_t *pn, uint32_t, uint32_t, u16x2 C2,
                                         uint32_t M2, uint32_t &par, uint32_t &ovor) {
        uint32_t fail = 0;  // OR over this lane's checks of each check's parity (not their XOR)
        step_all(std::make_integer_sequence<int, CPL>{}, reinterpret_cast<const char *>(pc), reinterpret_cast<char *>(pn),
                 C2, M2, fail, ovor);
        par = fail;
    }
    template <int Q>
    __device__ __forceinline__ void syndrome_q(const char *pcb, uint32_t &fail) const {
        constexpr int D = slots<Q>();
        const int d = degree<Q>();
        if (Q >= QLO && d == 0) return;
        uint32_t px = 0;
#pragma unroll
        for (int k = 0; k < D; ++k) {  // unrolled: off[] stays in registers
            const uint32_t V = *reinterpret_cast<const uint32_t *>(pcb + o16(Q, k));
            px ^= (k < DMIN || k < d) ? V : 0u;
        }
        fail |= (px ^ ((d & 1) ? 0x80008000u : 0u)) & 0x80008000u;
    }
    template <int... Qs>
    __device__ __forceinline__ void syndrome_all(std::integer_sequence<int, Qs...>, const char *pcb, uint32_t &fail) const {
        (syndrome_q<Qs>(pcb, fail), ...);
    }
    __device__ __forceinline__ uint32_t syndrome(const uint32_t *pc, uint32_t) const {
        uint32_t fail = 0;
        syndrome_all(std::make_integer_sequence<int, CPL>{}, reinterpret_cast<const char *>(pc), fail);
        return fail;
    }
    __device__ __forceinline__ void clear(int finished) {
#pragma unroll
        for (int q = 0; q < CPL; ++q)
#pragma unroll
            for (int k = 0; k < DC; ++k) {
                if (q < QLO && k >= DMIN) continue;  // slots the QLO passes never use
                if (finished & 1) st[q][k] -= (uint32_t)carry_lo(st[q][k]);
                if (finished & 2) st[q][k] = (uint32_t)carry_lo(st[q][k]);
            }
    }

    // ---- split form (kSplit) ----
    // state of the frame in half h -> pairs st[p][k] = (c2v of check p, of check p + 2) in carry form
    __device__ __forceinline__ void split_enter(int h) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int k = 0; k < DC; ++k) {
                const uint32_t a = st[p][k], b = st[p + 2][k];
                const int ca = h ? (int)(a - (uint32_t)carry_lo(a)) >> 16 : carry_lo(a);
                const int cb = h ? (int)(b - (uint32_t)carry_lo(b)) >> 16 : carry_lo(b);
                st[p][k] = (uint32_t)ca + ((uint32_t)cb << 16);
                st[p + 2][k] = 0;
            }
    }
    // One split pass: check PS in the low half, check PS + 2 in the high half, both of the frame in
    // half 0 of the posterior words.  The low check has degree DMIN (a QLO pass); the high one DMIN
    // (PS = 0) or its own degree dh in {0, DMIN, DC} (PS = 1): the DC-th slot, and every slot of an
    // absent check, is masked per half.  The same chains in the same order as step_q.
    template <int PS>
    __device__ __forceinline__ void split_pass(const char *pcb, char *pnb, u16x2 C2, uint32_t M2, uint32_t &fail,
                                               uint32_t &ovor) {
        constexpr uint32_t MAG = 0x7fff7fffu;
        constexpr int D = PS == 0 ? DMIN : DC;
        const int dh = PS == 0 ? DMIN : deg[3];
        // per-half validity of slot k: low k < DMIN, high k < dh
        auto vm = [&](int k) -> uint32_t { return (k < DMIN ? 0x0000ffffu : 0u) | (k < dh ? 0xffff0000u : 0u); };
        uint32_t sm[D];
        uint32_t S = 0, px = 0;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const uint32_t Vl = *reinterpret_cast<const uint32_t *>(pcb + o16(PS, k));
            const uint32_t Vh = *reinterpret_cast<const uint32_t *>(pcb + o16(PS + 2, k));
            const uint32_t V = __builtin_amdgcn_perm(Vh, Vl, 0x05040100u);  // (half 0 of Vl, half 0 of Vh)
            px ^= PS == 0 ? V : V & vm(k);
            sm[k] = V - st[PS][k];
        }
        if constexpr (D == 8) sign_mag_b_x(sm); else sign_mag_b_xg<D>(sm);
#pragma unroll
        for (int k = 0; k < D; ++k) S ^= PS == 0 ? sm[k] : sm[k] & vm(k);
        fail |= (px ^ ((DMIN & 1) ? 0x8000u : 0u) ^ ((dh & 1) ? 0x80000000u : 0u)) & 0x80008000u;
        uint32_t o[D];
        if constexpr (PS == 0) {  // both halves DMIN slots: the plain fold
            uint32_t B[D];
            B[D - 1] = sm[D - 1] & MAG;
#pragma unroll
            for (int k = D - 2; k >= 1; --k) B[k] = bp_mag2<kBpMany>(B[k + 1], sm[k] & MAG, C2, M2);
            uint32_t F = sm[0] & MAG;
            o[0] = B[1];
#pragma unroll
            for (int k = 1; k <= D - 2; ++k) {
                o[k] = bp_mag2<kBpMany>(F, B[k + 1], C2, M2);
                F = bp_mag2<kBpMany>(F, sm[k] & MAG, C2, M2);
            }
            o[D - 1] = F;
        } else {  // low DMIN = DC - 1 slots; high DC slots when dh == DC
            const uint32_t h8 = dh == DC ? 0xffff0000u : 0u;
            uint32_t B[D];
            B[D - 1] = sm[D - 1] & MAG;
            {
                const uint32_t b = bp_mag2<kBpMany>(B[D - 1], sm[D - 2] & MAG, C2, M2);
                B[D - 2] = (b & h8) | (sm[D - 2] & MAG & ~h8);
            }
#pragma unroll
            for (int k = D - 3; k >= 1; --k) B[k] = bp_mag2<kBpMany>(B[k + 1], sm[k] & MAG, C2, M2);
            uint32_t F = sm[0] & MAG;
            o[0] = B[1];
#pragma unroll
            for (int k = 1; k <= D - 3; ++k) {
                o[k] = bp_mag2<kBpMany>(F, B[k + 1], C2, M2);
                F = bp_mag2<kBpMany>(F, sm[k] & MAG, C2, M2);
            }
            {  // slot D - 2: the last slot of a DMIN check (F), an inner one of a DC check
                const uint32_t b = bp_mag2<kBpMany>(F, B[D - 1], C2, M2);
                o[D - 2] = (b & h8) | (F & ~h8);
                F = bp_mag2<kBpMany>(F, sm[D - 2] & MAG, C2, M2);
            }
            o[D - 1] = F;  // (high half only)
        }
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const uint32_t ok = PS == 0 ? o[k] : o[k] & vm(k);  // (an absent high check: dh = 0)
            ovor |= ok;
            uint32_t t = sm[k];
            emit_c2v(t, ok, S, dummy_);
            st[PS][k] = t;
            const int lo = carry_lo(t);
            if (k < DMIN) lds_add(reinterpret_cast<int *>(pnb + o16(PS, k)), lo);
            if (PS == 0 || k < dh) lds_add(reinterpret_cast<int *>(pnb + o16(PS + 2, k)), (int)(t - (uint32_t)lo) >> 16);
        }
    }
    __device__ __forceinline__ void split_step(const uint32_t *pc, uint32_t *pn, uint32_t, uint32_t, u16x2 C2,
                                               uint32_t M2, uint32_t &par, uint32_t &ovor) {
        uint32_t fail = 0;
        split_pass<0>(reinterpret_cast<const char *>(pc), reinterpret_cast<char *>(pn), C2, M2, fail, ovor);
        split_pass<1>(reinterpret_cast<const char *>(pc), reinterpret_cast<char *>(pn), C2, M2, fail, ovor);
        par = (fail | fail >> 16) & 0x8000u;  // the one frame fails if either half's check does
    }
    uint32_t dummy_ = 0;
};


// (the tail's split step, for the policies that have one)
template <class CK>
__device__ __forceinline__ void split_step_of(CK &ck, const uint32_t *pcp, uint32_t *pnp, uint32_t pc, uint32_t pn,
                                              u16x2 C2, uint32_t M2, uint32_t &par, uint32_t &ovor) {
    if constexpr (CK::kSplit) ck.split_step(pcp, pnp, pc, pn, C2, M2, par, ovor);
}

template <class CK, int WAVES, int NT = kNT>
__global__ void __launch_bounds__(NT, WAVES) flood_pk(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    const int n = CK::kN ? CK::kN : a.n;
    uint32_t *const bufs = reinterpret_cast<uint32_t *>(smem);  // 3 x n posteriors, biased pairs
    uint32_t *const llrc = bufs + 3 * n;                          // n channel LLRs, biased pairs
    int *const misc = smem + 4 * n;
    // misc: [0,1] frame of half h (-1 idle)  [2,3] start step  [4,5] load taint  [6..8] flag words
    //       [12] final-pass syndrome word  [13] deferred range-check word
    //       [9,10] bit-error accumulators
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    u16x2 C2 = (u16x2)(unsigned short)a.C;
    uint32_t M2 = ((1u << a.bfe_w) - 1u) * 0x10001u;
    {  // box-plus constants in VGPRs, not SGPRs (bp_mag2)
        uint32_t c2w = W(C2);
        asm volatile("" : "+v"(c2w), "+v"(M2));
        C2 = U2(c2w);
    }

    for (int v = tid; v < 4 * n; v += NT) bufs[v] = 0x7fff7fffu;  // zero posteriors (biased pairs)
    if (tid < kMiscInts) misc[tid] = tid < 2 ? -1 : 0;
    CK ck;
    ck.init(a, tid, reinterpret_cast<uint32_t *>(smem + 4 * n + kMiscInts));  // (array LDS-offset table)
    constexpr int kRB = CK::kRefillBatch;  // refill: LLR words per thread in flight (0: one at a time)
    // kRB > 0: the masked-BER info positions / reference bits ([2][hard_words], the same for every
    // frame of the call) staged in LDS after the check table, so a frame's store reads no global
    // memory on its critical path (variant_lds reserves the words)
    uint32_t *const lmask = reinterpret_cast<uint32_t *>(smem + 4 * n + kMiscInts) + (size_t)a.m * CK::kTabWords;
    if (kRB > 0 && a.info_mask && a.k_info > 0)
        for (int i = tid; i < 2 * a.hard_words; i += NT) lmask[i] = a.info_mask[i];
    uint32_t ovf = 0;
    bool taint[2] = {false, false};
    __syncthreads();

    unsigned long long trace_t0 = 0;
    int trace_frames = 0;  // thread 0: frames pulled (diagnostic trace)
#if FPLDPC_PHASE_TRACE
    // diagnostic build only: thread 0's s_memrealtime ticks in the refills, the frame pulls inside
    // them (FPLDPC_PHASE_TRACE=2: the stores' ballot loops instead; 3: the refills' part up to the
    // second barrier) and the stores, and the steps run (3: the refills' load loops) (trace words 4..7)
    unsigned long long ph_refill = 0, ph_pull = 0, ph_store = 0, ph_steps = 0, ph_sloop = 0, ph_rhead = 0, ph_rload = 0;
#define PH_T0(v) const unsigned long long v = (tid == 0) ? __builtin_amdgcn_s_memrealtime() : 0ull
#define PH_ADD(acc, v) if (tid == 0) acc += __builtin_amdgcn_s_memrealtime() - v
#else
#define PH_T0(v)
#define PH_ADD(acc, v)
#endif
#if FPLDPC_WAIT_TRACE
    // diagnostic build only (tools/wait_trace.py): per wave, s_memtime cycles in the packed loop's
    // check step, at its per-step barrier, and in the whole packed loop, written after the
    // [grid][8] trace words as [grid][64]: wave w's {step, barrier, loop, steps, other barriers} at
    // 5w..5w+4 (up to 12 waves)
    unsigned long long wt_step = 0, wt_bar = 0, wt_loop0 = __builtin_amdgcn_s_memtime(), wt_steps = 0, wt_bar2 = 0;
    // the other barriers of the packed loop (refills, stores, the final-update syndrome pass, the
    // range check): their waits in wt_bar2.  FPLDPC_WAIT_TRACE=2: word 4 holds the per-step LLR copy
    // instead; 3: everything after the per-step barrier (decisions, stores, refills)
#if FPLDPC_WAIT_TRACE >= 2
#define PK_SYNC() __syncthreads()
#else
#define PK_SYNC()                                                         \
    do {                                                                  \
        const unsigned long long pk_t = __builtin_amdgcn_s_memtime();     \
        __syncthreads();                                                  \
        wt_bar2 += __builtin_amdgcn_s_memtime() - pk_t;                   \
    } while (0)
#endif
#else
#define PK_SYNC() __syncthreads()
#endif
#if FPLDPC_TAIL_TRACE
    // diagnostic build only (tools/tail_trace.py): thread 0's s_memrealtime when a pull first found
    // the queue empty and when the workgroup entered the split tail, and the steps it then ran with
    // two live frames, one live frame (packed) and in the split form (trace words 4..7)
    unsigned long long tt_empty = 0, tt_split = 0, tt_two = 0, tt_one = 0, tt_splits = 0;
#endif
    // (Re)fill the halves in `mask` before step s: new frames' LLRs into llrc, into the buffer
    // read at step s (pc) and the one accumulated at step s (pn); c2v state and overflow trackers
    // of the half cleared.  Uniform control flow (every thread calls it with the same arguments).
    auto refill = [&](int mask, int s, int cur_next) {
        PH_T0(ph_r0);
        // kRB > 0: one atomic for every refilled half, issued before the barrier so that its round
        // trip overlaps the wait (frames wi, wi + 1 in half order, as two pulls in a row would give)
        int got[2] = {-1, -1};
        if (kRB > 0 && tid == 0) {
            const int wi = atomicAdd(a.work_counter, (mask & 1) + (mask >> 1));
            const int lim = a.frame_list ? *a.frame_count : a.batch;
            const int w1 = wi + (mask & 1);
            if ((mask & 1) && wi < lim) got[0] = a.frame_list ? a.frame_list[wi] : wi;
            if ((mask & 2) && w1 < lim) got[1] = a.frame_list ? a.frame_list[w1] : w1;
        }
        // every wave has finished reading misc[0..3] (finish decision, store) before thread 0
        // replaces the frame ids and start steps
        PK_SYNC();
        if (tid == 0) {
            misc[13] = 0;  // deferred range-check word (read by every wave before the barrier above)
            for (int h = 0; h < 2; ++h)
                if (mask >> h & 1) {
                    PH_T0(ph_p0);
                    misc[h] = kRB > 0 ? got[h] : pull_frame(a, a.work_counter);
                    PH_ADD(ph_pull, ph_p0);
#if FPLDPC_TAIL_TRACE
                    if (misc[h] < 0 && !tt_empty) tt_empty = __builtin_amdgcn_s_memrealtime();
#endif
                    trace_frames += misc[h] >= 0;
                    misc[2 + h] = s;
                    misc[4 + h] = 0;
                    misc[9 + h] = 0;
                }
        }
        PK_SYNC();
        PH_ADD(ph_rhead, ph_r0);
        PH_T0(ph_l0);
        uint32_t *pc = bufs + cur_next * n;
        uint32_t *pn = bufs + ((cur_next + 1) % 3) * n;
        if constexpr (kRB > 0) {
            // both refilled halves at once, kRB words per thread with their loads in flight
            // together, one read-modify-write of each LDS word for both halves
            constexpr int KB = kRB > 0 ? kRB : 1;
            const int f0 = (mask & 1) ? misc[0] : -1, f1 = (mask & 2) ? misc[1] : -1;
            bool big0 = false, big1 = false;
            int v0 = tid;
            asm volatile("" : "+v"(v0));
            auto ld = [&](int f, int v) -> int {
                const size_t i = (size_t)f * n + v;
                return a.llr_i16 ? (int)static_cast<const int16_t *>(a.llr)[i] : static_cast<const int32_t *>(a.llr)[i];
            };
            for (int vb = v0; vb < n; vb += KB * NT) {
                int x0[KB], x1[KB];
#pragma unroll
                for (int j = 0; j < KB; ++j) {
                    const int v = vb + j * NT;
                    x0[j] = (v < n && f0 >= 0) ? ld(f0, v) : 0;
                    x1[j] = (v < n && f1 >= 0) ? ld(f1, v) : 0;
                }
#pragma unroll
                for (int j = 0; j < KB; ++j) {
                    const int v = vb + j * NT;
                    if (v < n) {
                        if (x0[j] > kLlrMax || x0[j] < -kLlrMax) {
                            big0 = true;
                            x0[j] = 0;
                        }
                        if (x1[j] > kLlrMax || x1[j] < -kLlrMax) {
                            big1 = true;
                            x1[j] = 0;
                        }
                        uint32_t L = llrc[v], C = pc[v], N = pn[v];
                        if (mask & 1) {
                            L = bias_set(L, 0, x0[j]);
                            C = bias_set(C, 0, x0[j]);
                            N = bias_set(N, 0, x0[j]);
                        }
                        if (mask & 2) {
                            L = bias_set(L, 1, x1[j]);
                            C = bias_set(C, 1, x1[j]);
                            N = bias_set(N, 1, x1[j]);
                        }
                        llrc[v] = L;
                        pc[v] = C;
                        pn[v] = N;
                    }
                }
            }
            if (big0) atomicOr(&misc[4], 1);
            if (big1) atomicOr(&misc[5], 1);
        }
        for (int h = 0; h < 2 && kRB == 0; ++h) {
            if (!(mask >> h & 1)) continue;
            const int f = misc[h];
            bool big = false;
            // (an opaque start, so the loop's per-lane bounds are not hoisted out of the step loop
            // and held in VGPRs across it -- A 163 -> 142 VGPRs, +4.7 %; R's spills gone,
            // profiles/r3/ab/opaque_loops*.txt)
            int v0 = tid;
            asm volatile("" : "+v"(v0));
            for (int v = v0; v < n; v += NT) {
                int x = 0;
                if (f >= 0) {
                    const size_t i = (size_t)f * n + v;
                    x = a.llr_i16 ? (int)static_cast<const int16_t *>(a.llr)[i] : static_cast<const int32_t *>(a.llr)[i];
                    if (x > kLlrMax || x < -kLlrMax) {
                        big = true;
                        x = 0;
                    }
                }
                llrc[v] = bias_set(llrc[v], h, x);
                pc[v] = bias_set(pc[v], h, x);
                pn[v] = bias_set(pn[v], h, x);
            }
            if (big) atomicOr(&misc[4 + h], 1);
        }
        PH_ADD(ph_rload, ph_l0);
        PK_SYNC();
        PH_ADD(ph_refill, ph_r0);
    };

    // Outputs of the frame in half h: posteriors / hard decisions from buffer pf (biased pairs),
    // or the channel decision on a pre-check pass (posteriors left untouched).
    // calculateBER (ArrayLDPC_Decoder.cpp:707-722) with distinct info positions (a.info_mask) comes
    // out of the hard-decision ballots: errors = popcount((hard ^ ref) & mask) per 32 variables,
    // instead of a gather of k_info scattered posteriors and their index / bit tables per frame.
    // The workgroup's totals are summed in LDS and added to a.totals once, at exit.
    auto store = [&](int h, const uint32_t *pf, bool pre, int iters, int ok) {
        PH_T0(ph_s0);
        const int f = misc[h];
        int v0 = tid, b0 = wave * 64;  // opaque loop starts (see refill)
        asm volatile("" : "+v"(v0), "+v"(b0));
        if (a.post && !pre)
            for (int v = v0; v < n; v += NT) a.post[(size_t)f * n + v] = bias_half(pf[v], h);
        const bool masked = a.k_info > 0 && a.info_mask;
        if (kRB > 0 && (a.hard || masked)) {
            // kRB > 0: the posterior words of four ballots read together, the info masks from LDS
            uint32_t *hd = a.hard ? a.hard + (size_t)f * a.hard_words : nullptr;
            int e = 0;
            for (int base = b0; base < n; base += 4 * NT) {
                uint32_t pv[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int v = base + j * NT + lane;
                    pv[j] = v < n ? pf[v] : 0u;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int bj = base + j * NT;
                    if (bj >= n) break;
                    const unsigned long long b = __ballot(bj + lane < n && bias_half(pv[j], h) <= 0);
                    if (lane == 0) {
                        const int w = bj >> 5;
                        const bool two = w + 1 < a.hard_words;
                        if (hd) {
                            hd[w] = (uint32_t)b;
                            if (two) hd[w + 1] = (uint32_t)(b >> 32);
                        }
                        if (masked) {
                            const uint32_t *mk = lmask, *rf = lmask + a.hard_words;
                            e += __popc(((uint32_t)b ^ rf[w]) & mk[w]);
                            if (two) e += __popc(((uint32_t)(b >> 32) ^ rf[w + 1]) & mk[w + 1]);
                        }
                    }
                }
            }
            if (masked && e) atomicAdd(&misc[9 + h], e);
            PH_ADD(ph_sloop, ph_s0);
        } else if (a.hard || masked) {
            uint32_t *hd = a.hard ? a.hard + (size_t)f * a.hard_words : nullptr;
            int e = 0;
            for (int base = b0; base < n; base += NT) {
                const int v = base + lane;
                const unsigned long long b = __ballot(v < n && bias_half(pf[v], h) <= 0);
                if (lane == 0) {
                    const int w = base >> 5;
                    const bool two = w + 1 < a.hard_words;
                    if (hd) {
                        hd[w] = (uint32_t)b;
                        if (two) hd[w + 1] = (uint32_t)(b >> 32);
                    }
                    if (masked) {
                        const uint32_t *mk = a.info_mask, *rf = a.info_mask + a.hard_words;
                        e += __popc(((uint32_t)b ^ rf[w]) & mk[w]);
                        if (two) e += __popc(((uint32_t)(b >> 32) ^ rf[w + 1]) & mk[w + 1]);
                    }
                }
            }
            if (masked && e) atomicAdd(&misc[9 + h], e);
        }
        int errors = 0;
        if (a.k_info > 0) {
            if (!masked) {
                int e = 0;
                for (int i = v0; i < a.k_info; i += NT) e += ((bias_half(pf[a.info_idx[i]], h) <= 0) ? 1 : 0) != a.info_bits[i];
                if (e) atomicAdd(&misc[9 + h], e);
            }
            PK_SYNC();
            errors = misc[9 + h];
        }
        if (tid == 0) {
            if (a.iters) a.iters[f] = iters;
            if (a.syn_ok) a.syn_ok[f] = (uint8_t)ok;
            if (a.bit_errors) a.bit_errors[f] = errors;
            if (a.totals) {
                misc[kTotW] += errors;
                misc[kTotW + 1] += errors > 0;
                misc[kTotW + 2] += 1;
                misc[kTotW + 3] += iters;
            }
        }
        PH_ADD(ph_store, ph_s0);
    };

    clock_probe(a, 0);
    if (a.wgtrace) trace_t0 = __builtin_amdgcn_s_memrealtime();  // every lane: a wave-uniform (SGPR) value
    refill(3, 1, 0);
    taint[0] = misc[4] != 0;
    taint[1] = misc[5] != 0;
    // Frame ids and start steps of the two halves in (wave-uniform) registers, so the per-step
    // decisions need one LDS read (the flag word) instead of a chain of dependent ones (A +1.5 %; W
    // +13.5 % together with the final-update syndrome pass below, profiles/r4/ab/w_regctl.txt --
    // round 3's table-policy build lost 4 % with it to SGPR spills).
    int frm_r[2], sst_r[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        frm_r[h] = __builtin_amdgcn_readfirstlane(misc[h]);
        sst_r[h] = __builtin_amdgcn_readfirstlane(misc[2 + h]);
    }
    auto frm = [&](int h) { return frm_r[h]; };
    auto sst = [&](int h) { return sst_r[h]; };
    // The steps after whose barrier nothing can happen -- every live half's fail flag set (no
    // pre-check or early-termination end) and s < q_until (no half at max_iter or one short of it)
    // -- skip the end decisions: 60-odd scalar instructions per wave and step, which R's twelve
    // waves (one workgroup per CU) issue one after another on the CU's scalar unit between two
    // steps (A +2.1 %, A @ 4.5 dB +3.1 %, W +2.8 %, W @ 2 dB +2.0 %, R +1.4 %,
    // profiles/r6/ab/quick_exit.txt).  q_live: the live halves (bit h), whose fail flags must be set.
    int q_live = 0, q_until = 0;
    auto set_quick = [&]() {
        q_live = (frm(0) >= 0 ? 1 : 0) | (frm(1) >= 0 ? 2 : 0);
        q_until = 0x7fffffff;
        for (int h = 0; h < 2; ++h)
            if (frm(h) >= 0) q_until = min(q_until, sst(h) + a.max_iter - 1);
    };
    set_quick();
    int cur = 0;
    int s = 1;
    bool more = true;
    // (a half goes idle only at a refill: the tail check runs there, and once before the first step)
    bool tail = CK::kSplit && a.split_tail && (frm(0) < 0) != (frm(1) < 0);
    for (; !tail; ++s) {
        if (q_live == 0) {  // both halves idle
            clock_probe(a, 2);
            if (a.wgtrace && tid == 0) {
                unsigned long long *t = a.wgtrace + 8 * (size_t)blockIdx.x;
                t[0] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                       (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_XCC_ID, HW_REG_HW_ID
                t[1] = trace_t0;
                t[2] = __builtin_amdgcn_s_memrealtime();
                t[3] = (unsigned long long)trace_frames;
#if FPLDPC_PHASE_TRACE
                t[4] = ph_refill;
                t[5] = FPLDPC_PHASE_TRACE == 3 ? ph_rhead : FPLDPC_PHASE_TRACE == 2 ? ph_sloop : ph_pull;
                t[6] = ph_store;
                t[7] = FPLDPC_PHASE_TRACE == 3 ? ph_rload : ph_steps;
#endif
#if FPLDPC_TAIL_TRACE
                t[4] = tt_empty;
                t[5] = tt_split;
                t[6] = tt_two | tt_one << 32;
                t[7] = tt_splits;
#endif
            }
#if FPLDPC_WAIT_TRACE
            if (a.wgtrace && lane == 0) {
                unsigned long long *w = a.wgtrace + 8 * (size_t)gridDim.x + 64 * (size_t)blockIdx.x + 5 * wave;
                w[0] = wt_step;
                w[1] = wt_bar;
                w[2] = __builtin_amdgcn_s_memtime() - wt_loop0;
                w[3] = wt_steps;
                w[4] = wt_bar2;
            }
#endif
            more = false;
            break;
        }
        const uint32_t *pc = bufs + cur * n;
        uint32_t *pn = bufs + ((cur + 1) % 3) * n;
        uint32_t *pr = bufs + ((cur + 2) % 3) * n;
#if FPLDPC_WAIT_TRACE == 2
        const unsigned long long wc0 = __builtin_amdgcn_s_memtime();
#endif
        {
            int v0 = tid;  // opaque: keeps the compiler from hoisting 3 x 9 addresses across steps
            asm volatile("" : "+v"(v0));
            if (CK::kN) {
#pragma unroll
                for (int v = v0, j = 0; j < (CK::kN + NT - 1) / NT; ++j, v += NT)
                    if (j < CK::kN / NT || v < CK::kN) pr[v] = llrc[v];
            } else if ((n & 3) == 0) {  // 16-byte chunks, every buffer 16-byte aligned (W +1.3-1.4 %, W @ 2 dB +2.0 %, profiles/r6/ab/w_copy16.txt)
                const int n4 = n >> 2;
                const uint4 *l4 = reinterpret_cast<const uint4 *>(llrc);
                uint4 *p4 = reinterpret_cast<uint4 *>(pr);
                for (int vb = v0; vb < n4; vb += 2 * NT) {
                    const uint4 t0 = l4[vb];
                    uint4 t1 = {};
                    if (vb + NT < n4) t1 = l4[vb + NT];
                    p4[vb] = t0;
                    if (vb + NT < n4) p4[vb + NT] = t1;
                }
            } else {  // 8 loads in flight per thread, then 8 stores
                for (int vb = v0; vb < n; vb += 8 * NT) {
                    uint32_t t[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) t[j] = vb + j * NT < n ? llrc[vb + j * NT] : 0u;
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (vb + j * NT < n) pr[vb + j * NT] = t[j];
                }
            }
        }
#if FPLDPC_WAIT_TRACE == 2
        wt_bar2 += __builtin_amdgcn_s_memtime() - wc0;
#endif
        // flag word of step s+1: last read at step s-2, and every thread has passed the barrier of
        // step s-1 since; it is next written after this step's barrier
        if (tid == 0) {
#if FPLDPC_PHASE_TRACE
            ++ph_steps;
#endif
#if FPLDPC_TAIL_TRACE
            if (tt_empty) {
                if (frm(0) >= 0 && frm(1) >= 0) ++tt_two;
                else ++tt_one;
            }
#endif
            misc[6 + (s + 1) % 3] = 0;
            misc[12] = 0;  // flag word of a final-update syndrome pass (below), read after this step's barrier
        }
        uint32_t par = 0, ovor = 0;
        // When every frame in flight is at its last iteration (or the half is idle), this step only
        // needs the syndrome of pc: the frames end here whatever it says, so the check update into pn
        // (whose results nobody reads) is skipped -- max_iter updates per frame instead of max_iter + 1.
#if FPLDPC_WAIT_TRACE
        const unsigned long long wt0 = __builtin_amdgcn_s_memtime();
#endif
        ck.step(a, pc, pn, lds_addr(pc), lds_addr(pn), C2, M2, par, ovor);
        ovf |= ovor;
        // per-step flags: fail (syndrome) for each half, OR over the block.  The int16 range flags
        // (ovf, sticky per lane until the half is refilled) are reduced only when a frame ends,
        // below: an overflow taints every frame in flight, and no frame is stored before that check
        // (two ballots per step instead of four: W +0.6 %, R +0.3 %, A within noise; profiles/r2/ab/flags.txt).
        {
            const uint32_t bits = (par >> 15 & 1u) | (par >> 30 & 2u);
            uint32_t wb = 0;
#pragma unroll
            for (int b = 0; b < 2; ++b) wb |= __ballot((bits >> b) & 1u) ? (1u << b) : 0u;
            if (wb) atomicOr(&misc[6 + s % 3], (int)wb);  // (wave-uniform: the atomic optimizer elects one lane)
        }
#if FPLDPC_WAIT_TRACE
        const unsigned long long wt1 = __builtin_amdgcn_s_memtime();
        wt_step += wt1 - wt0;
        ++wt_steps;
#endif
        __syncthreads();
#if FPLDPC_WAIT_TRACE
        wt_bar += __builtin_amdgcn_s_memtime() - wt1;
#endif
#if FPLDPC_WAIT_TRACE == 3
        const unsigned long long wd0 = __builtin_amdgcn_s_memtime();
#endif
        uint32_t flags = (uint32_t)__builtin_amdgcn_readfirstlane(misc[6 + s % 3]);
        int finished = 0;
        if (!((flags & (uint32_t)q_live) == (uint32_t)q_live && s < q_until)) {
            // When no frame ends on pc's syndrome but every frame still running has just made its last
            // update (max_iter) into pn, check pn now (one syndrome pass after the barrier) instead of in
            // the next step's gather: a frame then costs max_iter check updates, not max_iter + 1.
            const uint32_t *pf = pc;
            int dadj = 0;
            {
                bool any = false, last = true, ends = false;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (frm(h) < 0) continue;
                    const int d = s - sst(h);
                    const bool fail = flags >> h & 1u;
                    ends = ends || (d == 0 && a.precheck && !fail) || (d >= 1 && a.early_term && !fail) || d >= a.max_iter;
                    any = true;
                    last = last && d + 1 == a.max_iter;
                }
                if (any && last && !ends) {
                    const uint32_t p2 = ck.syndrome(pn, lds_addr(pn));
                    const uint32_t b2 = (p2 >> 15 & 1u) | (p2 >> 30 & 2u);
                    uint32_t w2 = 0;
                    for (int b = 0; b < 2; ++b) w2 |= __ballot((b2 >> b) & 1u) ? (1u << b) : 0u;
                    if (lane == 0 && w2) atomicOr(&misc[12], (int)w2);
                    PK_SYNC();
                    flags = (flags & ~3u) | (uint32_t)__builtin_amdgcn_readfirstlane(misc[12]);
                    pf = pn;
                    dadj = 1;
                }
            }
            int ending = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (frm(h) < 0) continue;
                const int d = s - sst(h) + dadj;
                const bool fail = flags >> h & 1u;
                if ((d == 0 && a.precheck && !fail) || (d >= 1 && a.early_term && !fail) || d >= a.max_iter) ending |= 1 << h;
            }
            if (ending) {
                // the deferred int16 range check: a c2v at or above 2^b (a.cmax = 2^b - 1) in either half
                // since that half's refill corrupts both halves' posterior words, so it taints every
                // frame in flight (misc[13] is cleared again by the refill that follows)
                const uint32_t hi_bits = ~(a.cmax * 0x10001u);
                if (__ballot((ovf & hi_bits) != 0u) && lane == 0) atomicOr(&misc[13], 1);
                PK_SYNC();
                if (__builtin_amdgcn_readfirstlane(misc[13])) {
                    taint[0] = taint[0] || frm(0) >= 0;
                    taint[1] = taint[1] || frm(1) >= 0;
                }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (!(ending >> h & 1)) continue;
                const int d = s - sst(h) + dadj;  // completed updates in pf for this frame
                const bool fail = flags >> h & 1u;
                const bool pre = d == 0 && a.precheck && !fail;
                finished |= 1 << h;
                if (taint[h]) {
                    if (tid == 0) a.fb_list[atomicAdd(a.fb_count, 1)] = frm(h);
                } else {
                    store(h, pre ? llrc : pf, pre, pre ? 0 : d, pre ? 1 : !fail);
                }
            }
        }
        cur = (cur + 1) % 3;
        if (finished) {
            refill(finished, s + 1, cur);
            // the refilled half starts from zero c2v state and a fresh range tracker
            const uint32_t keep = (finished & 1 ? 0xffff0000u : 0xffffffffu) & (finished & 2 ? 0x0000ffffu : 0xffffffffu);
            ck.clear(finished);
            ovf &= keep;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (finished >> h & 1) taint[h] = misc[4 + h] != 0;
                frm_r[h] = __builtin_amdgcn_readfirstlane(misc[h]);
                sst_r[h] = __builtin_amdgcn_readfirstlane(misc[2 + h]);
            }
            if constexpr (CK::kSplit) tail = a.split_tail && (frm(0) < 0) != (frm(1) < 0);
            set_quick();
        }
#if FPLDPC_WAIT_TRACE == 3
        wt_bar2 += __builtin_amdgcn_s_memtime() - wd0;
#endif
    }
    // (the split loop's step)
    auto step_body = [&](int s, auto split_c) -> bool {
        constexpr bool SPLIT = decltype(split_c)::value;
        if (frm(0) < 0 && frm(1) < 0) {
            clock_probe(a, 2);
            if (a.wgtrace && tid == 0) {
                unsigned long long *t = a.wgtrace + 8 * (size_t)blockIdx.x;
                t[0] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                       (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_XCC_ID, HW_REG_HW_ID
                t[1] = trace_t0;
                t[2] = __builtin_amdgcn_s_memrealtime();
                t[3] = (unsigned long long)trace_frames;
#if FPLDPC_PHASE_TRACE
                t[4] = ph_refill;
                t[5] = FPLDPC_PHASE_TRACE == 3 ? ph_rhead : FPLDPC_PHASE_TRACE == 2 ? ph_sloop : ph_pull;
                t[6] = ph_store;
                t[7] = FPLDPC_PHASE_TRACE == 3 ? ph_rload : ph_steps;
#endif
#if FPLDPC_TAIL_TRACE
                t[4] = tt_empty;
                t[5] = tt_split;
                t[6] = tt_two | tt_one << 32;
                t[7] = tt_splits;
#endif
            }
            return false;
        }
        const uint32_t *pc = bufs + cur * n;
        uint32_t *pn = bufs + ((cur + 1) % 3) * n;
        uint32_t *pr = bufs + ((cur + 2) % 3) * n;
        {
            int v0 = tid;  // opaque: keeps the compiler from hoisting 3 x 9 addresses across steps
            asm volatile("" : "+v"(v0));
            if (CK::kN) {
#pragma unroll
                for (int v = v0, j = 0; j < (CK::kN + NT - 1) / NT; ++j, v += NT)
                    if (j < CK::kN / NT || v < CK::kN) pr[v] = llrc[v];
            } else if ((n & 3) == 0) {  // 16-byte chunks, every buffer 16-byte aligned (W +1.3-1.4 %, W @ 2 dB +2.0 %, profiles/r6/ab/w_copy16.txt)
                const int n4 = n >> 2;
                const uint4 *l4 = reinterpret_cast<const uint4 *>(llrc);
                uint4 *p4 = reinterpret_cast<uint4 *>(pr);
                for (int vb = v0; vb < n4; vb += 2 * NT) {
                    const uint4 t0 = l4[vb];
                    uint4 t1 = {};
                    if (vb + NT < n4) t1 = l4[vb + NT];
                    p4[vb] = t0;
                    if (vb + NT < n4) p4[vb + NT] = t1;
                }
            } else {  // 8 loads in flight per thread, then 8 stores
                for (int vb = v0; vb < n; vb += 8 * NT) {
                    uint32_t t[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) t[j] = vb + j * NT < n ? llrc[vb + j * NT] : 0u;
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (vb + j * NT < n) pr[vb + j * NT] = t[j];
                }
            }
        }
        // flag word of step s+1: last read at step s-2, and every thread has passed the barrier of
        // step s-1 since; it is next written after this step's barrier
        if (tid == 0) {
#if FPLDPC_PHASE_TRACE
            ++ph_steps;
#endif
#if FPLDPC_TAIL_TRACE
            ++tt_splits;
#endif
            misc[6 + (s + 1) % 3] = 0;
            misc[12] = 0;  // flag word of a final-update syndrome pass (below), read after this step's barrier
        }
        uint32_t par = 0, ovor = 0;
        // When every frame in flight is at its last iteration (or the half is idle), this step only
        // needs the syndrome of pc: the frames end here whatever it says, so the check update into pn
        // (whose results nobody reads) is skipped -- max_iter updates per frame instead of max_iter + 1.
        if constexpr (SPLIT)
            split_step_of(ck, pc, pn, lds_addr(pc), lds_addr(pn), C2, M2, par, ovor);
        else
            ck.step(a, pc, pn, lds_addr(pc), lds_addr(pn), C2, M2, par, ovor);
        ovf |= ovor;
        // per-step flags: fail (syndrome) for each half, OR over the block.  The int16 range flags
        // (ovf, sticky per lane until the half is refilled) are reduced only when a frame ends,
        // below: an overflow taints every frame in flight, and no frame is stored before that check
        // (two ballots per step instead of four: W +0.6 %, R +0.3 %, A within noise; profiles/r2/ab/flags.txt).
        {
            const uint32_t bits = (par >> 15 & 1u) | (par >> 30 & 2u);
            uint32_t wb = 0;
#pragma unroll
            for (int b = 0; b < 2; ++b) wb |= __ballot((bits >> b) & 1u) ? (1u << b) : 0u;
            if (lane == 0 && wb) atomicOr(&misc[6 + s % 3], (int)wb);
        }
        __syncthreads();
        uint32_t flags = (uint32_t)__builtin_amdgcn_readfirstlane(misc[6 + s % 3]);
        {  // the packed loop's quick exit (from the control words: q_live / q_until are the packed loop's)
            bool q = true;
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (frm(h) >= 0) q = q && (flags >> h & 1u) && s < sst(h) + a.max_iter - 1;
            if (q) {
                cur = (cur + 1) % 3;
                return true;
            }
        }
        // When no frame ends on pc's syndrome but every frame still running has just made its last
        // update (max_iter) into pn, check pn now (one syndrome pass after the barrier) instead of in
        // the next step's gather: a frame then costs max_iter check updates, not max_iter + 1.
        const uint32_t *pf = pc;
        int dadj = 0;
        {
            bool any = false, last = true, ends = false;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (frm(h) < 0) continue;
                const int d = s - sst(h);
                const bool fail = flags >> h & 1u;
                ends = ends || (d == 0 && a.precheck && !fail) || (d >= 1 && a.early_term && !fail) || d >= a.max_iter;
                any = true;
                last = last && d + 1 == a.max_iter;
            }
            if (any && last && !ends) {
                const uint32_t p2 = ck.syndrome(pn, lds_addr(pn));
                const uint32_t b2 = (p2 >> 15 & 1u) | (p2 >> 30 & 2u);
                uint32_t w2 = 0;
                for (int b = 0; b < 2; ++b) w2 |= __ballot((b2 >> b) & 1u) ? (1u << b) : 0u;
                if (lane == 0 && w2) atomicOr(&misc[12], (int)w2);
                __syncthreads();
                flags = (flags & ~3u) | (uint32_t)__builtin_amdgcn_readfirstlane(misc[12]);
                pf = pn;
                dadj = 1;
            }
        }
        int ending = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (frm(h) < 0) continue;
            const int d = s - sst(h) + dadj;
            const bool fail = flags >> h & 1u;
            if ((d == 0 && a.precheck && !fail) || (d >= 1 && a.early_term && !fail) || d >= a.max_iter) ending |= 1 << h;
        }
        if (ending) {
            // the deferred int16 range check: a c2v at or above 2^b (a.cmax = 2^b - 1) in either half
            // since that half's refill corrupts both halves' posterior words, so it taints every
            // frame in flight (misc[13] is cleared again by the refill that follows)
            const uint32_t hi_bits = ~(a.cmax * 0x10001u);
            if (__ballot((ovf & hi_bits) != 0u) && lane == 0) atomicOr(&misc[13], 1);
            __syncthreads();
            if (__builtin_amdgcn_readfirstlane(misc[13])) {
                taint[0] = taint[0] || frm(0) >= 0;
                taint[1] = taint[1] || frm(1) >= 0;
            }
        }
        int finished = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (!(ending >> h & 1)) continue;
            const int d = s - sst(h) + dadj;  // completed updates in pf for this frame
            const bool fail = flags >> h & 1u;
            const bool pre = d == 0 && a.precheck && !fail;
            finished |= 1 << h;
            if (taint[h]) {
                if (tid == 0) a.fb_list[atomicAdd(a.fb_count, 1)] = frm(h);
            } else {
                store(h, pre ? llrc : pf, pre, pre ? 0 : d, pre ? 1 : !fail);
            }
        }
        cur = (cur + 1) % 3;
        if (finished) {
            refill(finished, s + 1, cur);
            // the refilled half starts from zero c2v state and a fresh range tracker.  (In the split
            // form the queue is empty -- a half goes idle only when a pull finds it so -- and this
            // refill finds no frame: the workgroup ends.)
            const uint32_t keep = (finished & 1 ? 0xffff0000u : 0xffffffffu) & (finished & 2 ? 0x0000ffffu : 0xffffffffu);
            ck.clear(finished);
            ovf &= keep;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (finished >> h & 1) taint[h] = misc[4 + h] != 0;
                frm_r[h] = __builtin_amdgcn_readfirstlane(misc[h]);
                sst_r[h] = __builtin_amdgcn_readfirstlane(misc[2 + h]);
            }
        }
        return true;
    };
    if constexpr (CK::kSplit) {
        if (more) {
            // The tail: this frame continues in half 0 of the LDS words with its check split over the
            // lane halves (ArrayChecks::split_step, about 55 % of the packed step's instructions), so
            // the frames the launch waits on at its end run at a shorter step latency.  A frame in half
            // 1 is moved to half 0 first: posterior, next-posterior and LLR words rotated, its control
            // words swapped.
            const int h = frm(0) < 0 ? 1 : 0;
            if (h) {
                for (int v = tid; v < 4 * n; v += NT) bufs[v] = CK::rot16(bufs[v]);
                if (tid == 0) {
                    for (int i : {0, 2, 4, 9}) {
                        const int t = misc[i];
                        misc[i] = misc[i + 1];
                        misc[i + 1] = t;
                    }
                }
                const int f0 = frm_r[0], s0 = sst_r[0];
                const bool t0 = taint[0];
                frm_r[0] = frm_r[1];
                sst_r[0] = sst_r[1];
                taint[0] = taint[1];
                frm_r[1] = f0;
                sst_r[1] = s0;
                taint[1] = t0;
                ovf >>= 16;
            } else {
                ovf &= 0xffffu;
            }
            ck.split_enter(h);
#if FPLDPC_TAIL_TRACE
            if (tid == 0) tt_split = __builtin_amdgcn_s_memrealtime();
#endif
            __syncthreads();
            for (;; ++s)
                if (!step_body(s, std::true_type{})) break;
        }
    }
    if (a.totals && tid == 0) {  // this workgroup's frames (each counter < 2^31 per workgroup)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (misc[kTotW + c]) atomicAdd(&a.totals[c], (unsigned long long)(unsigned)misc[kTotW + c]);
    }
    chain_exit(a);
}

// ------------------------------------------------------------------------------------------
// LDS-state kernel for array codes whose c2v state does not fit registers (p47/r24: 1128 checks x
// 47 edges).  One frame per 1024-thread workgroup; each lane owns check tid and, for m > 1024,
// check tid + 1024.  The c2v state lives in LDS as int16 ([check][slot]); the
// posteriors stay int32.  Magnitude chains use 16-bit min (full rate on gfx950) and 32-bit
// add/sub/shift/and.  Exact while every |v2c| < 2^14 (then every chain value, a + b and c2v fit
// 16 bits); a frame that leaves that range stops and is re-decoded by the int32 kernel.
constexpr int kNT16 = 1024;  // 16 waves: 4 per SIMD (checks tid, tid + 1024)

__device__ __forceinline__ uint32_t bp_mag16(uint32_t a, uint32_t b, unsigned short C, uint32_t M) {
    const uint32_t mn = __builtin_elementwise_min((unsigned short)a, (unsigned short)b);
    const uint32_t s = a + b;
    const uint32_t d = sub2x(s, mn);  // max - min
    const uint32_t q1 = __builtin_elementwise_min((unsigned short)((s >> 2) & M), C);
    const uint32_t q2 = __builtin_elementwise_min((unsigned short)((d >> 2) & M), C);
    return mn + q2 - q1;
}

// Edge k of a check in the LDS-state kernel: posterior p (int32 LDS) and stored c2v (int16 LDS)
// give v2c m = p - c2v (:143-152); returns |m| and folds the flags into S (sign parity, bit 31 of
// the XOR) and par (hard-decision parity, bit 31: post <= 0, :305-308).
__device__ __forceinline__ uint32_t edge16(const char *pcb, unsigned short t4, int koff, int c2v, uint32_t &S,
                                           uint32_t &par, uint32_t &ovor) {
    const int p = *reinterpret_cast<const int *>(pcb + koff + t4);
    par ^= (uint32_t)(p - 1);
    const int mm = p - c2v;
    const uint32_t sg = (uint32_t)(mm >> 31);
    const uint32_t av = ((uint32_t)mm ^ sg) - sg;
    ovor |= av;
    S ^= sg;
    return av;
}

// c2v = sign * o (sign in bit 31 of sb) into the next posterior and the check's state
__device__ __forceinline__ void put16(char *pn_addr, int16_t *st, uint32_t o, uint32_t sb) {
    const uint32_t nm = 0u - (sb >> 31);
    const int v = (int)((o ^ nm) - nm);
    lds_add(reinterpret_cast<int *>(pn_addr), v);
    *st = (int16_t)v;
}

__device__ __forceinline__ unsigned short wrap_up(unsigned short t, unsigned short step, unsigned short wrap) {
    t = (unsigned short)(t + step);
    return __builtin_elementwise_min(t, (unsigned short)(t - wrap));
}
__device__ __forceinline__ unsigned short wrap_down(unsigned short t, unsigned short step, unsigned short wrap) {
    t = (unsigned short)(t - step);
    return __builtin_elementwise_min(t, (unsigned short)(t + wrap));
}

// One check of the LDS-state kernel; returns the syndrome parity of pc over the check.  Nothing per
// edge is kept in registers across the two passes: pass 1 reads every edge once (building the
// middle-out chains F_0..F_{L-1}, B_{L+1}..B_{P-1} and the parities), pass 2 re-reads each edge
// (LDS is cheap next to VGPRs here) to extend the chains and emit c2v_k = F_{k-1} [+] B_{k+1}.
// Compiler-only fence between the steps of check_lds16's passes: keeps the scheduler from hoisting
// every edge load of a pass to its top (2 x 47 live VGPRs -> spills / fewer resident waves).
__device__ __forceinline__ void lds16_step_fence() { asm volatile("" ::: "memory"); }

template <int P>
__device__ __forceinline__ int check_lds16(int c, const int *pc, int *pn, int16_t *st16, bool update,
                                           unsigned short C, uint32_t M, uint32_t &ovor) {
    constexpr int L = (P - 1) / 2;
    const unsigned short row = (unsigned short)(c / P), col = (unsigned short)(c % P);
    const unsigned short step4 = (unsigned short)(4 * row), wrap4 = (unsigned short)(4 * P);
    const char *pcb = reinterpret_cast<const char *>(pc);
    int16_t *const stc = st16 + c * P;  // this check's c2v state ([check][slot]: constant offsets)
    uint32_t par = 0, S = 0, dummy = 0;
    // byte offsets (within a block column) of slot 0 and slot P-1: (col + row*k) mod P
    unsigned short tl = (unsigned short)(4 * col);
    unsigned short tr = (unsigned short)(4 * ((col + (uint32_t)row * (P - 1)) % P));
    asm volatile("" : "+v"(tl), "+v"(tr));
    uint32_t FB[P];
    FB[0] = edge16(pcb, tl, 0, stc[0], S, par, ovor);
    FB[P - 1] = edge16(pcb, tr, (P - 1) * P * 4, stc[P - 1], S, par, ovor);
#pragma unroll
    for (int j = 1; j < P - 1 - L; ++j) {
        lds16_step_fence();
        if (j < L) {
            tl = wrap_up(tl, step4, wrap4);
            FB[j] = bp_mag16(FB[j - 1], edge16(pcb, tl, j * P * 4, stc[j], S, par, ovor), C, M);
        }
        tr = wrap_down(tr, step4, wrap4);
        FB[P - 1 - j] = bp_mag16(FB[P - j], edge16(pcb, tr, (P - 1 - j) * P * 4, stc[P - 1 - j], S, par, ovor), C, M);
        // fold the flags now: left to itself the compiler sinks the par / ovor / S chains past pass 2
        // and keeps all 2 x 47 posteriors and magnitudes live (93 VGPRs of spills at 1024 threads)
        asm volatile("" : "+v"(par), "+v"(ovor), "+v"(S));
    }
    tl = wrap_up(tl, step4, wrap4);  // slot L
    const unsigned short tL = tl;
    const uint32_t aL = edge16(pcb, tL, L * P * 4, stc[L], S, par, ovor);
    if (!update) return (int)(par >> 31);
    // memory clobber: pass 2 re-reads the LDS state instead of the compiler keeping the 47 values
    // of pass 1 live in registers
    asm volatile("" ::: "memory");
    // pass 2: outputs from the middle outwards; the sign of c2v_k is S ^ sign(m_k)
    char *pnb = reinterpret_cast<char *>(pn);
    uint32_t F, B;
    {
        uint32_t S2 = 0;
        const int p = *reinterpret_cast<const int *>(pcb + L * P * 4 + tL);
        S2 = (uint32_t)((p - (int)stc[L]) >> 31);
        const uint32_t o = bp_mag16(FB[L - 1], FB[L + 1], C, M);
        F = bp_mag16(FB[L - 1], aL, C, M);
        B = bp_mag16(FB[L + 1], aL, C, M);
        put16(pnb + L * P * 4 + tL, stc + L, o, S ^ S2);
    }
    unsigned short uf = tL, ub = tL;
#pragma unroll
    for (int j = 1; j <= (L > P - 1 - L ? L : P - 1 - L); ++j) {
        const int kf = L + j, kb = L - j;
        lds16_step_fence();
        if (kf <= P - 1) {
            uf = wrap_up(uf, step4, wrap4);
            uint32_t sgk = 0;
            const uint32_t ak = edge16(pcb, uf, kf * P * 4, stc[kf], sgk, dummy, dummy);
            uint32_t o = F;  // c2v_{P-1} = F_{P-2}
            if (kf <= P - 2) {
                o = bp_mag16(F, FB[kf + 1], C, M);
                F = bp_mag16(F, ak, C, M);
            }
            put16(pnb + kf * P * 4 + uf, stc + kf, o, S ^ sgk);
        }
        if (kb >= 0) {
            ub = wrap_down(ub, step4, wrap4);
            uint32_t sgk = 0;
            const uint32_t ak = edge16(pcb, ub, kb * P * 4, stc[kb], sgk, dummy, dummy);
            uint32_t o = B;  // c2v_0 = B_1
            if (kb >= 1) {
                o = bp_mag16(FB[kb - 1], B, C, M);
                B = bp_mag16(B, ak, C, M);
            }
            put16(pnb + kb * P * 4 + ub, stc + kb, o, S ^ sgk);
        }
    }
    return (int)(par >> 31);
}

template <int P, int NT = kNT16>
__global__ void __launch_bounds__(NT, NT / 256) flood_lds16(KArgs a) {
    if (empty_list(a)) return;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    constexpr int n = P * P;
    int *const bufs = smem;
    int *const llr_s = smem + 3 * n;
    int *const misc = smem + 4 * n;  // [0] frame [1] bit errors [2..4] flag words
    int16_t *const st16 = reinterpret_cast<int16_t *>(smem + 4 * n + 16);
    const int tid = threadIdx.x, m = a.m;
    const unsigned short C = (unsigned short)a.C;
    const uint32_t M = (1u << a.bfe_w) - 1u;

    for (;;) {
        __syncthreads();
        if (tid == 0) {
            misc[0] = pull_frame(a, a.work_counter);
            misc[1] = 0;
            misc[2] = misc[3] = misc[4] = 0;
        }
        __syncthreads();
        const int cw = misc[0];
        if (cw < 0) break;
        frame_load<NT>(a, cw, bufs, llr_s);
        for (int e = tid; e < m * P; e += NT) st16[e] = 0;
        __syncthreads();
        int cur = 0;
        const int *pf = nullptr;
        bool pre = false, taint = false;
        int iters = 0, ok = 0;
        for (int it = 1;; ++it) {
            const bool update = it <= a.max_iter;
            const int *pc = bufs + cur * n;
            int *pn = bufs + ((cur + 1) % 3) * n;
            int *pr = bufs + ((cur + 2) % 3) * n;
            if (update)
                for (int v = tid; v < n; v += NT) pr[v] = llr_s[v];
            if (tid == 0) misc[2 + (it + 1) % 3] = 0;  // flag word of step it+1 (see flood_array2)
            int fail = 0;
            uint32_t ovor = 0;
            for (int c = tid; c < m; c += NT) fail |= check_lds16<P>(c, pc, pn, st16, update, C, M, ovor);
            {
                const uint32_t bits = (uint32_t)fail | (ovor >= (1u << 14) ? 2u : 0u);
                uint32_t wb = (__ballot(bits & 1u) ? 1u : 0u) | (__ballot(bits & 2u) ? 2u : 0u);
                if ((tid & 63) == 0 && wb) atomicOr(&misc[2 + it % 3], (int)wb);
            }
            __syncthreads();
            const int flags = misc[2 + it % 3];
            if (flags & 2) {  // left the exact 16-bit range: hand the frame to the int32 kernel
                taint = true;
                break;
            }
            fail = flags & 1;
            const int done = it - 1;
            if (done == 0 && a.precheck && !fail) {
                pf = llr_s;
                pre = true;
                iters = 0;
                ok = 1;
                break;
            }
            if ((done >= 1 && a.early_term && !fail) || done >= a.max_iter) {
                pf = pc;
                iters = done;
                ok = !fail;
                break;
            }
            cur = (cur + 1) % 3;
        }
        if (taint) {
            if (tid == 0) a.fb_list[atomicAdd(a.fb_count, 1)] = cw;
            continue;
        }
        frame_store<NT>(a, cw, pf, !pre, iters, ok, misc);
    }
    chain_exit(a);
}

typedef void (*KernelFn)(KArgs);

#if FPLDPC_TU_ARRAY1 || FPLDPC_TU_TABLE1
}  // namespace

#if FPLDPC_TU_ARRAY1
// fpldpc_kernels_a1.hip: this file with FPLDPC_TU_ARRAY1 = 1 holds the packed 47-slot array kernel
// (the A configuration's, flood_pk<ArrayChecks<47>, 3>) and nothing else, compiled with the post-RA
// machine scheduler off (_build.py SOURCE_FLAGS): +3.3 % on A at 0 dB and +3.8 % at 4.5 dB, while the
// other packed kernels lose 1-5 % without it (profiles/r5/ab/post_ra.txt).  The main translation unit
// takes the kernel's host stub from here, so launches and occupancy queries reach this code object.
// (const void *: KArgs lives in each translation unit's unnamed namespace)
const void *array47_pair_kernel() { return reinterpret_cast<const void *>(&flood_pk<ArrayChecks<47>, 3>); }
#else
// fpldpc_kernels_w1.hip: this file with FPLDPC_TU_TABLE1 = 1 holds the degree-sorted packed table
// kernel (the W configuration's, flood_pk<TableChecks<8, 4, 7, 3>, 4>) and nothing else, so that it
// too gets code-generation options of its own (_build.py SOURCE_FLAGS).
const void *table8_pair_kernel() { return reinterpret_cast<const void *>(&flood_pk<TableChecks<8, 4, 7, 3>, 4>); }
#endif

}  // namespace fpldpc
#else
}  // namespace
// the A and W kernels' host stubs (fpldpc_kernels_a1.hip, fpldpc_kernels_w1.hip, compiled separately)
const void *array47_pair_kernel();
const void *table8_pair_kernel();
namespace {

struct VariantInfo {
    Variant v;
    KernelFn fn;
    int dc;       // kernel DC
    int max_m;    // 0 = any
    bool regular; // requires every check degree == dc
    bool gmem;
    const char *name;
    int array_p = 0;  // > 0: forward array code with this p only (computed addressing)
    bool low_mask = false;  // width_mask must be 2^w - 1 (bit-field extract)
    Variant fallback = Variant::kNone;  // int32 kernel re-decoding frames the packed kernel rejects
    int nt = kNT;           // threads per workgroup
    bool lds_state = false; // c2v state in LDS (int16 [dc][m])
    int dmin = 2;           // smallest check degree the variant handles
    int tab_words = 0;      // LDS table words per check after the control words (array LDS offsets)
    int lo_passes = 0;      // > 0: checks listed by ascending degree, the first lo_passes * nt of degree dmin
};

size_t variant_lds(const VariantInfo &x, const fpldpc_code &c) {
    size_t b = (size_t)(4 * c.n + kMiscInts) * sizeof(int);
    if (x.lds_state) b += (size_t)c.m * x.dc * sizeof(int16_t);
    b += (size_t)c.m * x.tab_words * sizeof(uint32_t);
    b += 2 * (size_t)((c.n + 31) / 32) * sizeof(uint32_t);  // flood_pk: the info masks staged in LDS
    return b;
}

const VariantInfo kVariants[] = {
    {Variant::kArray47x2, reinterpret_cast<KernelFn>(const_cast<void *>(array47_pair_kernel())), 47, kNT, true, false, "flood_array2<P=47,W=3>", 47, true, Variant::kArray47},
    // array codes with up to 1536 checks (R: 1128): 2 checks per lane in one 768-thread workgroup,
    // 3 waves / SIMD (168 VGPRs; the few spills sit in the per-step control code, not in the check
    // update).  SIMD loads 5 / 5 / 4 / 4 check-units per step, as with 3 checks per lane at 2 waves
    // / SIMD, which measured 8.7 % slower (profiles/r2/ab/r_cpl.txt).  int16 range misses go to the
    // LDS-state kernel and from there to the global one.
    // the same with the slot offsets in an LDS table (143 KB of LDS with R's): no offset walking
    // R (since round 3): 2 checks per lane up to check 1024, the rest two lanes per check -- 4.5
    // units on every SIMD instead of 5 / 5 / 4 / 4 (+8.6 %, profiles/r3/ab/r_mix.txt)
    {Variant::kArray47x2mix, flood_pk<MixChecks<47>, 1, 768>, 47, 768 + 256 + 128, true, false,
     "flood_array2<P=47,CPL=2,ldsoffs,mix>", 47, true, Variant::kLds16_47, 768, false, 2, MixChecks<47>::kTabWords},
    {Variant::kArray47x2c2t, flood_pk<ArrayChecks<47, 2, 768, true, true>, 1, 768>, 47, 2 * 768, true, false,
     "flood_array2<P=47,CPL=2,ldsoffs>", 47, true, Variant::kLds16_47, 768, false, 2, ArrayChecks<47, 2, 768, true, true>::kTabWords},
    {Variant::kArray47x2c2, flood_pk<ArrayChecks<47, 2, 768>, 1, 768>, 47, 2 * 768, true, false,
     "flood_array2<P=47,CPL=2>", 47, true, Variant::kLds16_47, 768},
    {Variant::kArray47, flood_array<47>, 47, kNT, true, false, "flood_array<P=47>", 47, true},
    // degrees 7..8 with at least 768 checks of degree 7 (W: 810 of 972): passes 0-2 fold 7 slots
    {Variant::kTab8x4lo3, reinterpret_cast<KernelFn>(const_cast<void *>(table8_pair_kernel())), 8, 4 * kNT, false, false,
     "flood_tab2<DC=8,CPL=4,lo=3>", 0, true, Variant::kReg8x4, kNT, false, 7, 0, 3},
    {Variant::kTab8x4p, flood_pk<TableChecks<8, 4, 7>, 4>, 8, 4 * kNT, false, false, "flood_tab2<DC=8,CPL=4>", 0, true,
     Variant::kReg8x4, kNT, false, 7},
    {Variant::kLds16_47, flood_lds16<47>, 47, 2 * kNT16, true, false, "flood_lds16<P=47>", 47, true, Variant::kGmem48,
     kNT16, true},
    {Variant::kReg47x1Regular, flood_reg<47, 1, true>, 47, kNT, true, false, "flood_reg<DC=47,CPL=1,regular>"},
    {Variant::kReg8x1, flood_reg<8, 1, false>, 8, kNT, false, false, "flood_reg<DC=8,CPL=1>"},
    {Variant::kReg8x4, flood_reg<8, 4, false>, 8, 4 * kNT, false, false, "flood_reg<DC=8,CPL=4>"},
    {Variant::kReg16x2, flood_reg<16, 2, false>, 16, 2 * kNT, false, false, "flood_reg<DC=16,CPL=2>"},
    {Variant::kGmem8, flood_gmem<8>, 8, 0, false, true, "flood_gmem<DC=8>"},
    {Variant::kGmem16, flood_gmem<16>, 16, 0, false, true, "flood_gmem<DC=16>"},
    {Variant::kGmem32, flood_gmem<32>, 32, 0, false, true, "flood_gmem<DC=32>"},
    {Variant::kGmem48, flood_gmem<48>, 48, 0, false, true, "flood_gmem<DC=48>"},
    {Variant::kGmem64, flood_gmem<64>, 64, 0, false, true, "flood_gmem<DC=64>"},
};

const VariantInfo *find_variant(Variant v) {
    for (const auto &x : kVariants)
        if (x.v == v) return &x;
    return nullptr;
}

}  // namespace

int fail_hip(int hip_status, const char *what) {
    return fail(FPLDPC_ERR_HIP, std::string(what) + ": " + hipGetErrorString((hipError_t)hip_status));
}

int kernel_dc(Variant v) {
    const VariantInfo *vi = find_variant(v);
    return vi ? vi->dc : 0;
}

// int16 range of the packed kernels: with |LLR| <= kLlrMax and every c2v magnitude <= cm, |post| <=
// kLlrMax + dv*cm and |v2c| <= kLlrMax + (dv+1)*cm; a box-plus chain value is at most its last v2c
// input + C (bp_mag <= min + C: the WIDTH_MASK wrap can make part1 exceed part2), so every chain value
// stays below 2^15 -- magnitudes keep bit 15 clear and a + b never carries out of a 16-bit half -- when
// kLlrMax + (dv+1)*cm + max(64, C) <= 32767.  Returns the largest such cm = 2^b - 1, or 0 when not even
// cm = 1 fits (C = 5/8 * 2^FRAC_WIDTH, ArrayLDPCMacro.h:175: FRAC_WIDTH >= 16 on any code).
uint32_t packed_cmax(const fpldpc_code &code, int C) {
    const uint64_t margin = (uint64_t)std::max(64, C);
    auto fits = [&](uint64_t cm) { return (uint64_t)kLlrMax + (uint64_t)(code.dv_max + 1) * cm + margin <= 32767; };
    if (!fits(1)) return 0;
    uint32_t cm = 1;
    while (fits(2 * (uint64_t)cm + 1)) cm = 2 * cm + 1;
    return cm;
}

// flood_lds16 is exact while |v2c| < 2^14 (checked per step): its chain values and c2v are then at
// most 2^14 - 1 + C, which its u16 minima and int16 c2v state hold while C <= 2^14 (FRAC_WIDTH <= 14).
constexpr int kLds16MaxC = 1 << 14;

int choose_kernel(const fpldpc_code &code, int device, int mask, int C, KernelChoice *out) {
    const bool low_mask = mask >= 3 && (mask & (mask + 1)) == 0;
    const uint32_t cmax = packed_cmax(code, C);
    // an int16 kernel, or a chain that hands frames down to one, is exact at this C
    auto int16_ok = [&](const VariantInfo &x) {
        for (const VariantInfo *y = &x; y; y = y->fallback == Variant::kNone ? nullptr : find_variant(y->fallback))
            if (y->lds_state && C > kLds16MaxC) return false;
        return x.fallback == Variant::kNone || x.lds_state || cmax > 0;
    };
    for (int r = 0; r < code.m; r++)
        if (code.cdeg[r] < 2) return fail(FPLDPC_ERR_UNSUPPORTED, "check of degree < 2 (reference behaviour undefined)");
    if (code.dc_max > 64) return fail(FPLDPC_ERR_UNSUPPORTED, "check degree above 64");
    if ((size_t)(4 * code.n + kMiscInts) * sizeof(int) > 160 * 1024)
        return fail(FPLDPC_ERR_UNSUPPORTED, "code length too large for LDS-resident posteriors");
    // The reference iterates its checks in block order and folds each in clist order; the kernel
    // folds in clist order per check, so only the degree envelope matters for the choice.
    int actual_dc = 0;
    for (int r = 0; r < code.m; r++) actual_dc = std::max(actual_dc, (int)code.cdeg[r]);
    bool regular = true;
    int min_dc = actual_dc;
    for (int r = 0; r < code.m; r++) {
        regular &= code.cdeg[r] == actual_dc;
        min_dc = std::min(min_dc, (int)code.cdeg[r]);
    }
    int n_min_dc = 0;  // checks of the smallest degree (listed first when a variant sorts them)
    for (int r = 0; r < code.m; r++) n_min_dc += code.cdeg[r] == min_dc;
    const VariantInfo *pick = nullptr;
    // FPLDPC_KERNEL=<name prefix> forces a variant (A/B measurements); it must still fit the code
    const char *force = getenv("FPLDPC_KERNEL");
    for (const auto &x : kVariants) {
        if (force && *force && strncmp(x.name, force, strlen(force)) != 0) continue;
        if (x.gmem) continue;
        if (x.array_p && !(code.array_p == x.array_p && code.array_forward)) continue;
        if (x.low_mask && !low_mask) continue;
        if (x.fallback != Variant::kNone && mask > 0xffff) continue;  // packed halves: mask within 16 bits
        if (!int16_ok(x)) continue;
        if (variant_lds(x, code) > 160 * 1024) continue;
        if (min_dc < x.dmin) continue;
        if (x.regular ? !(regular && actual_dc == x.dc) : actual_dc > x.dc) continue;
        if (code.m > x.max_m) continue;
        if (x.lo_passes && !(min_dc == x.dmin && n_min_dc >= x.lo_passes * x.nt)) continue;
        pick = &x;
        break;
    }
    if (!pick)
        for (const auto &x : kVariants)
            if (x.gmem && actual_dc <= x.dc && !(force && *force && strncmp(x.name, force, strlen(force)) != 0)) {
                pick = &x;
                break;
            }
    if (!pick) return fail(FPLDPC_ERR_UNSUPPORTED, "no kernel variant for this code");
    const size_t lds = variant_lds(*pick, code);
    int dev = device;
    if (dev < 0) {
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return fail_hip(e, "hipGetDevice");
    }
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return fail_hip(e, "hipGetDeviceProperties");
    if (lds > 64 * 1024) {
        e = hipFuncSetAttribute((const void *)pick->fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return fail_hip(e, "hipFuncSetAttribute");
    }
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pick->fn, pick->nt, lds);
    if (e != hipSuccess) return fail_hip(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    if (per_cu < 1) return fail(FPLDPC_ERR_UNSUPPORTED, "kernel cannot be resident (occupancy 0)");
    // Diagnostic: FPLDPC_GRID_PER_CU=k caps the persistent grid at k workgroups per CU (A/B runs)
    if (const char *g = getenv("FPLDPC_GRID_PER_CU"))
        if (atoi(g) > 0) per_cu = std::min(per_cu, atoi(g));
    out->v = pick->v;
    out->threads = pick->nt;
    out->grid = per_cu * prop.multiProcessorCount;
    out->fallback = pick->fallback;
    const int m_pad = (code.m + 63) / 64 * 64;
    out->scratch_ints = pick->gmem ? (size_t)out->grid * pick->dc * m_pad : 0;
    // a fallback kernel: rare work, so one workgroup per CU is plenty and exits fast when empty
    auto setup_fallback = [&](Variant v, int *grid, int *threads, size_t *lds_out) -> int {
        const VariantInfo *fb = find_variant(v);
        const size_t fb_lds = variant_lds(*fb, code);
        if (fb_lds > 64 * 1024) {
            e = hipFuncSetAttribute((const void *)fb->fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fb_lds);
            if (e != hipSuccess) return fail_hip(e, "hipFuncSetAttribute");
        }
        int fb_cu = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&fb_cu, fb->fn, fb->nt, fb_lds);
        if (e != hipSuccess) return fail_hip(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
        if (fb_cu < 1) return fail(FPLDPC_ERR_UNSUPPORTED, "fallback kernel cannot be resident");
        *grid = prop.multiProcessorCount;
        *threads = fb->nt;
        *lds_out = fb_lds;
        if (fb->gmem) out->scratch_ints = std::max(out->scratch_ints, (size_t)*grid * fb->dc * m_pad);
        return FPLDPC_OK;
    };
    if (pick->fallback != Variant::kNone) {
        int st = setup_fallback(pick->fallback, &out->fb_grid, &out->fb_threads, &out->fb_lds);
        if (st) return st;
        const VariantInfo *fb = find_variant(pick->fallback);
        if (fb->fallback != Variant::kNone) {  // e.g. packed R kernel -> LDS-state int16 -> global int32
            out->fallback2 = fb->fallback;
            st = setup_fallback(fb->fallback, &out->fb2_grid, &out->fb2_threads, &out->fb2_lds);
            if (st) return st;
        }
        out->cmax = cmax;  // (packed_cmax)
    }
    out->lds_bytes = lds;
    out->name = pick->name;
    out->sort_checks = pick->lo_passes > 0;
    return FPLDPC_OK;
}

int launch_decode(const KernelChoice &kc, const DeviceCode &dcode, const LaunchArgs &la, void *stream) {
    const VariantInfo *vi = find_variant(kc.v);
    if (!vi) return fail(FPLDPC_ERR_ARG, "decoder has no kernel");
    if (la.batch <= 0) return FPLDPC_OK;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    // A launch that fails leaves the counter block for the next call to find non-zero: re-zero it.
    auto launch_failed = [&](hipError_t err, const char *what) {
        (void)hipMemsetAsync(la.work_counter, 0, kCounterInts * sizeof(int32_t), s);
        return fail_hip(err, what);
    };
    KArgs a{};
    a.counters = la.work_counter;
    a.llr = la.llr;
    a.llr_i16 = la.llr_i16;
    a.n = dcode.n;
    a.m = dcode.m;
    a.m_pad = dcode.m_pad;
    a.batch = la.batch;
    a.max_iter = la.max_iter;
    a.C = la.C;
    a.mask = la.mask;
    a.early_term = la.early_term;
    a.precheck = la.precheck;
    a.vidx = dcode.vidx;
    a.cdeg = dcode.cdeg;
    a.hard = la.hard;
    a.hard_words = la.hard_words;
    a.iters = la.iters;
    a.syn_ok = la.syn_ok;
    a.post = la.post;
    a.bit_errors = la.bit_errors;
    a.totals = la.totals;
    a.info_idx = la.info_idx;
    a.info_bits = la.info_bits;
    a.k_info = la.k_info;
    a.info_mask = la.info_mask;
    a.work_counter = la.work_counter;
    a.c2v_scratch = la.c2v_scratch;
    a.bfe_w = la.bfe_w;
    a.probe = la.probe;
    a.wgtrace = la.wgtrace;
    a.split_tail = la.split_tail;
    if (kc.fallback == Variant::kNone) {
        const int grid = std::min(kc.grid, la.batch);
        a.last_in_chain = 1;
        hipLaunchKernelGGL(vi->fn, dim3(grid), dim3(kc.threads), kc.lds_bytes, s, a);
        e = hipGetLastError();
        if (e != hipSuccess) return launch_failed(e, "kernel launch");
        return FPLDPC_OK;
    }
    // packed kernel (two frames per workgroup), then the exact kernels of the fallback chain over
    // the frames each one rejected.  Counters: [0] work, [1] fallback work, [2] list-0 count,
    // [3] second fallback work, [4] list-1 count; list l is fb_list + l * batch.
    if (!la.fb_list) return fail(FPLDPC_ERR_ARG, "packed kernel needs a fallback list");
    int *const c = la.work_counter;
    a.fb_list = la.fb_list;
    a.fb_count = c + 2;
    a.cmax = kc.cmax;
    const int per_wg = vi->lds_state ? 1 : 2;  // frames in flight per workgroup
    const int grid = std::min(kc.grid, (la.batch + per_wg - 1) / per_wg);
    hipLaunchKernelGGL(vi->fn, dim3(grid), dim3(kc.threads), kc.lds_bytes, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return launch_failed(e, "kernel launch");
    KArgs b = a;
    b.last_in_chain = kc.fallback2 == Variant::kNone;
    b.frame_list = la.fb_list;
    b.frame_count = c + 2;
    b.work_counter = c + 1;
    b.fb_list = kc.fallback2 != Variant::kNone ? la.fb_list + la.batch : nullptr;
    b.fb_count = kc.fallback2 != Variant::kNone ? c + 4 : nullptr;
    const VariantInfo *fb = find_variant(kc.fallback);
    hipLaunchKernelGGL(fb->fn, dim3(std::min(kc.fb_grid, la.batch)), dim3(kc.fb_threads), kc.fb_lds, s, b);
    e = hipGetLastError();
    if (e != hipSuccess) return launch_failed(e, "fallback kernel launch");
    if (kc.fallback2 == Variant::kNone) return FPLDPC_OK;
    KArgs b2 = b;
    b2.last_in_chain = 1;
    b2.frame_list = la.fb_list + la.batch;
    b2.frame_count = c + 4;
    b2.work_counter = c + 3;
    b2.fb_list = nullptr;
    b2.fb_count = nullptr;
    const VariantInfo *fb2 = find_variant(kc.fallback2);
    hipLaunchKernelGGL(fb2->fn, dim3(std::min(kc.fb2_grid, la.batch)), dim3(kc.fb2_threads), kc.fb2_lds, s, b2);
    e = hipGetLastError();
    if (e != hipSuccess) return launch_failed(e, "second fallback kernel launch");
    return FPLDPC_OK;
}

int edge_kernel_dc(int dc_max) {
    for (int d : {8, 16, 32, 48, 64})
        if (dc_max <= d) return d;
    return 0;
}

int launch_decode_frame(const LaunchArgs &la, const EdgeTables &t, int32_t *edge, int keep, void *stream) {
    KArgs a{};
    a.llr = la.llr;
    a.llr_i16 = la.llr_i16;
    a.n = t.n;
    a.m = t.m;
    a.batch = 1;
    a.max_iter = la.max_iter;
    a.C = la.C;
    a.mask = la.mask;
    a.early_term = la.early_term;
    a.precheck = la.precheck;
    a.hard = la.hard;
    a.hard_words = la.hard_words;
    a.iters = la.iters;
    a.syn_ok = la.syn_ok;
    a.post = la.post;
    const EdgeArgs e{t.vidx, t.cdeg, edge, t.c2v, keep, t.dc_max};
    size_t lds = (size_t)(4 * t.n + kMiscInts) * sizeof(int);
    if (lds > 160 * 1024) return fail(FPLDPC_ERR_UNSUPPORTED, "code length too large for LDS-resident posteriors");
    // the c2v double buffer [2][dc][m] int32 and the index table [dc][m] uint16 in LDS when they fit
    const size_t lds_state = lds + (size_t)t.dc * t.m * (2 * sizeof(int32_t) + sizeof(uint16_t));
    const bool in_lds = lds_state <= 160 * 1024 && !getenv("FPLDPC_EDGES_GLOBAL");
    if (in_lds) lds = lds_state;
    void (*fn)(KArgs, EdgeArgs) = nullptr;
    switch (t.dc) {
        case 8: fn = in_lds ? flood_edges<8, true> : flood_edges<8, false>; break;
        case 16: fn = in_lds ? flood_edges<16, true> : flood_edges<16, false>; break;
        case 32: fn = in_lds ? flood_edges<32, true> : flood_edges<32, false>; break;
        case 48: fn = in_lds ? flood_edges<48, true> : flood_edges<48, false>; break;
        case 64: fn = in_lds ? flood_edges<64, true> : flood_edges<64, false>; break;
        default: return fail(FPLDPC_ERR_UNSUPPORTED, "check degree above 64");
    }
    hipError_t err;
    if (lds > 64 * 1024) {
        err = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (err != hipSuccess) return fail_hip(err, "hipFuncSetAttribute");
    }
    hipLaunchKernelGGL(fn, dim3(1), dim3(kNT), lds, (hipStream_t)stream, a, e);
    err = hipGetLastError();
    if (err != hipSuccess) return fail_hip(err, "edge-state kernel launch");
    return FPLDPC_OK;
}

}  // namespace fpldpc
#endif  // FPLDPC_TU_ARRAY1 || FPLDPC_TU_TABLE1
