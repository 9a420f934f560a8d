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
#include <string>

#include "fpldpc_internal.hpp"

namespace fpldpc {
namespace {

constexpr int kNT = 256;  // threads per workgroup (4 waves)

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
    int *work_counter;
    int32_t *c2v_scratch;
    uint32_t bfe_w;  // width_mask = 2^(bfe_w + 2) - 1 (contiguous-mask kernels only)
};

// x [+] y = sgn(x) sgn(y) (min(|x|,|y|) + max(0, C - ((|x|+|y|) & mask) >> 2)
//                                      - max(0, C - (||x|-|y|| & mask) >> 2)),  sgn(0) = -1.
// ArrayLDPC_Decoder.cpp:677-694, ArrayLDPCMacro.h:222-224.  The magnitude term r is never
// negative (checked exhaustively for masks 0x3f..0xfff, tests/test_oracle.py), so the sign of the
// result is + iff (x > 0) == (y > 0), and r == 0 gives 0 either way.
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
__device__ __forceinline__ void frame_load(const KArgs &a, int cw, int *bufs, int *llr_s) {
    const int n = a.n;
    const size_t base = (size_t)cw * n;
    for (int v = threadIdx.x; v < n; v += kNT) {
        const int x = load_llr(a, base + v);
        llr_s[v] = x;
        bufs[v] = x;
        bufs[n + v] = x;
    }
}

// Frame epilogue: posteriors, packed hard decisions, per-frame BER and totals.
__device__ __forceinline__ void frame_store(const KArgs &a, int cw, const int *pf, bool write_post, int iters,
                                            int ok, int *misc) {
    const int n = a.n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (a.post && write_post)
        for (int v = tid; v < n; v += kNT) a.post[(size_t)cw * n + v] = pf[v];
    if (a.hard) {
        uint32_t *h = a.hard + (size_t)cw * a.hard_words;
        for (int base = wave * 64; base < n; base += kNT) {
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
        for (int i = tid; i < a.k_info; i += kNT) e += ((pf[a.info_idx[i]] <= 0) ? 1 : 0) != a.info_bits[i];
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
            misc[0] = atomicAdd(a.work_counter, 1);
            misc[1] = 0;
        }
        __syncthreads();
        const int cw = misc[0];
        if (cw >= a.batch) break;
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
            misc[0] = atomicAdd(a.work_counter, 1);
            misc[1] = 0;
        }
        __syncthreads();
        const int cw = misc[0];
        if (cw >= a.batch) break;
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
}

// ------------------------------------------------------------------------------------------
// Sign/magnitude kernels.  Box-plus splits exactly into a magnitude chain and a sign parity:
//   |x [+] y| = bp_mag(|x|, |y|), sign = XOR of the (v <= 0) flags,
// because a zero magnitude absorbs (bp_mag(0, b) = 0, so the sgn(0) = -1 rule of
// ArrayLDPCMacro.h:222-224 can only ever multiply a zero).  The serial fold ORDER of the
// magnitudes is kept exactly as the reference's (ArrayLDPC_Decoder.cpp:83-116); only the sign
// bookkeeping leaves the chain: one parity S per check, c2v_k sign = S ^ neg(m_k).
// Checked exhaustively against the reference fold in tests/test_oracle.py::test_sign_split.
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
            misc[0] = atomicAdd(a.work_counter, 1);
            misc[1] = 0;
        }
        __syncthreads();
        const int cw = misc[0];
        if (cw >= a.batch) break;
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
}

typedef void (*KernelFn)(KArgs);

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
};

const VariantInfo kVariants[] = {
    {Variant::kArray47, flood_array<47>, 47, kNT, true, false, "flood_array<P=47>", 47, true},
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

int choose_kernel(const fpldpc_code &code, int device, int mask, KernelChoice *out) {
    const bool low_mask = mask >= 3 && (mask & (mask + 1)) == 0;
    for (int r = 0; r < code.m; r++)
        if (code.cdeg[r] < 2) return fail(FPLDPC_ERR_UNSUPPORTED, "check of degree < 2 (reference behaviour undefined)");
    if (code.dc_max > 64) return fail(FPLDPC_ERR_UNSUPPORTED, "check degree above 64");
    const size_t lds = (size_t)(4 * code.n + 4) * sizeof(int);
    if (lds > 160 * 1024) return fail(FPLDPC_ERR_UNSUPPORTED, "code length too large for LDS-resident posteriors");
    // The reference iterates its checks in block order and folds each in clist order; the kernel
    // folds in clist order per check, so only the degree envelope matters for the choice.
    int actual_dc = 0;
    for (int r = 0; r < code.m; r++) actual_dc = std::max(actual_dc, (int)code.cdeg[r]);
    bool regular = true;
    for (int r = 0; r < code.m; r++) regular &= code.cdeg[r] == actual_dc;
    const VariantInfo *pick = nullptr;
    for (const auto &x : kVariants) {
        if (x.gmem) continue;
        if (x.array_p && !(code.array_p == x.array_p && code.array_forward)) continue;
        if (x.low_mask && !low_mask) continue;
        if (x.regular ? !(regular && actual_dc == x.dc) : actual_dc > x.dc) continue;
        if (code.m > x.max_m) continue;
        pick = &x;
        break;
    }
    if (!pick)
        for (const auto &x : kVariants)
            if (x.gmem && actual_dc <= x.dc) {
                pick = &x;
                break;
            }
    if (!pick) return fail(FPLDPC_ERR_UNSUPPORTED, "no kernel variant for this code");
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
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pick->fn, kNT, lds);
    if (e != hipSuccess) return fail_hip(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    if (per_cu < 1) return fail(FPLDPC_ERR_UNSUPPORTED, "kernel cannot be resident (occupancy 0)");
    out->v = pick->v;
    out->threads = kNT;
    out->grid = per_cu * prop.multiProcessorCount;
    out->lds_bytes = lds;
    out->name = pick->name;
    const int m_pad = (code.m + 63) / 64 * 64;
    out->scratch_ints = pick->gmem ? (size_t)out->grid * pick->dc * m_pad : 0;
    return FPLDPC_OK;
}

int launch_decode(const KernelChoice &kc, const DeviceCode &dcode, const LaunchArgs &la, void *stream) {
    const VariantInfo *vi = find_variant(kc.v);
    if (!vi) return fail(FPLDPC_ERR_ARG, "decoder has no kernel");
    if (la.batch <= 0) return FPLDPC_OK;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(la.work_counter, 0, 16, s);
    if (e != hipSuccess) return fail_hip(e, "hipMemsetAsync(work counter)");
    KArgs a;
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
    a.work_counter = la.work_counter;
    a.c2v_scratch = la.c2v_scratch;
    a.bfe_w = la.bfe_w;
    const int grid = std::min(kc.grid, la.batch);
    hipLaunchKernelGGL(vi->fn, dim3(grid), dim3(kc.threads), kc.lds_bytes, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return fail_hip(e, "kernel launch");
    return FPLDPC_OK;
}

}  // namespace fpldpc
