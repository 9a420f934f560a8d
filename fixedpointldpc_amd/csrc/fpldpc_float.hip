// fpldpc_float.hip -- the reference's floating-point BP decoder (FP_Decoder::decode_general,
// ArrayLDPC_Decoder.cpp:735-933) on gfx950: exact-Jacobian box-plus in double
// (sxor(double, double), :724-732), the same flooding schedule and fold order as the fixed-point
// path, early termination on checkPost (:335-372).  A comparison mode next to the bit-exact
// fixed-point decoder.
//
// Layout: one persistent workgroup decodes one frame at a time (frames pulled from an atomic
// counter).  Posteriors live in LDS (double[n]); edge messages live in a per-workgroup HBM/L2
// scratch in the reference's EdgeRAM layout edge[slot * m + check] (ArrayLDPCMacro.h:95-97,162),
// so a lane per check reads its slots coalesced across the wavefront.  The check phase writes the
// forward chain F_k to a second scratch plane and walks back once: c2v_k = F_{k-1} [+] B_{k+1},
// the reference's operand order.  The variable phase sums c2v in vlist order, then adds the
// channel value (:888-910), and writes v2c = post - c2v.
//
// Exactness: the box-plus is the reference's exact Jacobian sxor.  By default each check is folded in
// the tanh domain (check_update_tanh*: E = exp(-|x|), E_r = (E_x + E_y) / (1 + E_x E_y), one exp in
// and one log out per edge instead of two exps and two logs per box-plus) -- the same function with
// different rounding -- and a check holding a message of magnitude >= 690 (where E would leave the
// normal doubles) in the log domain, operation for operation as the reference (-ffp-contract=off, no
// reassociation; exp / log as the device libm's sequence and an fdlibm-style log, within an ulp of
// glibc's).  FPLDPC_FLOAT_TANH=0 builds the log domain everywhere.  tests/test_gpu_float.py measures
// how often either moves a hard decision or an iteration count (BER-level tolerance):
// round 4, tanh default: 0 frames differ in every float GPU test, posteriors within 1.2e-10 relative.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <type_traits>
#include <vector>

#include "fpldpc_internal.hpp"
#include "fpldpc_float_math.hpp"

namespace fpldpc {

namespace {
struct FArgs;
}

struct FloatState {
    int device = -1;
    int grid = 0;             // resident workgroups
    size_t lds = 0;
    void (*fn)(FArgs) = nullptr;
    int32_t *d_cvar = nullptr;   // [dc_max][m] var of slot k of check c (-1 pad)
    uint8_t *d_cdeg = nullptr;   // [m]
    int32_t *d_vedge = nullptr;  // [dv_max][n] edge index slot*m + c of the k-th check of v
    uint8_t *d_vdeg = nullptr;   // [n]
    double *d_msg = nullptr;     // [grid][planes][dc_max * m]: edge messages (+ forward chain, generic kernel)
    int planes = 2;
    int *d_counter = nullptr;
    ~FloatState() {
        (void)hipFree(d_cvar);
        (void)hipFree(d_cdeg);
        (void)hipFree(d_vedge);
        (void)hipFree(d_vdeg);
        (void)hipFree(d_msg);
        (void)hipFree(d_counter);
    }
};

void free_float_state(FloatState *s) { delete s; }

namespace {

constexpr int kFT = 256;           // threads per workgroup
constexpr int kMaxFloatN = 16384;  // posteriors in LDS: 128 KiB
// 1 + exp(-x) == 1 exactly for x >= kLogUlp (exp(-x) < 2^-53, half an ulp of 1), so the log term is
// exactly 0 there and both transcendental calls can be skipped without changing a bit.
constexpr double kLogUlp = 36.75;

struct FArgs {
    const double *llr;
    int batch, n, m, dc, dv, max_iter, early_term;
    const int32_t *cvar;
    const uint8_t *cdeg;
    const int32_t *vedge;
    const uint8_t *vdeg;
    double *msg;
    int *counter;
    uint32_t *hard;
    int hard_words;
    int32_t *iters;
    uint8_t *syn_ok;
    double *post;
    int32_t *bit_errors;
    unsigned long long *totals;
    const int32_t *info_idx;
    const uint8_t *info_bits;
    int k_info;
};

// log(1 + exp(-x)): exp_neg and log_1to2 (fpldpc_float_math.hpp), the libm's operations
__device__ __forceinline__ double log1pexp_neg(double x) {  // log(1 + exp(-x)) as the reference writes it
    if (x >= kLogUlp) return 0.0;
    const double y = __dadd_rn(1.0, exp_neg(x));
    return log_1to2(y);
}

// sxor(double, double), ArrayLDPC_Decoder.cpp:724-732: sgn(x)*sgn(y)*(min + log(..) - log(..)),
// sgn(0) = -1 (ArrayLDPCMacro.h:218-220); the int*int*double product is an exact sign flip.
__device__ __forceinline__ double sxor_f64(double x, double y) {
    const double v1 = fabs(x), v2 = fabs(y);
    const double sum_abs = __dadd_rn(v1, v2), diff_abs = fabs(__dsub_rn(v1, v2));
    const double mn = v2 < v1 ? v2 : v1;  // std::min
    const double r = __dsub_rn(__dadd_rn(mn, log1pexp_neg(sum_abs)), log1pexp_neg(diff_abs));
    return ((x > 0.0) == (y > 0.0)) ? r : -r;
}

// Check phase for check c of degree deg >= 2: edge slots hold v2c on entry, c2v on exit.  The
// forward chain F_k = F_{k-1} [+] v_k (F_0 = v_0, k <= deg-2) goes to the fwd scratch; the walk
// back emits c2v_{deg-1} = F_{deg-2}, c2v_k = F_{k-1} [+] B_{k+1}, c2v_0 = B_1 with
// B_{deg-1} = v_{deg-1}, B_k = B_{k+1} [+] v_k (:799-832; F_{deg-1} and B_0 are never used).
__device__ __forceinline__ void check_update(double *msg, double *fwd, int m, int c, int deg) {
    double F = msg[c];
    fwd[c] = F;
    for (int k = 1; k <= deg - 2; ++k) {
        F = sxor_f64(F, msg[k * m + c]);
        fwd[k * m + c] = F;
    }
    double B = msg[(deg - 1) * m + c];
    msg[(deg - 1) * m + c] = F;
    for (int k = deg - 2; k >= 1; --k) {
        const double vk = msg[k * m + c];
        msg[k * m + c] = sxor_f64(fwd[(k - 1) * m + c], B);
        B = sxor_f64(B, vk);
    }
    msg[c] = B;
}

// Register form for check degrees <= DC (DC a template constant, REGULAR: every check has degree
// DC): only c2v is state.  The edge scratch holds c2v (no v2c plane, no forward-chain plane): the
// check phase forms v2c_k = post[v_k] - c2v_k on the fly -- the same __dsub_rn(acc, c2v) the
// reference's variable phase stores (:888-910), so bit-identical -- and keeps the forward chain
// F_0..F_{deg-2} in registers.  Per edge and iteration: c2v read twice and written once by the
// check phase (the backward walk re-reads v_k), read once by the variable phase; 32 B instead of
// the generic kernel's 52 B (msg + fwd planes).  first: c2v = 0 (edge init v2c = LLR, :762-778).
// Regular codes of large degree (A, R: 47): fully unrolled around an out-of-line box-plus (135
// inlined copies of two exp/log pairs would not fit the instruction cache, and hipcc refuses the
// unroll), with the forward chain F_0..F_{DC-2} in VGPRs -- the loop form's dynamically indexed F[]
// lands in private scratch, 16 B per edge-iteration of HBM traffic (A: 64 -> 36 GB per 4096-frame
// launch, 3 % slower: 3 waves per SIMD at 167 VGPRs instead of 4, profiles/r2/float/).  Tried and
// slower: one box-plus per call in the walk back (-4 %), a middle-out schedule with two box-pluses
// in every call (-4 %: 24 argument moves per call).  A callee starts with s_waitcnt 0, so a load
// issued before a call cannot overlap it; the callee therefore does the step's memory work itself:
// it stores the previous output, issues the next slot's c2v and var-index loads, computes the
// box-plus, and only then reads the posterior from LDS and returns v2c = post - c2v (the
// __dsub_rn the variable phase of :888-910 stores).  The next call's s_waitcnt finds the store done.
struct SxOut {
    double r, v;
};
enum : int { kSxLoad = 1, kSxStore = 2, kSxFirst = 4 };
__device__ __attribute__((noinline)) SxOut sxor_step(double x, double y, const double *ld_c2v, const int32_t *ld_var,
                                                      uint32_t post_lds, double *st, double st_val, int ops) {
    if (ops & kSxStore) *st = st_val;
    int idx = 0;
    double c = 0.0;
    if (ops & kSxLoad) {
        idx = *ld_var;
        if (!(ops & kSxFirst)) c = *ld_c2v;
    }
    SxOut o;
    o.r = sxor_f64(x, y);
    o.v = 0.0;
    if (ops & kSxLoad) {
        const double p = reinterpret_cast<const __attribute__((address_space(3))) double *>((size_t)post_lds)[idx];
        o.v = (ops & kSxFirst) ? p : __dsub_rn(p, c);
    }
    return o;
}
// One walk-back step in one call: c2v_k = F_{k-1} [+] B_{k+1} and B_k = B_{k+1} [+] v_k are
// independent, so the callee interleaves their exp/log sequences (two dependency chains).
struct SxOut2 {
    double o, b, v;
};
__device__ __attribute__((noinline)) SxOut2 sxor_step2(double f, double B, double vk, const double *ld_c2v,
                                                        const int32_t *ld_var, uint32_t post_lds, double *st, double st_val,
                                                        int ops) {
    if (ops & kSxStore) *st = st_val;
    int idx = 0;
    double c = 0.0;
    if (ops & kSxLoad) {
        idx = *ld_var;
        if (!(ops & kSxFirst)) c = *ld_c2v;
    }
    SxOut2 o;
    o.o = sxor_f64(f, B);
    o.b = sxor_f64(B, vk);
    o.v = 0.0;
    if (ops & kSxLoad) {
        const double p = reinterpret_cast<const __attribute__((address_space(3))) double *>((size_t)post_lds)[idx];
        o.v = (ops & kSxFirst) ? p : __dsub_rn(p, c);
    }
    return o;
}
#ifndef FPLDPC_FLOAT_TANH
#define FPLDPC_FLOAT_TANH 1  // 0: the log-domain form everywhere (the reference's operation order)
#endif
template <int DC>
__device__ __forceinline__ void check_update_unrolled(double *msg, const double *s_post, const int32_t *cvar, int m, int c,
                                                      bool first) {
    const size_t stride = (size_t)m;
    double *pm = msg + c;  // slot 0 of this check
    const int32_t *pv = cvar + c;
    asm volatile("" : "+v"(pm), "+v"(pv));
    const uint32_t post_lds = (uint32_t)(size_t)(const __attribute__((address_space(3))) double *)s_post;
    const int fl = first ? kSxFirst : 0;
    double v0;
    {
        const double p = s_post[*pv];
        v0 = first ? p : __dsub_rn(p, *pm);
    }
    double *const p1 = pm + stride;
    double F[DC - 1];
    F[0] = v0;
    // v_1 (no box-plus yet: fetch through a dummy step would cost a call; load it here)
    double vk;
    {
        const double p = s_post[pv[stride]];
        vk = first ? p : __dsub_rn(p, *p1);
    }
    // forward: F_k = F_{k-1} [+] v_k (k = 1..DC-2), each call fetching v_{k+1}.  The slot pointers
    // are walked and made opaque at every step (else the compiler keeps all 47 edge addresses live).
    double *ql = p1;  // load position
    const int32_t *qv = pv + stride;
    auto adv = [&](int dir) {
        ql = dir > 0 ? ql + stride : ql - stride;
        qv = dir > 0 ? qv + stride : qv - stride;
        asm volatile("" : "+v"(ql), "+v"(qv));
    };
#pragma unroll
    for (int k = 1; k <= DC - 2; ++k) {
        adv(1);  // slot k + 1
        const SxOut o = sxor_step(F[k - 1], vk, ql, qv, post_lds, nullptr, 0.0, kSxLoad | fl);
        F[k] = o.r;
        vk = o.v;
    }
    double B = vk;  // B_{DC-1} = v_{DC-1}; ql at slot DC-1
    // v_{DC-2}: the forward step DC-2's input, needed again by the walk back (re-read)
    adv(-1);
    double vcur;
    {
        const double p = s_post[*qv];
        vcur = first ? p : __dsub_rn(p, *ql);
    }
    // backward: c2v_k = F_{k-1} [+] B_{k+1}, B_k = B_{k+1} [+] v_k (k = DC-2..1); the first call
    // stores c2v_{DC-1} = F_{DC-2}, each later one the previous step's c2v_{k+1}
    double prev = F[DC - 2];
    double *qs = ql + stride;  // store position: slot k + 1
#pragma unroll
    for (int k = DC - 2; k >= 1; --k) {
        adv(-1);  // slot k - 1
        const SxOut2 o = sxor_step2(F[k - 1], B, vcur, ql, qv, post_lds, qs, prev, (k >= 2 ? kSxLoad : 0) | kSxStore | fl);
        prev = o.o;
        B = o.b;
        vcur = o.v;
        qs -= stride;
        asm volatile("" : "+v"(qs));
    }
    pm[stride] = prev;  // c2v_1
    pm[0] = B;          // c2v_0 = B_1
}

// The same fold in the tanh domain: with E = exp(-|x|), the exact box-plus magnitude
// |x [+] y| = min + log(1 + e^-(|x|+|y|)) - log(1 + e^-||x|-|y||) (sxor, :724-732) becomes
// E_r = (E_x + E_y) / (1 + E_x E_y), and the sign is the parity of the (x <= 0) flags (sgn(0) = -1
// only ever multiplies a zero magnitude, E = 1).  Per edge and iteration: an exp on the way in (twice:
// the walk back recomputes v_k instead of keeping 47 values live), a log on the way out, three
// add / FMA / division box-pluses -- against three box-pluses of two exps and two logs each.  The
// same mathematics with different rounding: each operation is within an ulp, but E and the folded
// (E_x + E_y) / (1 + E_x E_y) sit next to 1 when a magnitude is small, so -log_unit() of them carries
// an ABSOLUTE error of about ulp(1) = 2.2e-16 per message -- a relative error only for |x| of order 1
// (for |x| ~ 1e-8 it is ~1e-8 relative).  The reference's min + log - log form can round such a tiny
// magnitude to 0 or below where this one keeps it positive.  Decisions are unaffected in every test:
// 0 frames differ from the reference and the oracle, posteriors of those frames within 1e-8 relative
// (measured worst 3.4e-9, W 1.0 dB; tests/test_gpu_float.py).  E stays a normal
// double while every |v| < kTanhMax; a check with a larger message returns false and is folded by
// the log-domain form instead (its chain values could underflow: converged frames' last iterations).
constexpr double kTanhMax = 690.0;
__device__ __forceinline__ double bp_tanh(double ea, double eb) {
    return div_1to2(__dadd_rn(ea, eb), fma(ea, eb, 1.0));
}
// The steps are out-of-line callees like sxor_step / sxor_step2, two slots per call (inlined across
// 47 unrolled slots, hipcc hoists the exp / log polynomials' 64-bit constants into VGPRs next to the
// 46 forward-chain values and spills).  A call's loads, issued two slots ahead, are in flight across
// two slots' arithmetic.  Measured (A / R Mb/s, profiles/r4/ab/float_pair.txt): one slot per call
// 560 / 29.0, two 684 / 35.6, three 664 / 35.3 (more VGPRs spilled around the calls); with computed
// array indices one slot 660 / 37.4, two 783 / 49.3; 2 or 4 workgroups per CU lower with the whole
// forward chain in VGPRs.  Keeping it at even k only (the walk back recomputes the odd F_k) frees 46
// VGPRs: 4 workgroups per CU, A +1.5 %, R +5 % (profiles/r4/ab/float_ckpt.txt).
//
// A slot's variable index: computed by the caller (ARRAY: forward array codes) or read from the
// [slot][check] table in the callee.  The table pointer is made opaque, else hipcc promotes it to the
// loaded value and moves the load into the caller, where the callee's entry wait exposes it.
template <bool ARRAY>
using VarRef = typename std::conditional<ARRAY, int, const int32_t *>::type;
template <bool ARRAY>
__device__ __forceinline__ void var_idx(VarRef<ARRAY> ra, VarRef<ARRAY> rb, int &ia, int &ib) {
    if constexpr (ARRAY) {
        ia = ra;
        ib = rb;
    } else {
        asm volatile("" : "+v"(ra), "+v"(rb));
        ia = *ra;
        ib = *rb;
    }
}
// Forward pair: F_k = F_{k-1} [+] E(v_k), F_{k+1} = F_k [+] E(v_{k+1}); then the v2c of the next two
// slots (c2v at ca, cb).
struct Tf2 {
    double f1, f2, v1, v2;
};
template <bool ARRAY>
__device__ __attribute__((noinline)) Tf2 tanh_fwd2(double f, double va, double vb, const double *ca, VarRef<ARRAY> ra,
                                                    const double *cb, VarRef<ARRAY> rb, uint32_t post_lds, int first) {
    int ia, ib;
    var_idx<ARRAY>(ra, rb, ia, ib);
    double c1 = 0.0, c2 = 0.0;
    if (!first) {
        c1 = *ca;
        c2 = *cb;
    }
    Tf2 o;
    o.f1 = bp_tanh(f, exp_neg(fmin(fabs(va), kTanhMax)));
    o.f2 = bp_tanh(o.f1, exp_neg(fmin(fabs(vb), kTanhMax)));
    const auto *P = reinterpret_cast<const __attribute__((address_space(3))) double *>((size_t)post_lds);
    const double p1 = P[ia], p2 = P[ib];
    o.v1 = first ? p1 : __dsub_rn(p1, c1);
    o.v2 = first ? p2 : __dsub_rn(p2, c2);
    return o;
}
struct Tb2 {
    double oa, ob, b, v1, v2;
};
// Walk-back pair over slots k (even) and k-1 (the caller keeps the forward chain at even k only):
// stores the two pending outputs (s2 may be null), recomputes F_{k-1} = F_{k-2} [+] E(v_{k-1}) (the
// forward step's operations on the same inputs, so the same value), returns the c2v magnitudes
// -log(F_{k-1} [+] B_{k+1}) and -log(F_{k-2} [+] B_k) and B_{k-1}; then the v2c of the next two slots
template <bool ARRAY>
__device__ __attribute__((noinline)) Tb2 tanh_bwd2c(double fe, double B, double va, double vb, const double *ca,
                                                     VarRef<ARRAY> ra, const double *cb, VarRef<ARRAY> rb, uint32_t post_lds,
                                                     double *s1, double w1, double *s2, double w2, int first) {
    *s1 = w1;
    if (s2) *s2 = w2;
    int ia, ib;
    var_idx<ARRAY>(ra, rb, ia, ib);
    double c1 = 0.0, c2 = 0.0;
    if (!first) {
        c1 = *ca;
        c2 = *cb;
    }
    Tb2 o;
    const double Eb = exp_neg(fabs(vb));  // |v| < kTanhMax here: = the forward step's E
    const double Fb = bp_tanh(fe, Eb);    // F_{k-1}
    o.oa = -log_unit(bp_tanh(Fb, B));
    const double B1 = bp_tanh(B, exp_neg(fabs(va)));
    o.ob = -log_unit(bp_tanh(fe, B1));
    o.b = bp_tanh(B1, Eb);
    const auto *P = reinterpret_cast<const __attribute__((address_space(3))) double *>((size_t)post_lds);
    const double p1 = P[ia], p2 = P[ib];
    o.v1 = first ? p1 : __dsub_rn(p1, c1);
    o.v2 = first ? p2 : __dsub_rn(p2, c2);
    return o;
}
// The walk back's first (single) step with the pair callees' memory work: stores c2v_{DC-1}, returns
// -log(F_{DC-3} [+] B_{DC-1}) and B_{DC-2}, then the v2c of the next two slots
template <bool ARRAY>
__device__ __attribute__((noinline)) Tb2 tanh_bwd1l(double f, double B, double va, const double *ca, VarRef<ARRAY> ra,
                                                     const double *cb, VarRef<ARRAY> rb, uint32_t post_lds, double *s1,
                                                     double w1, int first) {
    *s1 = w1;
    int ia, ib;
    var_idx<ARRAY>(ra, rb, ia, ib);
    double c1 = 0.0, c2 = 0.0;
    if (!first) {
        c1 = *ca;
        c2 = *cb;
    }
    Tb2 o;
    o.oa = -log_unit(bp_tanh(f, B));
    o.ob = 0.0;
    o.b = bp_tanh(B, exp_neg(fabs(va)));
    const auto *P = reinterpret_cast<const __attribute__((address_space(3))) double *>((size_t)post_lds);
    const double p1 = P[ia], p2 = P[ib];
    o.v1 = first ? p1 : __dsub_rn(p1, c1);
    o.v2 = first ? p2 : __dsub_rn(p2, c2);
    return o;
}
// F_{DC-2} (the forward chain's last step, no memory work)
__device__ __attribute__((noinline)) double tanh_fwd1(double f, double v) {
    return bp_tanh(f, exp_neg(fmin(fabs(v), kTanhMax)));
}

// One check in the tanh domain (DC odd: A, R); false (msg untouched) when a message has |v| >= kTanhMax.
// Forward pairs (1,2) .. (DC-4, DC-3) then F_{DC-2}; walk back c2v_{DC-1}, pairs (DC-2, DC-3) .. (3, 2),
// then c2v_1 and c2v_0 = B_1.  The v_k of the walk back are re-read (post - c2v), not kept.
template <int DC, bool ARRAY>
__device__ __forceinline__ bool check_update_tanh(double *msg, const double *s_post, const int32_t *cvar, int m, int c,
                                                  bool first) {
    static_assert(DC % 2 == 1 && DC >= 7, "odd degree");
    const size_t stride = (size_t)m;
    double *pm = msg + c;
    const int32_t *pv = cvar + c;
    asm volatile("" : "+v"(pm), "+v"(pv));
    const uint32_t post_lds = (uint32_t)(size_t)(const __attribute__((address_space(3))) double *)s_post;
    const int fl = first ? 1 : 0;
    // a slot cursor: c2v pointer and var-table pointer (ARRAY: slot k and x = (j + i*k) mod P of check
    // c = i*P + j, variable k*P + x), walked and made opaque at every step (else the compiler keeps all
    // 47 edge addresses live)
    const int arow = ARRAY ? c / DC : 0;
    struct Cur {
        double *q;
        const int32_t *v;
        int x, k;
    };
    auto adv = [&](Cur &u, int dir) {
        u.q = dir > 0 ? u.q + stride : u.q - stride;
        if constexpr (ARRAY) {
            u.k += dir;
            u.x = dir > 0 ? u.x + arow : u.x - arow;
            u.x = u.x >= DC ? u.x - DC : (u.x < 0 ? u.x + DC : u.x);
            asm volatile("" : "+v"(u.q), "+v"(u.x));
        } else {
            u.v = dir > 0 ? u.v + stride : u.v - stride;
            asm volatile("" : "+v"(u.q), "+v"(u.v));
        }
    };
    auto ref = [&](const Cur &u) -> VarRef<ARRAY> {
        if constexpr (ARRAY)
            return u.k * DC + u.x;
        else
            return u.v;
    };
    auto load = [&](const Cur &u) {
        int idx;
        if constexpr (ARRAY)
            idx = u.k * DC + u.x;
        else
            idx = *u.v;
        const double p = s_post[idx];
        return first ? p : __dsub_rn(p, *u.q);
    };
    // sign parity S of the (v <= 0) flags and the largest |v|, folded into VGPRs at every slot (left to
    // itself the compiler keeps 47 compare masks in SGPR pairs and spills)
    uint32_t S = 0;
    double amax = 0.0;
    auto track = [&](double v) {
        S ^= (v > 0.0) ? 0u : 1u;
        amax = fmax(amax, fabs(v));
        asm volatile("" : "+v"(S), "+v"(amax));
    };
    Cur cu{pm, pv, ARRAY ? c - arow * DC : 0, 0};
    asm volatile("" : "+v"(cu.x));
    // the forward chain kept at even k only (F[j] = F_{2j}: 46 VGPRs instead of 92, 4 workgroups per CU);
    // the walk back recomputes each odd F_k with the forward step's operations
    double F[(DC - 1) / 2];
    auto Fput = [&](int k, double x) {
        if (k % 2 == 0) F[k / 2] = x;
    };
    auto Fget = [&](int k) { return F[k / 2]; };
    const double v0 = load(cu);
    track(v0);
    Fput(0, exp_neg(fmin(fabs(v0), kTanhMax)));
    adv(cu, 1);
    double va = load(cu);  // v_1
    adv(cu, 1);
    double vb = load(cu);  // v_2; cursor at slot 2
#pragma unroll
    for (int k = 1; k + 1 <= DC - 3; k += 2) {
        track(va);
        track(vb);
        Cur c1 = cu;
        adv(c1, 1);
        Cur c2 = c1;
        adv(c2, 1);
        const Tf2 o = tanh_fwd2<ARRAY>(Fget(k - 1), va, vb, c1.q, ref(c1), c2.q, ref(c2), post_lds, fl);
        Fput(k, o.f1);
        Fput(k + 1, o.f2);
        va = o.v1;
        vb = o.v2;
        cu = c2;
    }
    // va = v_{DC-2}, vb = v_{DC-1}; cursor at slot DC-1
    track(va);
    track(vb);
    if (!(amax < kTanhMax)) return false;  // the log-domain form redoes the check
    const double Flast = tanh_fwd1(Fget(DC - 3), va);  // F_{DC-2}
    // c2v_k = (parity of the other edges' flags) * magnitude: S ^ flag(v_k)
    auto sgn = [&](double v, double mag) { return (S ^ ((v > 0.0) ? 0u : 1u)) ? -mag : mag; };
    double B = exp_neg(fabs(vb));  // B_{DC-1}
    double *s1 = cu.q;             // pending: c2v_{DC-1}
    double w1 = sgn(vb, -log_unit(Flast));
    double *s2 = nullptr, w2 = 0.0;
    {
        static_assert((DC - 3) % 2 == 0, "DC odd");
        // the single step k = DC-2, then pairs (k, k-1) for even k = DC-3 .. 2
        Cur d = cu;
        adv(d, -1);
        va = load(d);  // v_{DC-2}
        Cur e1 = d;
        adv(e1, -1);
        Cur e2 = e1;
        adv(e2, -1);
        Tb2 o = tanh_bwd1l<ARRAY>(Fget(DC - 3), B, va, e1.q, ref(e1), e2.q, ref(e2), post_lds, s1, w1, fl);
        s1 = d.q;
        w1 = sgn(va, o.oa);  // c2v_{DC-2}
        B = o.b;             // B_{DC-2}
        va = o.v1;           // v_{DC-3}
        vb = o.v2;           // v_{DC-4}
        Cur d1 = e1, d2 = e2;
#pragma unroll
        for (int k = DC - 3; k >= 2; k -= 2) {
            Cur f1 = d2;
            adv(f1, -1);  // slot k-2
            Cur f2 = f1;
            if (k >= 3) adv(f2, -1);  // slot k-3 (k = 2: slot 0 again)
            o = tanh_bwd2c<ARRAY>(Fget(k - 2), B, va, vb, f1.q, ref(f1), f2.q, ref(f2), post_lds, s1, w1, s2, w2, fl);
            s1 = d1.q;
            w1 = sgn(va, o.oa);  // c2v_k
            s2 = d2.q;
            w2 = sgn(vb, o.ob);  // c2v_{k-1}
            B = o.b;             // B_{k-1}
            va = o.v1;
            vb = o.v2;
            d1 = f1;
            d2 = f2;
        }
        // pending c2v_2, c2v_1; va = v_0 (slot 0), B = B_1
        *s1 = w1;
        *s2 = w2;
        *d1.q = sgn(va, -log_unit(B));  // c2v_0 = B_1
        return true;
    }
}

// The tanh form for small check degrees (deg <= DC <= 16, e.g. 802.11n's 7 and 8): inlined, with
// the forward chain in registers; returns false (msg untouched) for a check with a message of
// magnitude >= kTanhMax.
template <int DC, bool REGULAR>
__device__ __forceinline__ bool check_update_tanh_small(double *msg, const double *s_post, const int32_t *cvar, int m,
                                                        int c, int deg, bool first) {
    if (REGULAR) deg = DC;
    auto v2c = [&](int k) {
        const double p = s_post[cvar[k * m + c]];
        return first ? p : __dsub_rn(p, msg[k * m + c]);
    };
    // the inputs' E = exp(-|v|) and sign flags are kept for the walk back (no second read and exp)
    uint32_t S = 0, neg = 0;
    double amax = 0.0;
    auto track = [&](double v, int k) {
        const uint32_t f = (v > 0.0) ? 0u : 1u;
        S ^= f;
        neg |= f << k;
        amax = fmax(amax, fabs(v));
    };
    double F[DC - 1], E[DC - 1];
    double v = v2c(0);
    track(v, 0);
    E[0] = F[0] = exp_neg(fmin(fabs(v), kTanhMax));
#pragma unroll
    for (int k = 1; k <= DC - 2; ++k)
        if (REGULAR || k <= deg - 2) {
            v = v2c(k);
            track(v, k);
            E[k] = exp_neg(fmin(fabs(v), kTanhMax));
            F[k] = bp_tanh(F[k - 1], E[k]);
        }
    double Flast = F[DC - 2];
    if (!REGULAR) {
#pragma unroll
        for (int k = 0; k <= DC - 2; ++k)
            if (k == deg - 2) Flast = F[k];
    }
    const double vl = v2c(deg - 1);
    const uint32_t fl = (vl > 0.0) ? 0u : 1u;
    S ^= fl;
    amax = fmax(amax, fabs(vl));
    if (!(amax < kTanhMax)) return false;
    // c2v_k = (parity of the other inputs' flags) * magnitude
    auto sgn = [&](uint32_t f, double mag) { return (S ^ f) ? -mag : mag; };
    double B = exp_neg(fabs(vl));
    msg[(deg - 1) * m + c] = sgn(fl, -log_unit(Flast));
#pragma unroll
    for (int k = DC - 2; k >= 1; --k) {
        if (!REGULAR && k > deg - 2) continue;
        msg[k * m + c] = sgn(neg >> k & 1u, -log_unit(bp_tanh(F[k - 1], B)));
        B = bp_tanh(B, E[k]);  // = exp_neg(|v_k|): |v_k| < kTanhMax here
    }
    msg[c] = sgn(neg & 1u, -log_unit(B));
    return true;
}

template <int DC, bool REGULAR, bool ARRAY>
__device__ __forceinline__ void check_update_reg(double *msg, const double *s_post, const int32_t *cvar, int m, int c,
                                                 int deg, bool first) {
    if (REGULAR && DC > 16) {
#if FPLDPC_FLOAT_TANH
        if constexpr (DC % 2 == 1) {
            if (check_update_tanh<DC, ARRAY>(msg, s_post, cvar, m, c, first)) return;
        }
#endif
        check_update_unrolled<DC>(msg, s_post, cvar, m, c, first);
        return;
    }
#if FPLDPC_FLOAT_TANH
    if (DC <= 16 && check_update_tanh_small<DC, REGULAR>(msg, s_post, cvar, m, c, deg, first)) return;
#endif
    if (REGULAR) deg = DC;
    auto v2c = [&](int k) {
        const double p = s_post[cvar[k * m + c]];
        return first ? p : __dsub_rn(p, msg[k * m + c]);
    };
    double F[DC - 1];
    F[0] = v2c(0);
#pragma unroll
    for (int k = 1; k <= DC - 2; ++k)
        if (REGULAR || k <= deg - 2) F[k] = sxor_f64(F[k - 1], v2c(k));
    double Flast = F[DC - 2];
    if (!REGULAR) {
#pragma unroll
        for (int k = 0; k <= DC - 2; ++k)
            if (k == deg - 2) Flast = F[k];
    }
    double B = v2c(deg - 1);
    msg[(deg - 1) * m + c] = Flast;
#pragma unroll
    for (int k = DC - 2; k >= 1; --k) {
        if (!REGULAR && k > deg - 2) continue;
        const double vk = v2c(k);
        msg[k * m + c] = sxor_f64(F[k - 1], B);
        B = sxor_f64(B, vk);
    }
    msg[c] = B;
}

// ARRAY: a forward array code of P = DC (detect_array): variable indices computed in the check phase
// and checkPost, edge addresses in the variable phase -- no [slot][check] / [row][variable] table
// loads in front of the LDS and c2v accesses (A 684 -> 783, R 35.6 -> 49.3 Mb/s: profiles/r4/ab/float_pair.txt)
// Small degrees (W): 7 workgroups per CU (72 VGPRs, a few spilled) -- the check phase waits on its
// table, LDS and c2v loads, and more frames in flight pay: 5 / 6 / 7 / 8 per CU measured 603 / 650 /
// 710 / 435 Mb/s on W (8: 117 VGPRs spilled), with the walk back's E values kept (at 7 per CU,
// recomputing them measured 655; profiles/r4/ab/w_float.txt)
template <int DC, bool REGULAR, bool ARRAY = false>
__global__ void __launch_bounds__(kFT, DC > 16 ? 4 : 7) bp_float_reg(FArgs a) {
    extern __shared__ double s_post[];
    __shared__ int s_frame, s_err;
    const int tid = threadIdx.x, n = a.n, m = a.m;
    double *msg = a.msg + (size_t)blockIdx.x * (size_t)a.dc * m;
    for (;;) {
        if (tid == 0) {
            s_frame = atomicAdd(a.counter, 1);
            s_err = 0;
        }
        __syncthreads();
        const int f = s_frame;
        if (f >= a.batch) break;  // uniform: every wave leaves
        const double *llr = a.llr + (size_t)f * n;
        for (int v = tid; v < n; v += kFT) s_post[v] = llr[v];  // v2c = LLR in the first check phase
        __syncthreads();
        int it = 0, fail = 1;
        while (it < a.max_iter) {
            for (int c = tid; c < m; c += kFT) check_update_reg<DC, REGULAR, ARRAY>(msg, s_post, a.cvar, m, c, a.cdeg[c], it == 0);
            __syncthreads();
            // variable phase (:888-910): post = (sum of c2v in vlist order) + LLR; v2c is not stored
            for (int v = tid; v < n; v += kFT) {
                const int dv = a.vdeg[v];
                double acc = 0.0;
                if constexpr (ARRAY) {
                    // variable v = P*kb + x sits in slot kb of the checks i*P + ((x - i*kb) mod P), rows
                    // ascending (its vlist order): edge kb*m + i*P + j
                    const int kb = v / DC, x = v - kb * DC;
                    const double *mk = msg + (size_t)kb * m;
                    int j = x;
                    for (int i = 0; i < dv; ++i) {
                        acc = __dadd_rn(acc, mk[i * DC + j]);
                        j -= kb;
                        j = j < 0 ? j + DC : j;
                    }
                } else {
                    for (int k = 0; k < dv; ++k) acc = __dadd_rn(acc, msg[a.vedge[(size_t)k * n + v]]);
                }
                s_post[v] = __dadd_rn(acc, llr[v]);
            }
            __syncthreads();
            ++it;
            int bad = 0;  // checkPost (:335-372)
            for (int c = tid; c < m && !bad; c += kFT) {
                int par = 0;
                const int deg = a.cdeg[c];
                if constexpr (ARRAY) {  // slot k of check i*P + j: variable k*P + (j + i*k) mod P
                    const int row = c / DC;
                    int x = c - row * DC;
                    for (int k = 0; k < DC; ++k) {
                        par ^= !(s_post[k * DC + x] > 0.0);
                        x += row;
                        x = x >= DC ? x - DC : x;
                    }
                } else {
                    for (int k = 0; k < deg; ++k) par ^= !(s_post[a.cvar[k * m + c]] > 0.0);
                }
                bad = par;
            }
            fail = __syncthreads_or(bad);
            if (!fail && a.early_term) break;
        }
        if (a.post)
            for (int v = tid; v < n; v += kFT) a.post[(size_t)f * n + v] = s_post[v];
        if (a.hard) {
            uint32_t *h = a.hard + (size_t)f * a.hard_words;
            const int lane = tid & 63, wave = tid >> 6;
            for (int base = wave * 64; base < n; base += kFT) {
                const int v = base + lane;
                const unsigned long long b = __ballot(v < n && !(s_post[v] > 0.0));
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
            for (int i = tid; i < a.k_info; i += kFT) e += (!(s_post[a.info_idx[i]] > 0.0) ? 1 : 0) != a.info_bits[i];
            if (e) atomicAdd(&s_err, e);
            __syncthreads();
            errors = s_err;
        }
        if (tid == 0) {
            if (a.iters) a.iters[f] = it;
            if (a.syn_ok) a.syn_ok[f] = (uint8_t)!fail;
            if (a.bit_errors) a.bit_errors[f] = errors;
            if (a.totals) {
                atomicAdd(&a.totals[0], (unsigned long long)errors);
                atomicAdd(&a.totals[1], (unsigned long long)(errors > 0));
                atomicAdd(&a.totals[2], 1ull);
                atomicAdd(&a.totals[3], (unsigned long long)it);
            }
        }
        __syncthreads();  // s_post / s_frame reuse
    }
}

__global__ void __launch_bounds__(kFT) bp_float_kernel(FArgs a) {
    extern __shared__ double s_post[];
    __shared__ int s_frame, s_err;
    const int tid = threadIdx.x, n = a.n, m = a.m;
    double *msg = a.msg + (size_t)blockIdx.x * 2 * (size_t)a.dc * m, *fwd = msg + (size_t)a.dc * m;
    for (;;) {
        if (tid == 0) {
            s_frame = atomicAdd(a.counter, 1);
            s_err = 0;
        }
        __syncthreads();
        const int f = s_frame;
        if (f >= a.batch) break;  // uniform: every wave leaves
        const double *llr = a.llr + (size_t)f * n;
        // edge init with the channel values (:762-778)
        for (int e = tid; e < a.dc * m; e += kFT) {
            const int v = a.cvar[e];
            if (v >= 0) msg[e] = llr[v];
        }
        __syncthreads();
        int it = 0, fail = 1;
        while (it < a.max_iter) {
            for (int c = tid; c < m; c += kFT) check_update(msg, fwd, m, c, a.cdeg[c]);
            __syncthreads();
            for (int v = tid; v < n; v += kFT) {
                const int dv = a.vdeg[v];
                double acc = 0.0;
                for (int k = 0; k < dv; ++k) acc = __dadd_rn(acc, msg[a.vedge[(size_t)k * n + v]]);
                acc = __dadd_rn(acc, llr[v]);
                s_post[v] = acc;
                for (int k = 0; k < dv; ++k) {
                    const int e = a.vedge[(size_t)k * n + v];
                    msg[e] = __dsub_rn(acc, msg[e]);
                }
            }
            __syncthreads();
            ++it;
            // checkPost (:335-372): hard = post > 0 ? 0 : 1, XOR over each check
            int bad = 0;
            for (int c = tid; c < m && !bad; c += kFT) {
                int par = 0;
                const int deg = a.cdeg[c];
                for (int k = 0; k < deg; ++k) par ^= !(s_post[a.cvar[k * m + c]] > 0.0);
                bad = par;
            }
            fail = __syncthreads_or(bad);
            if (!fail && a.early_term) break;
        }
        // epilogue (as the fixed-point kernels): posteriors, packed hard bits, BER, totals
        if (a.post)
            for (int v = tid; v < n; v += kFT) a.post[(size_t)f * n + v] = s_post[v];
        if (a.hard) {
            uint32_t *h = a.hard + (size_t)f * a.hard_words;
            const int lane = tid & 63, wave = tid >> 6;
            for (int base = wave * 64; base < n; base += kFT) {
                const int v = base + lane;
                const unsigned long long b = __ballot(v < n && !(s_post[v] > 0.0));
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
            for (int i = tid; i < a.k_info; i += kFT) e += (!(s_post[a.info_idx[i]] > 0.0) ? 1 : 0) != a.info_bits[i];
            if (e) atomicAdd(&s_err, e);
            __syncthreads();
            errors = s_err;
        }
        if (tid == 0) {
            if (a.iters) a.iters[f] = it;
            if (a.syn_ok) a.syn_ok[f] = (uint8_t)!fail;
            if (a.bit_errors) a.bit_errors[f] = errors;
            if (a.totals) {
                atomicAdd(&a.totals[0], (unsigned long long)errors);
                atomicAdd(&a.totals[1], (unsigned long long)(errors > 0));
                atomicAdd(&a.totals[2], 1ull);
                atomicAdd(&a.totals[3], (unsigned long long)it);
            }
        }
        __syncthreads();  // s_post / s_frame reuse
    }
}

#define F_TRY(expr)                                            \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return fail_hip((int)_e, #expr); \
    } while (0)

int float_setup(fpldpc_decoder *dec) {
    if (dec->fl) return FPLDPC_OK;
    const fpldpc_code &H = dec->code;
    if (H.n > kMaxFloatN) return fail(FPLDPC_ERR_UNSUPPORTED, "float decoder: n > 16384");
    if (H.dc_max > 255) return fail(FPLDPC_ERR_UNSUPPORTED, "float decoder: check degree > 255");
    if (H.dv_max > 255) return fail(FPLDPC_ERR_UNSUPPORTED, "float decoder: variable degree > 255");
    std::unique_ptr<FloatState> s(new FloatState());
    s->device = dec->device;
    const int n = H.n, m = H.m, dc = H.dc_max, dv = H.dv_max;
    int min_dc = dc;
    for (int c = 0; c < m; c++) min_dc = std::min(min_dc, (int)H.cdeg[c]);
    // register forms (c2v the only state, forward chain in registers) for the codes' degree
    // envelopes; the generic kernel (v2c and forward-chain planes in the scratch) otherwise
    s->planes = 1;
    if (dc == 47 && min_dc == 47) {
        s->fn = H.array_forward ? bp_float_reg<47, true, true> : bp_float_reg<47, true>;
    } else if (dc <= 8 && min_dc >= 2) {
        s->fn = bp_float_reg<8, false>;
    } else {
        s->fn = bp_float_kernel;
        s->planes = 2;
    }
    std::vector<int32_t> cvar((size_t)dc * m, -1), vedge((size_t)dv * n, 0);
    std::vector<uint8_t> cdeg(m), vdeg(n);
    for (int c = 0; c < m; c++) {
        cdeg[c] = (uint8_t)H.cdeg[c];
        for (int k = 0; k < H.cdeg[c]; k++) cvar[(size_t)k * m + c] = H.clist[(size_t)c * dc + k];
    }
    // EdgeRAM bank of (v, k) = addr_count[c] at the time v is visited (:903-919): the rank of v in
    // clist[c] for ascending rows (validated by code_finalize)
    std::vector<int> addr_count(m, 0);
    for (int v = 0; v < n; v++) {
        vdeg[v] = (uint8_t)H.vdeg[v];
        for (int k = 0; k < H.vdeg[v]; k++) {
            const int c = H.vlist[(size_t)v * dv + k];
            vedge[(size_t)k * n + v] = addr_count[c]++ * m + c;
        }
    }
    hipDeviceProp_t prop;
    F_TRY(hipGetDeviceProperties(&prop, dec->device));
    s->lds = sizeof(double) * (size_t)n;
    if (s->lds > 64 * 1024) F_TRY(hipFuncSetAttribute((const void *)s->fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->lds));
    int per_cu = 0;
    F_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)s->fn, kFT, s->lds));
    if (per_cu < 1) return fail(FPLDPC_ERR_UNSUPPORTED, "float decoder: kernel does not fit a CU");
    // Diagnostic: FPLDPC_FLOAT_WG_PER_CU=k caps the persistent grid (the edge scratch is per workgroup)
    if (const char *g = getenv("FPLDPC_FLOAT_WG_PER_CU"))
        if (atoi(g) > 0) per_cu = std::min(per_cu, atoi(g));
    s->grid = per_cu * prop.multiProcessorCount;
    F_TRY(hipMalloc(&s->d_cvar, sizeof(int32_t) * cvar.size()));
    F_TRY(hipMalloc(&s->d_cdeg, m));
    F_TRY(hipMalloc(&s->d_vedge, sizeof(int32_t) * std::max<size_t>(vedge.size(), 1)));
    F_TRY(hipMalloc(&s->d_vdeg, n));
    F_TRY(hipMalloc(&s->d_msg, sizeof(double) * s->planes * (size_t)s->grid * dc * m));
    F_TRY(hipMalloc(&s->d_counter, sizeof(int)));
    F_TRY(hipMemcpy(s->d_cvar, cvar.data(), sizeof(int32_t) * cvar.size(), hipMemcpyHostToDevice));
    F_TRY(hipMemcpy(s->d_cdeg, cdeg.data(), m, hipMemcpyHostToDevice));
    F_TRY(hipMemcpy(s->d_vedge, vedge.data(), sizeof(int32_t) * vedge.size(), hipMemcpyHostToDevice));
    F_TRY(hipMemcpy(s->d_vdeg, vdeg.data(), n, hipMemcpyHostToDevice));
    dec->fl = s.release();
    return FPLDPC_OK;
}

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

}  // namespace
}  // namespace fpldpc

using namespace fpldpc;

extern "C" {

int fpldpc_decode_float(fpldpc_decoder_t dec, const double *llr, int32_t batch, uint32_t *hard, int32_t *iters,
                        uint8_t *syndrome_ok, double *post, int32_t *bit_errors, int64_t *totals, void *stream) {
    if (!dec) return fail(FPLDPC_ERR_ARG, "null decoder");
    if (batch < 0) return fail(FPLDPC_ERR_ARG, "negative batch");
    if (batch == 0) return FPLDPC_OK;
    if (!llr) return fail(FPLDPC_ERR_ARG, "null llr");
    if (bit_errors && dec->k_info == 0) return fail(FPLDPC_ERR_ARG, "bit_errors requested without fpldpc_set_reference");
    Guard g(dec->device);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    int st = float_setup(dec);
    if (st) return st;
    FloatState *s = dec->fl;
    hipStream_t hs = (hipStream_t)stream;
    F_TRY(hipMemsetAsync(s->d_counter, 0, sizeof(int), hs));
    FArgs a{};
    a.llr = llr;
    a.batch = batch;
    a.n = dec->code.n;
    a.m = dec->code.m;
    a.dc = dec->code.dc_max;
    a.dv = dec->code.dv_max;
    a.max_iter = dec->params.max_iter;
    a.early_term = dec->params.early_term;
    a.cvar = s->d_cvar;
    a.cdeg = s->d_cdeg;
    a.vedge = s->d_vedge;
    a.vdeg = s->d_vdeg;
    a.msg = s->d_msg;
    a.counter = s->d_counter;
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
    const int grid = std::min(s->grid, batch);
    hipLaunchKernelGGL(s->fn, dim3(grid), dim3(kFT), s->lds, hs, a);
    F_TRY(hipGetLastError());
    return FPLDPC_OK;
}

int fpldpc_decode_float_host(fpldpc_decoder_t dec, const double *llr, int32_t batch, uint32_t *hard, int32_t *iters,
                             uint8_t *syndrome_ok, double *post, int32_t *bit_errors, int64_t *totals) {
    if (!dec) return fail(FPLDPC_ERR_ARG, "null decoder");
    if (batch < 0) return fail(FPLDPC_ERR_ARG, "negative batch");
    if (batch == 0) return FPLDPC_OK;
    if (!llr) return fail(FPLDPC_ERR_ARG, "null llr");
    Guard g(dec->device);
    if (!g.ok) return fail(FPLDPC_ERR_HIP, "hipSetDevice failed");
    const size_t n = dec->code.n, B = batch, hw = (n + 31) / 32;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_llr = 0, o_hard = al(B * n * 8), o_it = o_hard + al(B * hw * 4), o_ok = o_it + al(B * 4),
                 o_post = o_ok + al(B), o_be = o_post + al(post ? B * n * 8 : 0), o_tot = o_be + al(B * 4),
                 total = o_tot + 64;
    char *d = nullptr;
    F_TRY(hipMalloc((void **)&d, total));
    struct Free {
        char *p;
        ~Free() { (void)hipFree(p); }
    } fr{d};
    hipStream_t hs = nullptr;
    F_TRY(hipMemcpy(d + o_llr, llr, B * n * 8, hipMemcpyHostToDevice));
    int64_t *d_tot = totals ? reinterpret_cast<int64_t *>(d + o_tot) : nullptr;
    if (totals) F_TRY(hipMemcpy(d_tot, totals, 32, hipMemcpyHostToDevice));
    int st = fpldpc_decode_float(dec, reinterpret_cast<const double *>(d + o_llr), batch,
                                 hard ? reinterpret_cast<uint32_t *>(d + o_hard) : nullptr,
                                 iters ? reinterpret_cast<int32_t *>(d + o_it) : nullptr,
                                 syndrome_ok ? reinterpret_cast<uint8_t *>(d + o_ok) : nullptr,
                                 post ? reinterpret_cast<double *>(d + o_post) : nullptr,
                                 bit_errors ? reinterpret_cast<int32_t *>(d + o_be) : nullptr, d_tot, hs);
    if (st) return st;
    F_TRY(hipDeviceSynchronize());
    if (hard) F_TRY(hipMemcpy(hard, d + o_hard, B * hw * 4, hipMemcpyDeviceToHost));
    if (iters) F_TRY(hipMemcpy(iters, d + o_it, B * 4, hipMemcpyDeviceToHost));
    if (syndrome_ok) F_TRY(hipMemcpy(syndrome_ok, d + o_ok, B, hipMemcpyDeviceToHost));
    if (post) F_TRY(hipMemcpy(post, d + o_post, B * n * 8, hipMemcpyDeviceToHost));
    if (bit_errors) F_TRY(hipMemcpy(bit_errors, d + o_be, B * 4, hipMemcpyDeviceToHost));
    if (totals) F_TRY(hipMemcpy(totals, d_tot, 32, hipMemcpyDeviceToHost));
    return FPLDPC_OK;
}

}  // extern "C"
