// fpldpc_float_math.hpp -- the float decoder's box-plus transcendentals (fpldpc_float.hip), shared
// with the bit-exactness check tools/float_exp_check.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace fpldpc {

// a * b + c with the constant c in an SGPR pair (VOP3 v_fma_f64): the compiler otherwise writes a
// 64-bit constant addend into VGPRs with two v_mov_b32 before each v_fmac_f64 -- VALU issue slots
// that the box-plus's exp / log polynomials spent as many of as on their FMAs.  The SGPR pair is
// loaded by scalar moves, which issue beside the VALU.
__device__ __forceinline__ double fma_sc(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}
// exp(-x) for 0 <= x < kLogUlp: the device libm's exp(double) sequence, operation for operation
// (k = rint(-x / ln2), r = -x - k ln2 in two parts, a degree-12 polynomial in Horner form, then
// 2^k), with its polynomial's constant addends in SGPRs (fma_sc).  No range handling is needed on
// this interval, so the result is bit for bit the libm's (tools/float_exp_check.hip).
__device__ __forceinline__ double exp_neg(double x) {
    const double k = __builtin_rint(__dmul_rn(x, -0x1.71547652b82fep+0));
    double r = fma(k, -0x1.62e42fefa39efp-1, -x);
    r = fma(-0x1.abc9e3b39803fp-56, k, r);
    double p = fma(0x1.ade156a5dcb37p-26, r, 0x1.28af3fca7ab0cp-22);
    p = fma_sc(r, p, 0x1.71dee623fde64p-19);
    p = fma_sc(r, p, 0x1.a01997c89e6b0p-16);
    p = fma_sc(r, p, 0x1.a01a014761f6ep-13);
    p = fma_sc(r, p, 0x1.6c16c1852b7b0p-10);
    p = fma_sc(r, p, 0x1.1111111122322p-7);
    p = fma_sc(r, p, 0x1.55555555502a1p-5);
    p = fma_sc(r, p, 0x1.5555555555511p-3);
    p = fma_sc(r, p, 0x1.000000000000bp-1);
    p = fma(r, p, 1.0);
    p = fma(r, p, 1.0);
    return __builtin_amdgcn_ldexp(p, (int)k);
}
// log(y) for y in [1, 2] (the argument is 1 + exp(-x)): the fdlibm algorithm (e_log.c: k = 0 / 1 by
// y against sqrt 2, f = m - 1 exact, s = f / (2 + f), log = k ln2 + f - hfsq + s (hfsq + R(s^2)))
// without its range reduction and special cases, the division as v_rcp_f64 with Newton steps and
// the polynomials in FMA form.  Within 1 ulp of the correctly rounded log, and equal to glibc's log
// for 99.1 % of arguments of the form 1 + exp(-x), x in [0, 36.75] (2e7 samples, host emulation of
// this code); the device libm's log costs 3.3x as many SIMD cycles (tools/ubench/f64_rate.hip:
// 364 cycles per wave-call at 4 waves per SIMD, against ~110 here).
__device__ __forceinline__ double log_1to2(double y) {
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                     Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                     Lg7 = 1.479819860511658591e-01;
    const bool hi = y > 1.4142135623730951;
    const double f = hi ? __dsub_rn(__dmul_rn(y, 0.5), 1.0) : __dsub_rn(y, 1.0);  // exact (Sterbenz)
    const double k = hi ? 1.0 : 0.0;
    const double d = __dadd_rn(2.0, f);
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    double s = __dmul_rn(f, r);
    s = fma(fma(-d, s, f), r, s);
    const double z = __dmul_rn(s, s), w = __dmul_rn(z, z);
    const double t1 = __dmul_rn(w, fma_sc(w, fma(w, Lg6, Lg4), Lg2));
    const double t2 = __dmul_rn(z, fma_sc(w, fma_sc(w, fma(w, Lg7, Lg5), Lg3), Lg1));
    const double R = __dadd_rn(t2, t1);
    const double hfsq = __dmul_rn(__dmul_rn(0.5, f), f);
    return fma(k, ln2_hi, -__dsub_rn(__dsub_rn(hfsq, fma(s, __dadd_rn(hfsq, R), __dmul_rn(k, ln2_lo))), f));
}

// log(x) for x in [2^-1022, 1] (the tanh-domain check update's outputs, fpldpc_float.hip): x = y 2^e
// with y in [1, 2) (v_frexp), then log_1to2's fdlibm kernel with the exponent folded into its k.
__device__ __forceinline__ double log_unit(double x) {
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                     Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                     Lg7 = 1.479819860511658591e-01;
    const int e = __builtin_amdgcn_frexp_exp(x) - 1;             // x = y 2^e, y = 2 * mant in [1, 2)
    const double y = __dmul_rn(__builtin_amdgcn_frexp_mant(x), 2.0);
    const bool hi = y > 1.4142135623730951;
    const double f = hi ? __dsub_rn(__dmul_rn(y, 0.5), 1.0) : __dsub_rn(y, 1.0);  // exact (Sterbenz)
    const double k = (double)(e + (hi ? 1 : 0));
    const double d = __dadd_rn(2.0, f);
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    double s = __dmul_rn(f, r);
    s = fma(fma(-d, s, f), r, s);
    const double z = __dmul_rn(s, s), w = __dmul_rn(z, z);
    const double t1 = __dmul_rn(w, fma_sc(w, fma(w, Lg6, Lg4), Lg2));
    const double t2 = __dmul_rn(z, fma_sc(w, fma_sc(w, fma(w, Lg7, Lg5), Lg3), Lg1));
    const double R = __dadd_rn(t2, t1);
    const double hfsq = __dmul_rn(__dmul_rn(0.5, f), f);
    return fma(k, ln2_hi, -__dsub_rn(__dsub_rn(hfsq, fma(s, __dadd_rn(hfsq, R), __dmul_rn(k, ln2_lo))), f));
}
// a / b for b in [1, 2] (the tanh-domain box-plus's 1 + E_a E_b): v_rcp_f64, two Newton steps and a
// final correction of the quotient (within an ulp; the IEEE division sequence costs twice as much)
__device__ __forceinline__ double div_1to2(double a, double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    r = fma(fma(-b, r, 1.0), r, r);
    const double q = __dmul_rn(a, r);
    return fma(fma(-b, q, a), r, q);
}

}  // namespace fpldpc
