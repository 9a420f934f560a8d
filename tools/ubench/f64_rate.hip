// FP64 VALU throughput per SIMD (diagnostic only; the float decoder's roofline, fpldpc_float.hip),
// measured as an aggregate like op_rate.hip: every wave runs the same instruction stream, 8
// independent chains per lane; rate = wave-instructions per SIMD / span (first wave's start to the
// last wave's end), W waves per SIMD.  Also the device libm calls the box-plus makes (exp, log of a
// double: OCML software sequences), per call, and v_add_u32 as the 2-cycle reference.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#define D8 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define F2(OP) asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t" OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t" \
                            OP " %4, %4, %8\n\t" OP " %5, %5, %8\n\t" OP " %6, %6, %8\n\t" OP " %7, %7, %8" : D8 : "v"(b))
#define F3(OP) asm volatile(OP " %0, %0, %8, %8\n\t" OP " %1, %1, %8, %8\n\t" OP " %2, %2, %8, %8\n\t" OP " %3, %3, %8, %8\n\t" \
                            OP " %4, %4, %8, %8\n\t" OP " %5, %5, %8, %8\n\t" OP " %6, %6, %8, %8\n\t" OP " %7, %7, %8, %8" : D8 : "v"(b))
#define F1(OP) asm volatile(OP " %0, %0\n\t" OP " %1, %1\n\t" OP " %2, %2\n\t" OP " %3, %3\n\t" \
                            OP " %4, %4\n\t" OP " %5, %5\n\t" OP " %6, %6\n\t" OP " %7, %7" : D8)

template <int K>
__global__ void __launch_bounds__(256) kern(double *out, unsigned long long *t, int iters) {
    double a0 = threadIdx.x * 1e-3 + 0.5, a1 = a0 + 0.01, a2 = a0 + 0.02, a3 = a0 + 0.03, a4 = a0 + 0.04, a5 = a0 + 0.05,
           a6 = a0 + 0.06, a7 = a0 + 0.07;
    double b = 1.0 + blockIdx.x * 1e-9;
    unsigned u0 = threadIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3, u4 = u0 + 4, u5 = u0 + 5, u6 = u0 + 6, u7 = u0 + 7;
    const unsigned ub = blockIdx.x | 1;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if (K == 0)
            for (int r = 0; r < 4; ++r)
                asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                             "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                             : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(ub));
        if (K == 1) { F3("v_fma_f64"); F3("v_fma_f64"); F3("v_fma_f64"); F3("v_fma_f64"); }
        if (K == 2) { F2("v_add_f64"); F2("v_add_f64"); F2("v_add_f64"); F2("v_add_f64"); }
        if (K == 3) { F2("v_mul_f64"); F2("v_mul_f64"); F2("v_mul_f64"); F2("v_mul_f64"); }
        if (K == 4) { F1("v_rcp_f64"); F1("v_rcp_f64"); F1("v_rcp_f64"); F1("v_rcp_f64"); }
        if (K == 5) { F2("v_min_f64"); F2("v_min_f64"); F2("v_min_f64"); F2("v_min_f64"); }
        if (K == 6) { F1("v_frexp_mant_f64"); F1("v_frexp_mant_f64"); F1("v_frexp_mant_f64"); F1("v_frexp_mant_f64"); }
        if (K == 7) {  // libm exp(double): 8 independent calls per iteration (32 "instructions" counted as 8 calls x 4)
            a0 = exp(-a0); a1 = exp(-a1); a2 = exp(-a2); a3 = exp(-a3); a4 = exp(-a4); a5 = exp(-a5); a6 = exp(-a6); a7 = exp(-a7);
        }
        if (K == 8) {  // libm log(double)
            a0 = log(1.5 + a0); a1 = log(1.5 + a1); a2 = log(1.5 + a2); a3 = log(1.5 + a3);
            a4 = log(1.5 + a4); a5 = log(1.5 + a5); a6 = log(1.5 + a6); a7 = log(1.5 + a7);
        }
        if (K == 9) {  // the reference's correction term log(1 + exp(-x))
            a0 = log(1 + exp(-a0)); a1 = log(1 + exp(-a1)); a2 = log(1 + exp(-a2)); a3 = log(1 + exp(-a3));
            a4 = log(1 + exp(-a4)); a5 = log(1 + exp(-a5)); a6 = log(1 + exp(-a6)); a7 = log(1 + exp(-a7));
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (double)(u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7);
    if (threadIdx.x == 0) {
        t[4 * blockIdx.x] = c0;
        t[4 * blockIdx.x + 1] = c1;
        t[4 * blockIdx.x + 2] = r0;
        t[4 * blockIdx.x + 3] = r1;
    }
}

typedef void (*Fn)(double *, unsigned long long *, int);
template <int K> void add(Fn *f) { f[K] = kern<K>; add<K - 1>(f); }
template <> void add<-1>(Fn *) {}

int main() {
    const int N = 10;
    const char *names[N] = {"v_add_u32", "v_fma_f64", "v_add_f64", "v_mul_f64", "v_rcp_f64", "v_min_f64",
                            "v_frexp_mant_f64", "exp(double) call", "log(double) call", "log(1+exp(-x)) call"};
    Fn f[N];
    add<N - 1>(f);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double *out;
    unsigned long long *t;
    (void)hipMalloc(&out, sizeof(double) * 256 * 4 * cus);
    (void)hipMalloc(&t, sizeof(unsigned long long) * 4 * 4 * cus);
    std::vector<unsigned long long> h(4 * 4 * cus);
    for (int k = 0; k < N; ++k)
        for (int w : {1, 2, 4}) {
            const int iters = k >= 7 ? 200 : 2000;
            const int blocks = cus * w;
            f[k]<<<blocks, 256>>>(out, t, 10);
            f[k]<<<blocks, 256>>>(out, t, iters);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            (void)hipMemcpy(h.data(), t, sizeof(unsigned long long) * 4 * blocks, hipMemcpyDeviceToHost);
            unsigned long long rmin = ~0ull, rmax = 0;
            double cyc = 0, real = 0;
            for (int i = 0; i < blocks; ++i) {
                rmin = std::min(rmin, h[4 * i + 2]);
                rmax = std::max(rmax, h[4 * i + 3]);
                cyc += (double)(h[4 * i + 1] - h[4 * i]);
                real += (double)(h[4 * i + 3] - h[4 * i + 2]);
            }
            const double ghz = cyc / real / 10.0;
            const double span = (double)(rmax - rmin) * 10.0 * ghz;
            const double per_simd = (double)w * iters * (k >= 7 ? 8 : 32);  // calls or instructions per SIMD
            printf("%-22s waves/SIMD=%d  cycles per wave-%s per SIMD %.2f  (clock %.2f GHz)\n", names[k], w,
                   k >= 7 ? "call" : "instruction", span / per_simd, ghz);
        }
    return 0;
}
