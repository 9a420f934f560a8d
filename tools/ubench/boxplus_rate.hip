// Box-plus chain micro-benchmark (diagnostic only): the packed kernel's bp_mag2 step
// (3 v_pk_min_u16 + 8 full-rate ops, as in fpldpc_kernels.hip) iterated in C independent chains
// per lane, WPS waves per SIMD on every CU; reports shader cycles (s_memtime) per VALU
// instruction per SIMD.  Compared with the v_add / v_pk_min rates of dep_latency.hip it shows
// what the decoder's own instruction mix can issue at.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 U2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t W(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t sub2x(uint32_t a, uint32_t x) {
    uint32_t r;
    asm("v_sub_u32 %0, %1, %2\n\tv_sub_u32 %0, %0, %2" : "=&v"(r) : "v"(a), "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t bp_mag2(uint32_t a, uint32_t b, u16x2 C2, uint32_t M2) {
    const uint32_t mn = W(__builtin_elementwise_min(U2(a), U2(b)));
    const uint32_t s = a + b;
    const uint32_t d = sub2x(s, mn);
    const uint32_t q1 = W(__builtin_elementwise_min(U2((s >> 2) & M2), C2));
    const uint32_t q2 = W(__builtin_elementwise_min(U2((d >> 2) & M2), C2));
    return mn + q2 - q1;
}

template <int C, int PAD = 0>
__global__ void __launch_bounds__(256) kern(uint32_t *out, unsigned long long *cyc, int iters, uint32_t seed) {
    uint32_t x[C], y[C];
    uint32_t pad[PAD > 0 ? PAD : 1];  // PAD extra live VGPRs (the decoder holds ~160)
#pragma unroll
    for (int i = 0; i < (PAD > 0 ? PAD : 1); ++i) pad[i] = threadIdx.x * (i + 3);
#pragma unroll
    for (int i = 0; i < (PAD > 0 ? PAD : 1); ++i) asm volatile("" : "+v"(pad[i]));
#pragma unroll
    for (int c = 0; c < C; ++c) {
        x[c] = (threadIdx.x * 2654435761u + c * 40503u + seed) & 0x0fff0fffu;
        y[c] = (threadIdx.x * 2246822519u + c * 9973u + seed) & 0x0fff0fffu;
    }
    const u16x2 C2 = (u16x2)(unsigned short)10;
    const uint32_t M2 = 0x003f003fu;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = bp_mag2(x[c], y[c] ^ (uint32_t)r, C2, M2) + 3u;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) acc ^= x[c];
#pragma unroll
    for (int i = 0; i < (PAD > 0 ? PAD : 1); ++i) asm volatile("" : "+v"(pad[i]));
#pragma unroll
    for (int i = 0; i < (PAD > 0 ? PAD : 1); ++i) acc ^= pad[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int C, int PAD = 0>
void run(uint32_t *out, unsigned long long *cyc, int wps) {
    const int blocks = 256 * wps, iters = 64;
    kern<C, PAD><<<blocks, 256>>>(out, cyc, 4, 1);
    kern<C, PAD><<<blocks, 256>>>(out, cyc, iters, 7);
    (void)hipDeviceSynchronize();
    static unsigned long long h[256 * 8];
    (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += (double)h[i];
    // VALU per bp_mag2 step as compiled: 3 pk_min + mn+s, 2 sub, 2 shr, 2 and, add, sub + xor(r) + add(3) = 15
    const double valu = (double)iters * 16 * C * 15;
    printf("bp_mag2 chains=%d pad=%3d waves/SIMD=%d  cycles per VALU per SIMD %.2f (per wave %.2f)\n", C, PAD, wps,
           s / blocks / valu / wps, s / blocks / valu);
}

int main() {
    uint32_t *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, sizeof(uint32_t) * 256 * 8 * 256) != hipSuccess) return 1;
    if (hipMalloc(&cyc, sizeof(unsigned long long) * 256 * 8) != hipSuccess) return 1;
    for (int wps : {1, 2, 3, 4}) {
        run<1>(out, cyc, wps);
        run<2>(out, cyc, wps);
        run<4>(out, cyc, wps);
    }
    for (int wps : {1, 3}) {
        run<2, 64>(out, cyc, wps);
        run<2, 140>(out, cyc, wps);
    }
    return 0;
}
