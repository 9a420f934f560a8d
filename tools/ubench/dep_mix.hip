// Dependent mixed-type VALU chains (diagnostic only): does a full-rate op that consumes a v_pk_*
// result (or the reverse) issue later than either type alone, and do VGPR bank conflicts (source
// operands in the same bank, reg % 4) cost issue cycles?  Shader cycles per VALU per SIMD,
// WPS waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

// K: 0 = chain add->pk->add->pk (dependent), 1 = two independent chains (add chain, pk chain)
//    2 = add chain with sources in the same bank (v_add a, a, b with b = a + 4 registers apart)
//    3 = add chain with sources in different banks
template <int K>
__global__ void __launch_bounds__(256) kern(unsigned *out, unsigned long long *cyc, int iters) {
    unsigned x = threadIdx.x, y = threadIdx.x * 3 + 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (K == 0)
                asm volatile("v_add_u32 %0, %0, %1\n\tv_pk_min_u16 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_pk_min_u16 %0, %0, %1\n\t"
                             "v_add_u32 %0, %0, %1\n\tv_pk_min_u16 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_pk_min_u16 %0, %0, %1"
                             : "+v"(x) : "v"(y));
            if (K == 1)
                asm volatile("v_add_u32 %0, %0, %2\n\tv_pk_min_u16 %1, %1, %2\n\tv_add_u32 %0, %0, %2\n\tv_pk_min_u16 %1, %1, %2\n\t"
                             "v_add_u32 %0, %0, %2\n\tv_pk_min_u16 %1, %1, %2\n\tv_add_u32 %0, %0, %2\n\tv_pk_min_u16 %1, %1, %2"
                             : "+v"(x), "+v"(y) : "v"(y ^ 5));
            if (K == 2)
                asm volatile("v_add_u32 v40, v40, v44\n\tv_add_u32 v40, v40, v44\n\tv_add_u32 v40, v40, v44\n\tv_add_u32 v40, v40, v44\n\t"
                             "v_add_u32 v40, v40, v44\n\tv_add_u32 v40, v40, v44\n\tv_add_u32 v40, v40, v44\n\tv_add_u32 v40, v40, v44" ::: "v40", "v44");
            if (K == 3)
                asm volatile("v_add_u32 v40, v41, v42\n\tv_add_u32 v40, v41, v42\n\tv_add_u32 v40, v41, v42\n\tv_add_u32 v40, v41, v42\n\t"
                             "v_add_u32 v40, v41, v42\n\tv_add_u32 v40, v41, v42\n\tv_add_u32 v40, v41, v42\n\tv_add_u32 v40, v41, v42" ::: "v40", "v41", "v42");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x ^ y;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char *name, unsigned *out, unsigned long long *cyc, int wps) {
    const int blocks = 256 * wps, iters = 256;
    kern<K><<<blocks, 256>>>(out, cyc, 4);
    kern<K><<<blocks, 256>>>(out, cyc, iters);
    (void)hipDeviceSynchronize();
    static unsigned long long h[256 * 8];
    (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += (double)h[i];
    printf("%-34s waves/SIMD=%d  cycles per VALU per SIMD %.2f\n", name, wps, s / blocks / (iters * 16 * 8.0) / wps);
}

int main() {
    unsigned *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, sizeof(unsigned) * 256 * 8 * 256) != hipSuccess) return 1;
    if (hipMalloc(&cyc, sizeof(unsigned long long) * 256 * 8) != hipSuccess) return 1;
    for (int wps : {1, 3}) {
        run<0>("add->pk->add dependent chain", out, cyc, wps);
        run<1>("add chain || pk chain interleaved", out, cyc, wps);
        run<2>("add, sources same bank", out, cyc, wps);
        run<3>("add, sources different banks", out, cyc, wps);
    }
    return 0;
}
