// Dependent-issue micro-benchmark (diagnostic only): cycles per VALU instruction for C independent
// dependency chains in one wave, with WPS waves per SIMD, measured with s_memtime inside the kernel.
// Tells how much instruction-level parallelism a wave needs to keep the VALU busy on gfx950
// (the decoder's box-plus chains are serial).
#include <hip/hip_runtime.h>
#include <cstdio>

#define A1(r) "v_add_u32 " r ", " r ", %[b]\n\t"
#define PKM1(r) "v_pk_min_u16 " r ", " r ", %[b]\n\t"

template <int C, int PK>
__global__ void __launch_bounds__(256) kern(unsigned *out, unsigned long long *cyc, int iters) {
    unsigned x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    const unsigned b = blockIdx.x | 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (PK == 0) {
                if (C == 1) asm volatile(A1("%0") A1("%0") A1("%0") A1("%0") A1("%0") A1("%0") A1("%0") A1("%0") : "+v"(x0) : [b] "v"(b));
                if (C == 2) asm volatile(A1("%0") A1("%1") A1("%0") A1("%1") A1("%0") A1("%1") A1("%0") A1("%1") : "+v"(x0), "+v"(x1) : [b] "v"(b));
                if (C == 4) asm volatile(A1("%0") A1("%1") A1("%2") A1("%3") A1("%0") A1("%1") A1("%2") A1("%3") : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : [b] "v"(b));
                if (C == 8) asm volatile(A1("%0") A1("%1") A1("%2") A1("%3") A1("%4") A1("%5") A1("%6") A1("%7") : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : [b] "v"(b));
            } else {
                if (C == 1) asm volatile(PKM1("%0") PKM1("%0") PKM1("%0") PKM1("%0") PKM1("%0") PKM1("%0") PKM1("%0") PKM1("%0") : "+v"(x0) : [b] "v"(b));
                if (C == 2) asm volatile(PKM1("%0") PKM1("%1") PKM1("%0") PKM1("%1") PKM1("%0") PKM1("%1") PKM1("%0") PKM1("%1") : "+v"(x0), "+v"(x1) : [b] "v"(b));
                if (C == 4) asm volatile(PKM1("%0") PKM1("%1") PKM1("%2") PKM1("%3") PKM1("%0") PKM1("%1") PKM1("%2") PKM1("%3") : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : [b] "v"(b));
                if (C == 8) asm volatile(PKM1("%0") PKM1("%1") PKM1("%2") PKM1("%3") PKM1("%4") PKM1("%5") PKM1("%6") PKM1("%7") : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : [b] "v"(b));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int C, int PK>
void run(unsigned *out, unsigned long long *cyc, int wps) {
    const int blocks = 256 * wps, iters = 256;
    kern<C, PK><<<blocks, 256>>>(out, cyc, 4);
    kern<C, PK><<<blocks, 256>>>(out, cyc, iters);
    (void)hipDeviceSynchronize();
    unsigned long long h[256 * 8];
    (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double s = 0, mn = 1e30, mx = 0;
    for (int i = 0; i < blocks; ++i) {
        s += (double)h[i];
        mn = h[i] < mn ? (double)h[i] : mn;
        mx = h[i] > mx ? (double)h[i] : mx;
    }
    const double per_wave_instr = (double)iters * 16 * 8;
    printf("%-12s chains=%d waves/SIMD=%d  cycles per instruction per wave %.2f (fastest %.2f, slowest %.2f)  -> per SIMD %.2f\n",
           PK ? "v_pk_min_u16" : "v_add_u32", C, wps, s / blocks / per_wave_instr, mn / per_wave_instr, mx / per_wave_instr,
           s / blocks / per_wave_instr / wps);
}

int main() {
    unsigned *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, sizeof(unsigned) * 256 * 8 * 256) != hipSuccess) return 1;
    if (hipMalloc(&cyc, sizeof(unsigned long long) * 256 * 8) != hipSuccess) return 1;
    for (int wps : {1, 2, 3, 4}) {
        run<1, 0>(out, cyc, wps);
        run<2, 0>(out, cyc, wps);
        run<4, 0>(out, cyc, wps);
        run<8, 0>(out, cyc, wps);
        run<1, 1>(out, cyc, wps);
        run<2, 1>(out, cyc, wps);
        run<4, 1>(out, cyc, wps);
        run<8, 1>(out, cyc, wps);
    }
    return 0;
}
