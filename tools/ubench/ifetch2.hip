// Instruction-fetch micro-benchmark, desynchronised waves (diagnostic only).  ifetch.hip ran every
// wave through the same straight-line body at about the same place; the decoder's waves (three
// workgroups per CU) sit at different places of a ~14 KB step body.  Here each wave enters its
// unrolled body at a different group (Duff's device), so the waves of a CU fetch from different
// lines, for bodies of 8-byte full-rate instructions (v_and_b32 with a literal) of 8 to 64 KiB.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define ANDK8 asm volatile("v_and_b32 %0, 0x7fff7fff, %0\n\tv_and_b32 %1, 0x7fff7fff, %1\n\tv_and_b32 %2, 0x7fff7fff, %2\n\tv_and_b32 %3, 0x7fff7fff, %3\n\t" \
                           "v_and_b32 %4, 0x7fff7fff, %4\n\tv_and_b32 %5, 0x7fff7fff, %5\n\tv_and_b32 %6, 0x7fff7fff, %6\n\tv_and_b32 %7, 0x7fff7fff, %7" : R8)
#define G128 ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8; ANDK8

template <int GROUPS, bool DESYNC>
__global__ void __launch_bounds__(256) kern(unsigned *out, unsigned long long *cyc, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const int wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
    int start = DESYNC ? (wave * 7) % GROUPS : 0;
    start = __builtin_amdgcn_readfirstlane(start);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        // enter the unrolled body at group `start` on the first pass (each group: 128 instructions, 1 KiB)
#pragma unroll
        for (int g = 0; g < GROUPS; ++g) {
            if (g >= start) { G128; }
        }
        start = 0;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int GROUPS, bool DESYNC>
void run(unsigned *out, unsigned long long *cyc, int wps) {
    const int blocks = 256 * wps, iters = 2048 / GROUPS;
    kern<GROUPS, DESYNC><<<blocks, 256>>>(out, cyc, 1);
    kern<GROUPS, DESYNC><<<blocks, 256>>>(out, cyc, iters);
    (void)hipDeviceSynchronize();
    static unsigned long long h[256 * 8];
    (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += (double)h[i];
    const double instr = (double)iters * GROUPS * 128;
    printf("body %3d KiB %-7s waves/SIMD=%d  cycles per instruction per SIMD %.2f\n", GROUPS, DESYNC ? "desync" : "sync", wps,
           s / blocks / instr / wps);
}

int main() {
    unsigned *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, sizeof(unsigned) * 256 * 8 * 256) != hipSuccess) return 1;
    if (hipMalloc(&cyc, sizeof(unsigned long long) * 256 * 8) != hipSuccess) return 1;
    for (int wps : {1, 3}) {
        run<8, false>(out, cyc, wps);
        run<8, true>(out, cyc, wps);
        run<16, false>(out, cyc, wps);
        run<16, true>(out, cyc, wps);
        run<32, false>(out, cyc, wps);
        run<32, true>(out, cyc, wps);
        run<64, false>(out, cyc, wps);
        run<64, true>(out, cyc, wps);
    }
    return 0;
}
