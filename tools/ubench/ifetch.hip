// Instruction-fetch / issue micro-benchmark (diagnostic only): does a long straight-line VALU
// loop body (the decoder's check step is ~3000 instructions, ~16 KB) issue slower than a short one,
// and how do the kernel's op mixes add up?  8 independent chains per lane, WPS waves per SIMD on
// every CU.  Prints Gwave-instr/s/SIMD per (body length, op mix, waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
// 8 instructions, one per chain
#define ADD8 asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t" \
                          "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : R8 : "v"(b))
#define PKM8 asm volatile("v_pk_min_u16 %0, %0, %8\n\tv_pk_min_u16 %1, %1, %8\n\tv_pk_min_u16 %2, %2, %8\n\tv_pk_min_u16 %3, %3, %8\n\t" \
                          "v_pk_min_u16 %4, %4, %8\n\tv_pk_min_u16 %5, %5, %8\n\tv_pk_min_u16 %6, %6, %8\n\tv_pk_min_u16 %7, %7, %8" : R8 : "v"(b))
// 8 instructions with a 32-bit literal each (8-byte encoding, full-rate op)
#define ANDK8 asm volatile("v_and_b32 %0, 0x7fff7fff, %0\n\tv_and_b32 %1, 0x7fff7fff, %1\n\tv_and_b32 %2, 0x7fff7fff, %2\n\tv_and_b32 %3, 0x7fff7fff, %3\n\t" \
                           "v_and_b32 %4, 0x7fff7fff, %4\n\tv_and_b32 %5, 0x7fff7fff, %5\n\tv_and_b32 %6, 0x7fff7fff, %6\n\tv_and_b32 %7, 0x7fff7fff, %7" : R8)
// one 32-instruction group of each mix
#define G_ADD ADD8; ADD8; ADD8; ADD8
#define G_PKM PKM8; PKM8; PKM8; PKM8
#define G_MIX ADD8; ADD8; ADD8; PKM8   // 3:1 like the box-plus chain
#define G_LIT ANDK8; ANDK8; ANDK8; ANDK8

#define REP4(X) X; X; X; X
#define REP16(X) REP4(X); REP4(X); REP4(X); REP4(X)

template <int MIX, int GROUPS>
__global__ void __launch_bounds__(256) kern(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned b = blockIdx.x | 1;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int g = 0; g < GROUPS; ++g) {
            if (MIX == 0) { G_ADD; }
            if (MIX == 1) { G_PKM; }
            if (MIX == 2) { G_MIX; }
            if (MIX == 3) { G_LIT; }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int MIX, int GROUPS>
void run(const char *name, unsigned *out, int wps) {
    const int threads = 256, blocks = 256 * wps;  // wps waves per SIMD on 256 CUs (4 waves per block)
    const long total_groups = 2048L * 8;           // same instruction count for every body length
    const int iters = (int)(total_groups / GROUPS);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<MIX, GROUPS><<<blocks, threads>>>(out, 4);
    (void)hipEventRecord(e0);
    kern<MIX, GROUPS><<<blocks, threads>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winstr = (double)blocks * (threads / 64) * iters * GROUPS * 32;
    printf("%-8s body=%5d instr  waves/SIMD=%d  %8.3f ms  %6.3f Gwave-instr/s/SIMD\n", name, GROUPS * 32, wps, ms,
           winstr / 1024 / (ms * 1e-3) / 1e9);
}

int main() {
    unsigned *out;
    if (hipMalloc(&out, sizeof(unsigned) * 256 * 8 * 256) != hipSuccess) return 1;
    for (int wps : {2, 3, 4, 8}) {
        run<0, 4>("add", out, wps);
        run<0, 32>("add", out, wps);
        run<0, 128>("add", out, wps);
        run<1, 4>("pk_min", out, wps);
        run<1, 128>("pk_min", out, wps);
        run<2, 4>("mix3:1", out, wps);
        run<2, 32>("mix3:1", out, wps);
        run<2, 128>("mix3:1", out, wps);
        run<3, 4>("and_lit", out, wps);
        run<3, 32>("and_lit", out, wps);
        run<3, 128>("and_lit", out, wps);
    }
    return 0;
}
