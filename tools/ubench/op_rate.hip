// VALU throughput per SIMD by instruction (diagnostic only), measured as an AGGREGATE: every wave
// runs the same number of instructions; the rate is (wave-instructions issued per SIMD) / (span from
// the first wave's start to the last wave's end, in shader cycles).  W waves per SIMD (256-thread
// workgroups, W per CU), 8 independent chains per lane.  Also 3:1 mixes with v_add_u32, and the
// packed kernels' bp_mag2 as written (3 v_pk_min_u16 + 8 full-rate ops).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define R8 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define C2(OP) asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t" OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t" \
                            OP " %4, %4, %8\n\t" OP " %5, %5, %8\n\t" OP " %6, %6, %8\n\t" OP " %7, %7, %8" : R8 : "v"(b))
#define CS(OP) asm volatile(OP " %0, %8, %0\n\t" OP " %1, %8, %1\n\t" OP " %2, %8, %2\n\t" OP " %3, %8, %3\n\t" \
                            OP " %4, %8, %4\n\t" OP " %5, %8, %5\n\t" OP " %6, %8, %6\n\t" OP " %7, %8, %7" : R8 : "s"(sb))
#define CL(OP, LIT) asm volatile(OP " %0, " LIT ", %0\n\t" OP " %1, " LIT ", %1\n\t" OP " %2, " LIT ", %2\n\t" OP " %3, " LIT ", %3\n\t" \
                                 OP " %4, " LIT ", %4\n\t" OP " %5, " LIT ", %5\n\t" OP " %6, " LIT ", %6\n\t" OP " %7, " LIT ", %7" : R8)
#define CPS(OP) asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t" OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t" \
                             OP " %4, %4, %8\n\t" OP " %5, %5, %8\n\t" OP " %6, %6, %8\n\t" OP " %7, %7, %8" : R8 : "s"(sb))
#define ADD asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t" \
                         "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : R8 : "v"(b))
#define MIX(OP) asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\t" OP " %3, %3, %8\n\t" \
                             "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\t" OP " %7, %7, %8" : R8 : "v"(b))

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

template <int K>
__global__ void __launch_bounds__(256) kern(unsigned *out, unsigned long long *t, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned b = (blockIdx.x | 1) & 0x3fff3fff;
    unsigned sb = __builtin_amdgcn_readfirstlane(b);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if (K == 0) { ADD; ADD; ADD; ADD; }
        if (K == 1) { C2("v_pk_min_u16"); C2("v_pk_min_u16"); C2("v_pk_min_u16"); C2("v_pk_min_u16"); }
        if (K == 2) { C2("v_min_u16"); C2("v_min_u16"); C2("v_min_u16"); C2("v_min_u16"); }
        if (K == 3) { C2("v_and_b32"); C2("v_and_b32"); C2("v_and_b32"); C2("v_and_b32"); }
        if (K == 4) { C2("v_lshrrev_b32"); C2("v_lshrrev_b32"); C2("v_lshrrev_b32"); C2("v_lshrrev_b32"); }
        if (K == 5) { C2("v_sub_u32"); C2("v_sub_u32"); C2("v_sub_u32"); C2("v_sub_u32"); }
        if (K == 6) { MIX("v_pk_min_u16"); MIX("v_pk_min_u16"); MIX("v_pk_min_u16"); MIX("v_pk_min_u16"); }
        if (K == 7) { MIX("v_min_u16"); MIX("v_min_u16"); MIX("v_min_u16"); MIX("v_min_u16"); }
        if (K == 8) { C2("v_pk_add_u16"); C2("v_pk_add_u16"); C2("v_pk_add_u16"); C2("v_pk_add_u16"); }
        if (K == 9) { C2("v_min_u32"); C2("v_min_u32"); C2("v_min_u32"); C2("v_min_u32"); }
        if (K == 10) { CS("v_and_b32"); CS("v_and_b32"); CS("v_and_b32"); CS("v_and_b32"); }
        if (K == 11) { C2("v_xor_b32"); C2("v_xor_b32"); C2("v_xor_b32"); C2("v_xor_b32"); }
        if (K == 12) { C2("v_add_u16"); C2("v_add_u16"); C2("v_add_u16"); C2("v_add_u16"); }
        if (K == 13) { C2("v_max_i16"); C2("v_max_i16"); C2("v_max_i16"); C2("v_max_i16"); }
        if (K == 14) { C2("v_pk_max_i16"); C2("v_pk_max_i16"); C2("v_pk_max_i16"); C2("v_pk_max_i16"); }
        if (K == 15) { C2("v_lshrrev_b16"); C2("v_lshrrev_b16"); C2("v_lshrrev_b16"); C2("v_lshrrev_b16"); }
        if (K == 16) { C2("v_cndmask_b32"); C2("v_cndmask_b32"); C2("v_cndmask_b32"); C2("v_cndmask_b32"); }
        if (K == 18) { CL("v_and_b32", "0x7fff7fff"); CL("v_and_b32", "0x7fff7fff"); CL("v_and_b32", "0x7fff7fff"); CL("v_and_b32", "0x7fff7fff"); }
        if (K == 19) { CL("v_add_u32", "-1"); CL("v_add_u32", "-1"); CL("v_add_u32", "-1"); CL("v_add_u32", "-1"); }
        if (K == 20) { CL("v_lshrrev_b32", "2"); CL("v_lshrrev_b32", "2"); CL("v_lshrrev_b32", "2"); CL("v_lshrrev_b32", "2"); }
        if (K == 21) { CPS("v_pk_min_u16"); CPS("v_pk_min_u16"); CPS("v_pk_min_u16"); CPS("v_pk_min_u16"); }
        if (K == 22) { CS("v_sub_u32"); CS("v_sub_u32"); CS("v_sub_u32"); CS("v_sub_u32"); }
        if (K == 23) { CS("v_add_u16"); CS("v_add_u16"); CS("v_add_u16"); CS("v_add_u16"); }
        if (K == 24) {  // bp_mag2 with the mask in a VGPR
            unsigned *x[8] = {&a0, &a1, &a2, &a3, &a4, &a5, &a6, &a7};
            const unsigned Mv = 0x003f003fu + (b >> 30);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                unsigned a = *x[c], mn, s, d;
                asm volatile("v_pk_min_u16 %[mn], %[a], %[b]\n\tv_add_u32 %[s], %[a], %[b]\n\t"
                             "v_sub_u32 %[d], %[s], %[mn]\n\tv_sub_u32 %[d], %[d], %[mn]\n\t"
                             "v_lshrrev_b32 %[s], 2, %[s]\n\tv_lshrrev_b32 %[d], 2, %[d]\n\t"
                             "v_and_b32 %[s], %[M], %[s]\n\tv_and_b32 %[d], %[M], %[d]\n\t"
                             "v_pk_min_u16 %[s], %[s], %[C]\n\tv_pk_min_u16 %[d], %[d], %[C]\n\t"
                             "v_sub_u32 %[a], %[mn], %[s]\n\tv_add_u32 %[a], %[a], %[d]"
                             : [a] "+v"(a), [mn] "=&v"(mn), [s] "=&v"(s), [d] "=&v"(d)
                             : [b] "v"(b), [M] "v"(Mv), [C] "s"(0x000a000au));
                *x[c] = a;
            }
        }
        if (K == 25) {  // 3:1 add:pk_min, pk grouped in pairs: pk pk add add add add add add
            asm volatile("v_pk_min_u16 %0, %0, %8\n\tv_pk_min_u16 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                         "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : R8 : "v"(b));
            asm volatile("v_pk_min_u16 %2, %2, %8\n\tv_pk_min_u16 %3, %3, %8\n\tv_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\t"
                         "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : R8 : "v"(b));
            asm volatile("v_pk_min_u16 %4, %4, %8\n\tv_pk_min_u16 %5, %5, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                         "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : R8 : "v"(b));
            asm volatile("v_pk_min_u16 %6, %6, %8\n\tv_pk_min_u16 %7, %7, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                         "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8" : R8 : "v"(b));
        }
        if (K == 26) {  // 3:1, pk grouped by 8: 8 pk then 24 add
            C2("v_pk_min_u16"); ADD; ADD; ADD;
        }
        if (K == 27) {  // 1:1 add:pk_min alternating
            asm volatile("v_pk_min_u16 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_pk_min_u16 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                         "v_pk_min_u16 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_pk_min_u16 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : R8 : "v"(b));
            asm volatile("v_pk_min_u16 %1, %1, %8\n\tv_add_u32 %0, %0, %8\n\tv_pk_min_u16 %3, %3, %8\n\tv_add_u32 %2, %2, %8\n\t"
                         "v_pk_min_u16 %5, %5, %8\n\tv_add_u32 %4, %4, %8\n\tv_pk_min_u16 %7, %7, %8\n\tv_add_u32 %6, %6, %8" : R8 : "v"(b));
            asm volatile("v_pk_min_u16 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_pk_min_u16 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                         "v_pk_min_u16 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_pk_min_u16 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : R8 : "v"(b));
            asm volatile("v_pk_min_u16 %1, %1, %8\n\tv_add_u32 %0, %0, %8\n\tv_pk_min_u16 %3, %3, %8\n\tv_add_u32 %2, %2, %8\n\t"
                         "v_pk_min_u16 %5, %5, %8\n\tv_add_u32 %4, %4, %8\n\tv_pk_min_u16 %7, %7, %8\n\tv_add_u32 %6, %6, %8" : R8 : "v"(b));
        }
        if (K == 28) {  // 1:1, grouped: 8 pk then 8 add
            C2("v_pk_min_u16"); ADD; C2("v_pk_min_u16"); ADD;
        }
        if (K == 29) { C2("v_min_u16_e64"); C2("v_min_u16_e64"); C2("v_min_u16_e64"); C2("v_min_u16_e64"); }
        if (K == 30) { C2("v_max_u16"); C2("v_max_u16"); C2("v_max_u16"); C2("v_max_u16"); }
        if (K == 17) {  // bp_mag2 on 8 chains (12 instructions each, written as in the decoder)
            unsigned *x[8] = {&a0, &a1, &a2, &a3, &a4, &a5, &a6, &a7};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                unsigned a = *x[c], mn, s, d;
                asm volatile("v_pk_min_u16 %[mn], %[a], %[b]\n\tv_add_u32 %[s], %[a], %[b]\n\t"
                             "v_sub_u32 %[d], %[s], %[mn]\n\tv_sub_u32 %[d], %[d], %[mn]\n\t"
                             "v_lshrrev_b32 %[s], 2, %[s]\n\tv_lshrrev_b32 %[d], 2, %[d]\n\t"
                             "v_and_b32 %[s], %[M], %[s]\n\tv_and_b32 %[d], %[M], %[d]\n\t"
                             "v_pk_min_u16 %[s], %[s], %[C]\n\tv_pk_min_u16 %[d], %[d], %[C]\n\t"
                             "v_sub_u32 %[a], %[mn], %[s]\n\tv_add_u32 %[a], %[a], %[d]"
                             : [a] "+v"(a), [mn] "=&v"(mn), [s] "=&v"(s), [d] "=&v"(d)
                             : [b] "v"(b), [M] "s"(0x003f003fu), [C] "s"(0x000a000au));
                *x[c] = a;
            }
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) {
        t[4 * blockIdx.x] = c0;
        t[4 * blockIdx.x + 1] = c1;
        t[4 * blockIdx.x + 2] = r0;
        t[4 * blockIdx.x + 3] = r1;
    }
}

typedef void (*Fn)(unsigned *, unsigned long long *, int);
template <int K> void add(Fn *f) { f[K] = kern<K>; add<K - 1>(f); }
template <> void add<-1>(Fn *) {}

int main() {
    const int N = 31;
    const char *names[N] = {"v_add_u32", "v_pk_min_u16", "v_min_u16", "v_and_b32", "v_lshrrev_b32", "v_sub_u32",
                            "3:1 add:v_pk_min_u16", "3:1 add:v_min_u16", "v_pk_add_u16", "v_min_u32", "v_and_b32 sgpr",
                            "v_xor_b32", "v_add_u16", "v_max_i16", "v_pk_max_i16", "v_lshrrev_b16", "v_cndmask_b32",
                            "bp_mag2 (12 instr)", "v_and_b32 literal", "v_add_u32 inline -1", "v_lshrrev_b32 inline 2",
                            "v_pk_min_u16 sgpr", "v_sub_u32 sgpr", "v_add_u16 sgpr", "bp_mag2 mask in VGPR",
                            "3:1 add:pk pairs", "3:1 add:pk 8-groups", "1:1 add:pk alternating", "1:1 add:pk 8-groups",
                            "v_min_u16_e64", "v_max_u16"};
    Fn f[N];
    add<N - 1>(f);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *out;
    unsigned long long *t;
    (void)hipMalloc(&out, sizeof(unsigned) * 256 * 8 * cus);
    (void)hipMalloc(&t, sizeof(unsigned long long) * 4 * 8 * cus);
    std::vector<unsigned long long> h(4 * 8 * cus);
    const int iters = 2000;
    for (int k = 0; k < N; ++k)
        for (int w : {2, 3, 4}) {
            if (k < 25 && k != 3 && k != 6 && k != 1) continue;
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
            const double instr_per_simd = (double)w * iters * 32;  // per wave: 4 macros x 8 instructions
            const double ipw = (k == 17 || k == 24) ? 12.0 * 8 / 32 : 1.0;         // bp_mag2: 96 instructions per iteration
            printf("%-22s waves/SIMD=%d  cycles per wave-instruction per SIMD %.2f  (clock %.2f GHz)\n", names[k], w,
                   span / (instr_per_simd * ipw), ghz);
        }
    return 0;
}
