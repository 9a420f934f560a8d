// VALU op-mix issue-rate micro-benchmark (diagnostic only).  ubench/ifetch.hip showed that a 3:1
// mix of v_add_u32 and v_pk_min_u16 issues slower than the two ops' separate rates predict; this
// measures, for each candidate op X, the rate of X alone and of the mix (24 v_add_u32 + 8 X) per
// 32-instruction group, 8 independent chains per lane, 4 waves per SIMD on every CU.
// "cost in mix" = (time of the mix - time of 24 adds) / 8, in units of one v_add_u32.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define I8(OP)                                                                                              \
    asm volatile(OP(0) "\n\t" OP(1) "\n\t" OP(2) "\n\t" OP(3) "\n\t" OP(4) "\n\t" OP(5) "\n\t" OP(6) "\n\t" \
                 OP(7) : R8 : "v"(b), "s"(sb))
#define ADD(i) "v_add_u32 %" #i ", %" #i ", %8"
#define PKMIN(i) "v_pk_min_u16 %" #i ", %" #i ", %8"
#define MINU16(i) "v_min_u16 %" #i ", %" #i ", %8"
#define MINU16_HI(i) "v_min_u16_sdwa %" #i ", %" #i ", %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
#define MINU16_LO(i) "v_min_u16_sdwa %" #i ", %" #i ", %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
#define MINU32(i) "v_min_u32 %" #i ", %" #i ", %8"
#define PKASHR(i) "v_pk_ashrrev_i16 %" #i ", 15, %" #i
#define XAD(i) "v_xad_u32 %" #i ", %" #i ", %8, %" #i
#define OR3(i) "v_or3_b32 %" #i ", %" #i ", %8, %" #i
#define SUB3(i) "v_sub_u32_e64 %" #i ", %" #i ", %8"
#define ADDU16(i) "v_add_u16 %" #i ", %" #i ", %8"
#define ADDU16_HI(i) "v_add_u16_sdwa %" #i ", %" #i ", %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
#define MED3(i) "v_med3_u32 %" #i ", %" #i ", %8, %" #i
#define BFE(i) "v_bfe_u32 %" #i ", %" #i ", 2, 6"
#define PKADD(i) "v_pk_add_u16 %" #i ", %" #i ", %8"
#define PKMIN_LO(i) "v_pk_min_u16 %" #i ", %" #i ", %8 op_sel_hi:[0,0]"
#define MINI16(i) "v_min_i16 %" #i ", %" #i ", %8"
#define CNDM(i) "v_cndmask_b32 %" #i ", %" #i ", %8, vcc"
#define LSHRA(i) "v_lshrrev_b32 %" #i ", 2, %" #i
#define ANDK(i) "v_and_b32 %" #i ", 0x3f003f, %" #i
#define LSHL(i) "v_lshlrev_b32 %" #i ", 16, %" #i
#define MULU24(i) "v_mul_u32_u24 %" #i ", %" #i ", %8"
#define MINF32(i) "v_min_f32 %" #i ", %" #i ", %8"
#define ADDF32(i) "v_add_f32 %" #i ", %" #i ", %8"
#define LSHLB16(i) "v_lshlrev_b16 %" #i ", 2, %" #i
#define LSHRB16(i) "v_lshrrev_b16 %" #i ", 2, %" #i
#define MAXU16(i) "v_max_u16 %" #i ", %" #i ", %8"
#define SUBREV(i) "v_subrev_u32 %" #i ", %" #i ", %8"
#define ADDCO(i) "v_add_co_u32 %" #i ", vcc, %" #i ", %8"
#define MOVB(i) "v_mov_b32 %" #i ", %8"
#define NOTB(i) "v_not_b32 %" #i ", %" #i
#define ANDS(i) "v_and_b32 %" #i ", %9, %" #i
#define ADDS(i) "v_add_u32 %" #i ", %9, %" #i
#define PKMINS(i) "v_pk_min_u16 %" #i ", %" #i ", %9"
#define XNOR(i) "v_xnor_b32 %" #i ", %" #i ", %8"
#define ADDU16S(i) "v_add_u16 %" #i ", %9, %" #i

#define ALONE(OP) I8(OP); I8(OP); I8(OP); I8(OP)
#define MIXED(OP) I8(ADD); I8(ADD); I8(ADD); I8(OP)
#define BASE I8(ADD); I8(ADD); I8(ADD)
// interleaved: add, add, add, X repeated (X every 4th instruction)
#define IL4(OP) asm volatile(ADD(0) "\n\t" ADD(1) "\n\t" ADD(2) "\n\t" OP(3) "\n\t" ADD(4) "\n\t" ADD(5) "\n\t" ADD(6) "\n\t" OP(7) : R8 : "v"(b), "s"(sb))
#define INTER(OP) IL4(OP); IL4(OP); IL4(OP); IL4(OP)

template <int K>
__global__ void __launch_bounds__(256) kern(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned b = blockIdx.x | 1;
    const unsigned sb = __builtin_amdgcn_readfirstlane(blockIdx.x | 0x30003);
    asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
#define CASE(ID, OP) if (K == 2 * ID) { ALONE(OP); } if (K == 2 * ID + 1) { MIXED(OP); }
            CASE(0, ADD) CASE(1, PKMIN) CASE(2, MINU16) CASE(3, MINU16_HI) CASE(4, MINU16_LO) CASE(5, MINU32)
            CASE(6, PKASHR) CASE(7, XAD) CASE(8, OR3) CASE(9, SUB3) CASE(10, ADDU16) CASE(11, ADDU16_HI) CASE(12, MED3)
            CASE(13, BFE) CASE(14, PKADD) CASE(15, PKMIN_LO) CASE(16, MINI16) CASE(17, CNDM) CASE(18, LSHRA) CASE(19, ANDK)
            CASE(20, LSHL) CASE(21, MULU24) CASE(22, MINF32) CASE(23, ADDF32) CASE(24, LSHLB16) CASE(25, LSHRB16)
            CASE(26, MAXU16) CASE(27, SUBREV) CASE(28, ADDCO) CASE(29, MOVB) CASE(30, NOTB)
            CASE(31, ANDS) CASE(32, ADDS) CASE(33, PKMINS) CASE(34, XNOR) CASE(35, ADDU16S)
            if (K == 100) { BASE; }
            if (K == 101) { INTER(PKMIN); }
            if (K == 102) { INTER(MINU16); }
            if (K == 103) { INTER(PKASHR); }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*Fn)(unsigned *, int);
template <int K> void add(Fn *t) { t[K] = kern<K>; add<K - 1>(t); }
template <> void add<-1>(Fn *) {}

static float timeit(Fn f, unsigned *out, int blocks, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    f<<<blocks, 256>>>(out, 8);
    (void)hipEventRecord(e0);
    f<<<blocks, 256>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    const int N = 36;
    const char *names[N] = {"v_add_u32", "v_pk_min_u16", "v_min_u16", "v_min_u16_sdwa hi", "v_min_u16_sdwa lo",
                            "v_min_u32", "v_pk_ashrrev_i16", "v_xad_u32", "v_or3_b32", "v_sub_u32_e64", "v_add_u16",
                            "v_add_u16_sdwa hi", "v_med3_u32", "v_bfe_u32", "v_pk_add_u16", "v_pk_min_u16 op_sel_hi0",
                            "v_min_i16", "v_cndmask_b32", "v_lshrrev_b32", "v_and_b32 lit", "v_lshlrev_b32 16",
                            "v_mul_u32_u24", "v_min_f32", "v_add_f32", "v_lshlrev_b16", "v_lshrrev_b16", "v_max_u16",
                            "v_subrev_u32", "v_add_co_u32", "v_mov_b32", "v_not_b32", "v_and_b32 sgpr",
                            "v_add_u32 sgpr", "v_pk_min_u16 sgpr", "v_xnor_b32", "v_add_u16 sgpr"};
    Fn fns[2 * N];
    add<2 * N - 1>(fns);
    unsigned *out;
    const int blocks = 256 * 4, iters = 1024;
    if (hipMalloc(&out, sizeof(unsigned) * blocks * 256) != hipSuccess) return 1;
    const float tb = timeit(kern<100>, out, blocks, iters);  // 24 adds per group
    const float ta = timeit(fns[0], out, blocks, iters);      // 32 adds per group
    const double unit = (ta - tb) / 8;                       // ms per 8 adds-per-group
    printf("base: 24 adds %.3f ms, 32 adds %.3f ms (%.3f Gwave-instr/s/SIMD)\n", tb, ta,
           (double)blocks * 4 * iters * 8 * 32 / 1024 / (ta * 1e-3) / 1e9);
    for (int k = 0; k < N; ++k) {
        const float t1 = timeit(fns[2 * k], out, blocks, iters), t2 = timeit(fns[2 * k + 1], out, blocks, iters);
        printf("%-26s alone %.3f ms (%.2fx add)   in 3:1 mix with add: cost %.2fx add\n", names[k], t1, t1 / ta,
               (t2 - tb) / 8 / (ta / 32));
    }
    const char *il[3] = {"v_pk_min_u16", "v_min_u16", "v_pk_ashrrev_i16"};
    Fn ilf[3] = {kern<101>, kern<102>, kern<103>};
    for (int k = 0; k < 3; ++k) {
        const float t2 = timeit(ilf[k], out, blocks, iters);
        printf("%-26s interleaved 1-in-4 with add: cost %.2fx add\n", il[k], (t2 - tb) / 8 / (ta / 32));
    }
    (void)unit;
    return 0;
}
