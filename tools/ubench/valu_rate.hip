// VALU issue-rate micro-benchmark (diagnostic only): wave-instructions per second per SIMD for
// integer ops on gfx950, 8 independent chains per lane, 8 waves per SIMD on every CU.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define C2(OP) asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t" OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t" \
                            OP " %4, %4, %8\n\t" OP " %5, %5, %8\n\t" OP " %6, %6, %8\n\t" OP " %7, %7, %8" : R8 : "v"(b))
#define C3(OP) asm volatile(OP " %0, %0, %8, %9\n\t" OP " %1, %1, %8, %9\n\t" OP " %2, %2, %8, %9\n\t" OP " %3, %3, %8, %9\n\t" \
                            OP " %4, %4, %8, %9\n\t" OP " %5, %5, %8, %9\n\t" OP " %6, %6, %8, %9\n\t" OP " %7, %7, %8, %9" : R8 : "v"(b), "v"(c))

#define K2(ID, OP) if (K == ID) { C2(OP); C2(OP); C2(OP); C2(OP); }
#define K3(ID, OP) if (K == ID) { C3(OP); C3(OP); C3(OP); C3(OP); }

template <int K>
__global__ void kern(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned b = blockIdx.x | 1, c = (blockIdx.x >> 3) | 3;
    for (int i = 0; i < iters; ++i) {
        K2(0, "v_add_u32") K2(1, "v_sub_u32") K2(2, "v_and_b32") K2(3, "v_xor_b32") K2(4, "v_lshrrev_b32")
        K2(5, "v_min_u32") K2(6, "v_max_i32") K2(7, "v_add_u16") K2(8, "v_min_u16") K2(9, "v_max_u16")
        K2(10, "v_sub_u16") K2(11, "v_lshrrev_b16") K2(12, "v_pk_add_u16") K2(13, "v_pk_min_u16") K2(14, "v_pk_lshrrev_b16")
        K3(15, "v_bfe_u32") K3(16, "v_med3_u32") K3(17, "v_min3_u32") K3(18, "v_add3_u32") K3(19, "v_sad_u32")
        K3(20, "v_and_or_b32") K3(21, "v_lshl_add_u32") K3(22, "v_bfi_b32") K3(23, "v_perm_b32") K3(24, "v_xad_u32")
        K3(25, "v_or3_b32") K3(26, "v_sad_u16") K2(27, "v_min_i16") K2(28, "v_mul_u32_u24") K3(29, "v_mad_u32_u24")
        K2(30, "v_ashrrev_i32") K2(31, "v_or_b32") K2(32, "v_sub_co_u32") K2(33, "v_max_u32") K2(34, "v_min_i32")
        K2(35, "v_lshlrev_b32") K3(36, "v_max3_u32") K3(37, "v_lshl_or_b32") K2(38, "v_pk_max_i16") K2(39, "v_pk_sub_u16")
        K2(40, "v_add_f32") K2(41, "v_min_f32") K2(42, "v_pk_add_f16") K2(43, "v_pk_min_f16") K3(44, "v_fma_f32")
        K3(45, "v_pk_fma_f16") K2(46, "v_sub_i32") K3(47, "v_alignbit_b32")
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*Fn)(unsigned *, int);
template <int K> void add(Fn *t) { t[K] = kern<K>; add<K - 1>(t); }
template <> void add<-1>(Fn *) {}

int main() {
    const int N = 48;
    const char *names[N] = {"v_add_u32", "v_sub_u32", "v_and_b32", "v_xor_b32", "v_lshrrev_b32", "v_min_u32", "v_max_i32",
                            "v_add_u16", "v_min_u16", "v_max_u16", "v_sub_u16", "v_lshrrev_b16", "v_pk_add_u16",
                            "v_pk_min_u16", "v_pk_lshrrev_b16", "v_bfe_u32", "v_med3_u32", "v_min3_u32", "v_add3_u32",
                            "v_sad_u32", "v_and_or_b32", "v_lshl_add_u32", "v_bfi_b32", "v_perm_b32", "v_xad_u32",
                            "v_or3_b32", "v_sad_u16", "v_min_i16", "v_mul_u32_u24", "v_mad_u32_u24", "v_ashrrev_i32",
                            "v_or_b32", "v_sub_co_u32", "v_max_u32", "v_min_i32", "v_lshlrev_b32", "v_max3_u32",
                            "v_lshl_or_b32", "v_pk_max_i16", "v_pk_sub_u16", "v_add_f32", "v_min_f32", "v_pk_add_f16",
                            "v_pk_min_f16", "v_fma_f32", "v_pk_fma_f16", "v_sub_i32", "v_alignbit_b32"};
    Fn fns[N];
    add<N - 1>(fns);
    const int blocks = 256 * 8, threads = 256, iters = 2048;
    unsigned *out;
    if (hipMalloc(&out, sizeof(unsigned) * blocks * threads) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    double base = 0;
    for (int k = 0; k < N; ++k) {
        fns[k]<<<blocks, threads>>>(out, 32);
        (void)hipEventRecord(e0);
        fns[k]<<<blocks, threads>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (k == 0) base = ms;
        const double winstr = (double)blocks * (threads / 64) * iters * 32;
        printf("%-18s %7.3f ms  %6.3f Gwave-instr/s/SIMD  cost %.2fx v_add_u32\n", names[k], ms, winstr / 1024 / (ms * 1e-3) / 1e9,
               ms / base);
    }
    return 0;
}
