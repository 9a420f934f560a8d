// LDS DMA (global_load_lds_dword) semantics check: each lane l of a wave writes LDS word base + l.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t *src, uint32_t *out, int nw) {
    extern __shared__ uint32_t sm[];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) sm[i] = 0xdeadbeef;
    __syncthreads();
    const int wave = threadIdx.x / 64;
    // each wave copies 64 dwords per instruction: lane l -> sm[base + l]
    for (int b = wave * 64; b < nw; b += blockDim.x) {
        __builtin_amdgcn_global_load_lds(src + b + (threadIdx.x & 63), sm + b, 4, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // crude: wait all
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) out[i] = sm[i];
}
int main() {
    const int nw = 700;
    uint32_t *s, *o; hipMalloc(&s, 4096); hipMalloc(&o, 4096);
    uint32_t h[1024]; for (int i = 0; i < 1024; ++i) h[i] = 1000000 + i;
    hipMemcpy(s, h, 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 4096, 0, s, o, nw);
    hipMemcpy(h, o, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; ++i) {
        uint32_t want = i < 768 ? 1000000 + i : 0xdeadbeef;  // waves copy whole 64-dword blocks up to 767
        if (h[i] != want) { if (bad < 5) printf("i=%d got %u want %u\n", i, h[i], want); ++bad; }
    }
    printf("bad %d (first %u %u %u)\n", bad, h[0], h[1], h[767]);
    return 0;
}
