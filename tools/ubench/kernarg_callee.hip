// The round-5 split-tail variant "call" (r5ab2, A @ 4.5 dB: hipErrorIllegalAddress) in miniature: an
// out-of-line device function that reads the launch arguments through
// __builtin_amdgcn_kernarg_segment_ptr().  Compile only, do not run:
//   hipcc --offload-arch=gfx950 -O3 --offload-device-only -S kernarg_callee.hip -o -
// The callee's pointer is `s_mov_b64 s[2:3], 0`: the AMDGPU backend lowers the intrinsic in a
// non-kernel function to null (the callable-function ABI passes the dispatch, queue and implicit-
// argument pointers, not the kernarg segment pointer, which only an entry function receives in its
// user SGPRs), so every KArgs field read in the tail loaded from address 0 + offset.  A @ 0 dB never
// entered the tail and passed.  profiles/r6/kernarg_callee.txt holds the ISA.
#include <hip/hip_runtime.h>
struct KArgs { int *out; int n; int pad[30]; };
__device__ __attribute__((noinline)) void tail(int i) {
    const KArgs *a = reinterpret_cast<const KArgs *>(__builtin_amdgcn_kernarg_segment_ptr());
    if (i < a->n) a->out[i] = i;
}
__global__ void k(KArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) a.out[i] = -1;
    if (i & 1) tail(i);
}
