// Does a VOP2 16-bit op (v_min_u16_e32, v_add_u16_e32) on gfx950 keep or zero bits 16-31 of its
// destination?  (Diagnostic only.)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *out) {
    unsigned d = 0xabcd1234u, a = 0x00050007u, b = 0x00090003u;
    asm volatile("v_min_u16 %0, %1, %2" : "+v"(d) : "v"(a), "v"(b));
    unsigned e = 0xabcd1234u;
    asm volatile("v_add_u16 %0, %1, %2" : "+v"(e) : "v"(a), "v"(b));
    unsigned f = 0xabcd1234u;
    asm volatile("v_lshrrev_b16 %0, 1, %1" : "+v"(f) : "v"(a));
    if (threadIdx.x == 0) { out[0] = d; out[1] = e; out[2] = f; }
}
int main() {
    unsigned *o, h[3];
    if (hipMalloc(&o, 12) != hipSuccess) return 1;
    k<<<1, 64>>>(o);
    (void)hipMemcpy(h, o, 12, hipMemcpyDeviceToHost);
    printf("v_min_u16 -> %08x  v_add_u16 -> %08x  v_lshrrev_b16 -> %08x  (dst was abcd1234; low results 0003 / 000a / 0003)\n", h[0], h[1], h[2]);
    return 0;
}
