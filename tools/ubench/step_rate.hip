// Check-step issue-rate micro-benchmark (diagnostic only): the decoder's own ArrayChecks<47>::step
// (fpldpc_kernels.hip, compiled here with FPLDPC_ABLATE=1: gather values derived from registers, no
// LDS atomics) called in a bare loop, without the persistent-kernel framework around it (flags,
// barrier, LLR copy, refill).  Shader cycles per step per wave, WPS workgroups of 256 threads per
// CU: tells whether the step's own instruction stream or the framework limits VALU issue.
#ifndef FPLDPC_ABLATE
#define FPLDPC_ABLATE 1  // 0: real LDS gather and scatter (dynamic LDS of 3 x 8836 B)
#endif
#include "../../fixedpointldpc_amd/csrc/fpldpc_kernels.hip"

namespace fpldpc {
int fail(int code, const std::string &) { return code; }  // error reporting lives in the library
}  // namespace fpldpc

namespace fpldpc {
namespace {
template <int MODE>
__global__ void __launch_bounds__(256, 3) step_kernel(KArgs a, unsigned *out, unsigned long long *cyc, int steps) {
    ArrayChecks<47> ck;
    ck.init(a, threadIdx.x);
    const u16x2 C2 = (u16x2)(unsigned short)10;
    const uint32_t M2 = 0x003f003fu;
    Stamps stp;
    uint32_t acc = 0, ovf = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    extern __shared__ __attribute__((aligned(16))) int smem_s[];
    for (int v = threadIdx.x; v < 3 * 2209; v += 256) smem_s[v] = 0x7fff7fff;
    __syncthreads();
    const uint32_t base = lds_addr(smem_s);
    for (int s = 0; s < steps; ++s) {
        uint32_t par = 0, ovor = 0;
        const uint32_t pc = base + (uint32_t)(s % 3) * 8836u, pn = base + (uint32_t)((s + 1) % 3) * 8836u;
        ck.step(a, nullptr, nullptr, pc, pn, C2, M2, par, ovor, stp);
        acc ^= par;
        ovf |= ovor;
        if (MODE == 1) __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ ovf;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
}  // namespace
}  // namespace fpldpc

int main() {
    using namespace fpldpc;
    unsigned *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, sizeof(unsigned) * 256 * 4 * 256) != hipSuccess) return 1;
    if (hipMalloc(&cyc, sizeof(unsigned long long) * 256 * 4) != hipSuccess) return 1;
    KArgs a{};
    a.m = 235;
    a.n = 2209;
    for (int mode = 0; mode < 2; ++mode)
        for (int wps : {1, 2, 3}) {
            const int blocks = 256 * wps, steps = 60;
            if (mode == 0) {
                step_kernel<0><<<blocks, 256, 3 * 8836>>>(a, out, cyc, 4);
                step_kernel<0><<<blocks, 256, 3 * 8836>>>(a, out, cyc, steps);
            } else {
                step_kernel<1><<<blocks, 256, 3 * 8836>>>(a, out, cyc, 4);
                step_kernel<1><<<blocks, 256, 3 * 8836>>>(a, out, cyc, steps);
            }
            (void)hipDeviceSynchronize();
            static unsigned long long h[256 * 4];
            (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
            double s = 0, mn = 1e30, mx = 0;
            for (int i = 0; i < blocks; ++i) {
                s += (double)h[i];
                mn = std::min(mn, (double)h[i]);
                mx = std::max(mx, (double)h[i]);
            }
            printf("LDS=%d %-10s WGs/CU=%d  cycles per step per wave: mean %.0f (fastest %.0f, slowest %.0f) -> per SIMD %.0f\n",
                   !(FPLDPC_ABLATE & 1), mode ? "+barrier" : "bare", wps, s / blocks / steps, mn / steps, mx / steps, s / blocks / steps / wps);
        }
    return 0;
}
