// Check-step throughput decomposition (diagnostic only).  The decoder's own ArrayChecks<47>::step
// (fpldpc_kernels.hip) in a bare loop with WPS workgroups of 256 threads per CU, like
// step_rate.hip, but reporting the AGGREGATE rate: shader cycles from the first workgroup's start
// to the last one's end, per wave-step per SIMD (steps x WPS wave-steps per SIMD).  Built with
// FPLDPC_ABLATE bits (timing only, wrong results) to price each part of the step's instruction
// stream: 1 no LDS, 16 emission, 32 gather sign-magnitude, 64 box-plus (tools/gpu_stepmix.sh).
#ifndef FPLDPC_ABLATE
#define FPLDPC_ABLATE 0
#endif
#include "../../fixedpointldpc_amd/csrc/fpldpc_kernels.hip"

#include <algorithm>

namespace fpldpc {
int fail(int code, const std::string &) { return code; }  // error reporting lives in the library
}  // namespace fpldpc

namespace fpldpc {
namespace {
__global__ void __launch_bounds__(256, 3) mix_kernel(KArgs a, unsigned *out, unsigned long long *t, int steps) {
    ArrayChecks<47> ck;
    ck.init(a, threadIdx.x);
    const u16x2 C2 = (u16x2)(unsigned short)10;
    const uint32_t M2 = 0x003f003fu;
    Stamps stp;
    uint32_t acc = 0, ovf = 0;
    extern __shared__ __attribute__((aligned(16))) int smem_s[];
    for (int v = threadIdx.x; v < 3 * 2209; v += 256) smem_s[v] = 0x7fff7fff ^ (v * 2654435761u & 0x00ff00ffu);
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t base = lds_addr(smem_s);
    for (int s = 0; s < steps; ++s) {
        uint32_t par = 0, ovor = 0;
        const uint32_t pc = base + (uint32_t)(s % 3) * 8836u, pn = base + (uint32_t)((s + 1) % 3) * 8836u;
        ck.step(a, nullptr, nullptr, pc, pn, C2, M2, par, ovor, stp);
        acc ^= par;
        ovf |= ovor;
        __syncthreads();
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ ovf;
    if (threadIdx.x == 0) {
        t[4 * blockIdx.x + 0] = c0;
        t[4 * blockIdx.x + 1] = c1;
        t[4 * blockIdx.x + 2] = r0;
        t[4 * blockIdx.x + 3] = r1;
    }
}
}  // namespace
}  // namespace fpldpc

int main() {
    using namespace fpldpc;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    unsigned *out;
    unsigned long long *t;
    if (hipMalloc(&out, sizeof(unsigned) * 256 * 4 * cus) != hipSuccess) return 1;
    if (hipMalloc(&t, sizeof(unsigned long long) * 4 * 4 * cus) != hipSuccess) return 1;
    KArgs a{};
    a.m = 235;
    a.n = 2209;
    const int steps = 60;
    std::vector<unsigned long long> h(4 * 4 * cus);
    for (int wps : {1, 2, 3}) {
        const int blocks = cus * wps;
        mix_kernel<<<blocks, 256, 3 * 8836>>>(a, out, t, 4);
        mix_kernel<<<blocks, 256, 3 * 8836>>>(a, out, t, steps);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        (void)hipMemcpy(h.data(), t, sizeof(unsigned long long) * 4 * blocks, hipMemcpyDeviceToHost);
        unsigned long long r_min = ~0ull, r_max = 0;
        double cyc = 0, real = 0;
        for (int i = 0; i < blocks; ++i) {
            r_min = std::min(r_min, h[4 * i + 2]);
            r_max = std::max(r_max, h[4 * i + 3]);
            cyc += (double)(h[4 * i + 1] - h[4 * i]);
            real += (double)(h[4 * i + 3] - h[4 * i + 2]);
        }
        const double ghz = cyc / real / 10.0;            // s_memrealtime ticks at 100 MHz
        const double span_cyc = (double)(r_max - r_min) * 10.0 * ghz;
        printf("ABLATE=%d WGs/CU=%d  aggregate cycles per wave-step per SIMD %.0f  (span %.1f us, clock %.2f GHz)\n",
               FPLDPC_ABLATE, wps, span_cyc / (steps * wps), (r_max - r_min) / 100.0, ghz);
    }
    return 0;
}
