// Bit-exactness check of the float decoder's exp_neg (fpldpc_float_math.hpp) against the device
// libm's exp(-x) on x in [0, 36.75): 2^26 uniform samples plus every double in small windows around
// the reduction's switch points x = (j + 1/2) ln2.  Prints the count of differing results.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I fixedpointldpc_amd/csrc
//        tools/float_exp_check.hip -o build/float_exp_check
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "fpldpc_float_math.hpp"

__global__ void check(unsigned long long n, unsigned long long *bad, double *first) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x;
    const unsigned long long nu = 1ull << 26;
    if (i < nu) {
        x = 36.75 * ((double)i / (double)nu);
    } else {  // 64 consecutive doubles on each side of (j + 1/2) ln2, j = 0..52
        const unsigned long long t = i - nu, j = t / 128, o = t % 128;
        double c = ((double)j + 0.5) * 0.6931471805599453;
        long long b;
        memcpy(&b, &c, 8);
        b += (long long)o - 64;
        memcpy(&x, &b, 8);
        if (!(x >= 0.0 && x < 36.75)) return;
    }
    const double a = exp(-x), e = fpldpc::exp_neg(x);
    if (__builtin_bit_cast(unsigned long long, a) != __builtin_bit_cast(unsigned long long, e)) {
        if (atomicAdd(bad, 1ull) == 0) *first = x;
    }
}

int main() {
    const unsigned long long n = (1ull << 26) + 53 * 128;
    unsigned long long *bad;
    double *first;
    if (hipMallocManaged(&bad, 8) != hipSuccess || hipMallocManaged(&first, 8) != hipSuccess) return 2;
    *bad = 0;
    *first = -1;
    hipLaunchKernelGGL(check, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("exp_neg vs libm exp(-x): %llu of %llu samples differ (first at x = %.17g)\n", *bad, n, *first);
    return *bad ? 1 : 0;
}
