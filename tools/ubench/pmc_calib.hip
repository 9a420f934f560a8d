// pmc_calib.hip -- what FETCH_SIZE / WRITE_SIZE report for the float decoder's access width
// (diagnostic only): one kernel streams N doubles in (8 B per lane, coalesced, read once) and
// another streams N doubles out (8 B per lane), 1 GiB each, far beyond the 256 MiB Infinity Cache.
// Run each under its own rocprofv3 --pmc pass and compare the counters with the byte counts.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void rd8(const double *__restrict__ x, size_t n, double *out) {
    double acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += x[i];
    if (acc == 12345.678) out[0] = acc;  // keep the loads
}
__global__ void wr8(double *__restrict__ y, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) y[i] = (double)i;
}
__global__ void rd16(const double2 *__restrict__ x, size_t n, double *out) {
    double acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += x[i].x + x[i].y;
    if (acc == 12345.678) out[0] = acc;
}

int main() {
    const size_t bytes = 1ull << 30, n = bytes / 8;
    double *x, *y, *o;
    if (hipMalloc(&x, bytes) || hipMalloc(&y, bytes) || hipMalloc(&o, 64)) return 1;
    (void)hipMemset(x, 0, bytes);
    for (int r = 0; r < 2; ++r) {
        rd8<<<4096, 256>>>(x, n, o);
        wr8<<<4096, 256>>>(y, n);
        rd16<<<4096, 256>>>(reinterpret_cast<const double2 *>(x), n / 2, o);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("each kernel moves %zu bytes\n", bytes);
    return 0;
}
