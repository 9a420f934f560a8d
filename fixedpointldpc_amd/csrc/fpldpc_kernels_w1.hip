// fpldpc_kernels_w1.hip -- the degree-sorted packed table kernel (W: flood_pk<TableChecks<8, 4, 7, 3>,
// 4>) in a translation unit of its own, so that it can be compiled with its own code-generation
// options (_build.py SOURCE_FLAGS; the A kernel has fpldpc_kernels_a1.hip for the same reason).
#define FPLDPC_TU_TABLE1 1
#include "fpldpc_kernels.hip"
