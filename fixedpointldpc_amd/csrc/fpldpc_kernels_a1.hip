// fpldpc_kernels_a1.hip -- the packed 47-slot array kernel (A: flood_pk<ArrayChecks<47>, 3>) in a
// translation unit of its own, so that it can be compiled with its own code-generation options
// (_build.py SOURCE_FLAGS; why: fpldpc_kernels.hip at array47_pair_kernel).
#define FPLDPC_TU_ARRAY1 1
#include "fpldpc_kernels.hip"
