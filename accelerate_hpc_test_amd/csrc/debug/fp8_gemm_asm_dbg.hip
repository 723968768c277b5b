// Debug build of kernels/fp8_gemm_asm.hip: same source with the device bounds checks compiled in (kernels/common.h).
#define ACC_DEBUG_BOUNDS 1
#include "../kernels/fp8_gemm_asm.hip"
