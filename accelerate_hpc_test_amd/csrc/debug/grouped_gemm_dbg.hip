// Debug build of kernels/grouped_gemm.hip: same source with the device bounds checks compiled in (kernels/common.h).
#define ACC_DEBUG_BOUNDS 1
#include "../kernels/grouped_gemm.hip"
