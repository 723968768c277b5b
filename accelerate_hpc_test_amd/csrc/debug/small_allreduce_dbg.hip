// Debug build of kernels/small_allreduce.hip: same source with the device bounds checks compiled in (kernels/common.h).
#define ACC_DEBUG_BOUNDS 1
#include "../kernels/small_allreduce.hip"
