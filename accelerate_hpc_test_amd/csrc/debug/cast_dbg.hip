// Debug build of kernels/cast.hip: same source with the device bounds checks compiled in (kernels/common.h).
#define ACC_DEBUG_BOUNDS 1
#include "../kernels/cast.hip"
