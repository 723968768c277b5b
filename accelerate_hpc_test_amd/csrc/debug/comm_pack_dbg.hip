// Debug build of kernels/comm_pack.hip: same source with the device bounds checks compiled in (kernels/common.h).
#define ACC_DEBUG_BOUNDS 1
#include "../kernels/comm_pack.hip"
