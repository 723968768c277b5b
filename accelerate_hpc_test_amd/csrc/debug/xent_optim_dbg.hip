// Debug build of kernels/xent_optim.hip: same source with the device bounds checks compiled in (kernels/common.h).
#define ACC_DEBUG_BOUNDS 1
#include "../kernels/xent_optim.hip"
