// Debug build of kernels/flash_attn.hip: same source with the device bounds checks compiled in (kernels/common.h).
#define ACC_DEBUG_BOUNDS 1
#include "../kernels/flash_attn.hip"
