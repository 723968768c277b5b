// Debug build of runtime/cpu_adam.cpp (module accelerate_hpc_test_amd._C_debug).
#define ACC_DEBUG_BOUNDS 1
#include "../runtime/cpu_adam.cpp"
