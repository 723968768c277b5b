// Debug build of bindings.cpp (module accelerate_hpc_test_amd._C_debug).
#define ACC_DEBUG_BOUNDS 1
#include "../bindings.cpp"
