// Debug build of runtime/h2d_engine.cpp (module accelerate_hpc_test_amd._C_debug).
#define ACC_DEBUG_BOUNDS 1
#include "../runtime/h2d_engine.cpp"
