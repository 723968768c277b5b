// Debug build of runtime/d2h_writer.cpp (module accelerate_hpc_test_amd._C_debug).
#define ACC_DEBUG_BOUNDS 1
#include "../runtime/d2h_writer.cpp"
