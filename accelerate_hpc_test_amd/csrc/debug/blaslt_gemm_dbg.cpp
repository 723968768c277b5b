// Debug build of runtime/blaslt_gemm.cpp (module accelerate_hpc_test_amd._C_debug).
#define ACC_DEBUG_BOUNDS 1
#include "../runtime/blaslt_gemm.cpp"
