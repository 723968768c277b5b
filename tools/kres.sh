#!/bin/bash
# Per-kernel register / spill / occupancy report of one HIP source (device-only compile for gfx950).
# usage: tools/kres.sh accelerate_hpc_test_amd/csrc/kernels/flash_attn.hip [extra hipcc flags]
src=$1; shift
TI=$(python -c "import torch.utils.cpp_extension as c; print(' '.join('-I'+p for p in c.include_paths('cuda')))")
cd /tmp && hipcc -I/root/repo/accelerate_hpc_test_amd/csrc/kernels $TI -I/usr/include/python3.10 -D__HIP_PLATFORM_AMD__=1 \
  -DUSE_ROCM=1 -DHIPBLAS_V2 -fPIC -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -DTORCH_API_INCLUDE_EXTENSION_H \
  -DTORCH_EXTENSION_NAME=_C -fno-gpu-rdc -c "/root/repo/$src" -o /tmp/kres.o --offload-device-only \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | grep remark | sed 's/.*remark: //' | \
  grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size" | paste - - - - - - | \
  sed -E 's/Function Name: //; s/\[-Rpass-analysis=kernel-resource-usage\]//g' | awk '{$1=$1; print}' | cut -c1-300
