#!/bin/bash
# Per-kernel register / LDS / occupancy report of one HIP source (device-only compile for gfx950, torch flags).
#   bash tools/kernel_resources.sh accelerate_hpc_test_amd/csrc/kernels/flash_attn.hip
set -e
SRC=$1
TORCH=$(python -c "import torch,os;print(os.path.dirname(torch.__file__))")
ROOT=$(cd "$(dirname "$0")/.." && pwd)
hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -fno-slp-vectorize --offload-device-only -c "$SRC" -o /tmp/kres.o \
  -I"$ROOT/accelerate_hpc_test_amd/csrc/kernels" -I"$TORCH/include" -I"$TORCH/include/torch/csrc/api/include" \
  -I"$TORCH/include/THH" -I/opt/rocm/include -I/usr/include/python3.10 \
  -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_API_INCLUDE_EXTENSION_H -DTORCH_EXTENSION_NAME=_C \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "error|Function Name|VGPRs:|AGPRs:|Occupancy|LDS Size|ScratchSize" | sed 's/.*remark: //'
