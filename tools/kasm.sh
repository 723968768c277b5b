#!/bin/bash
# Device assembly of one kernel source, compiled exactly as setup.py does (gfx950):
#   bash tools/kasm.sh accelerate_hpc_test_amd/csrc/kernels/flash_attn.hip /tmp/asm
# -> /tmp/asm/<name>-hip-amdgcn-amd-amdhsa-gfx950.s ; then: python tools/asm_loop.py <that .s> attn_bwd_dkdv
src=$(readlink -f "$1"); out=${2:-/tmp/asm}
mkdir -p "$out" && cd "$out" || exit 1
T=/usr/local/lib/python3.10/dist-packages/torch/include
/opt/rocm/bin/hipcc -I"$(dirname "$src")" -I$T -I$T/torch/csrc/api/include -I$T/THH -I/opt/rocm/include -I/usr/include/python3.10 \
  -c "$src" -o /dev/null -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DHIPBLAS_V2 -fPIC -DCUDA_HAS_FP16=1 -D__HIP_NO_HALF_OPERATORS__=1 \
  -D__HIP_NO_HALF_CONVERSIONS__=1 -DHIP_ENABLE_WARP_SYNC_BUILTINS=1 -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize \
  -DTORCH_API_INCLUDE_EXTENSION_H -DTORCH_EXTENSION_NAME=_C -fno-gpu-rdc -save-temps $KASM_FLAGS 2>&1 | grep -E "error|spill" | head
ls "$out"/*gfx950*.s
