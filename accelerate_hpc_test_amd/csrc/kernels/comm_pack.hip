// Elementwise kernels around the FSDP / DDP collectives (gfx950, memory-bound: 16 B per lane per access).
//
//  * grad_shard_update: fp32 gradient shard (=|+=) scale * reduce-scatter output (bf16 or fp32) in ONE pass. It
//    replaces "bf16 -> fp32 copy, then multiply by 1/W" (two full passes over the shard, profiles/r2_*).
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include "common.h"

namespace {

using acc::bf16_t;
using acc::bf16x8;

template <bool ACC>
__global__ __launch_bounds__(256) void grad_update_bf16_kernel(float* __restrict__ dst, const bf16_t* __restrict__ src,
                                                                float scale, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const bf16x8 s = reinterpret_cast<const bf16x8*>(src)[i];
    float4* d = reinterpret_cast<float4*>(dst) + 2 * i;
    float4 a = make_float4(acc::bf2f(s.v[0]) * scale, acc::bf2f(s.v[1]) * scale, acc::bf2f(s.v[2]) * scale, acc::bf2f(s.v[3]) * scale);
    float4 b = make_float4(acc::bf2f(s.v[4]) * scale, acc::bf2f(s.v[5]) * scale, acc::bf2f(s.v[6]) * scale, acc::bf2f(s.v[7]) * scale);
    if (ACC) {
      const float4 o0 = d[0], o1 = d[1];
      a.x += o0.x; a.y += o0.y; a.z += o0.z; a.w += o0.w;
      b.x += o1.x; b.y += o1.y; b.z += o1.z; b.w += o1.w;
    }
    d[0] = a;
    d[1] = b;
  }
}

template <bool ACC>
__global__ __launch_bounds__(256) void grad_update_f32_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                               float scale, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 s = reinterpret_cast<const float4*>(src)[i];
    s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
    float4* d = reinterpret_cast<float4*>(dst) + i;
    if (ACC) {
      const float4 o = *d;
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
    }
    *d = s;
  }
}

int grid_for(int64_t work, int block) {
  // 256 CUs x 8 resident 256-thread blocks; grid-stride beyond that
  const int64_t want = (work + block - 1) / block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, 256 * 8));
}

}  // namespace

ACC_DEBUG_TAKE_FN(acc_dbg_take_comm_pack)

// dst (fp32, contiguous, n) = or += scale * src (bf16 / fp32, contiguous, n). n must be a multiple of 8.
void grad_shard_update(torch::Tensor dst, torch::Tensor src, double scale, bool accumulate) {
  TORCH_CHECK(dst.is_cuda() && src.is_cuda() && dst.is_contiguous() && src.is_contiguous(), "grad_shard_update: contiguous GPU tensors");
  TORCH_CHECK(dst.scalar_type() == at::kFloat, "grad_shard_update: dst must be fp32");
  TORCH_CHECK(dst.numel() == src.numel(), "grad_shard_update: size mismatch");
  const int64_t n = dst.numel();
  TORCH_CHECK(n % 8 == 0, "grad_shard_update: numel must be a multiple of 8, got ", n);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
              "grad_shard_update: 16-byte aligned buffers required");
  if (n == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const float s = static_cast<float>(scale);
  if (src.scalar_type() == at::kBFloat16) {
    const int64_t n8 = n / 8;
    auto* d = dst.data_ptr<float>();
    auto* x = reinterpret_cast<const bf16_t*>(src.data_ptr());
    if (accumulate)
      hipLaunchKernelGGL(grad_update_bf16_kernel<true>, dim3(grid_for(n8, 256)), dim3(256), 0, stream, d, x, s, n8);
    else
      hipLaunchKernelGGL(grad_update_bf16_kernel<false>, dim3(grid_for(n8, 256)), dim3(256), 0, stream, d, x, s, n8);
  } else {
    TORCH_CHECK(src.scalar_type() == at::kFloat, "grad_shard_update: src must be bf16 or fp32");
    const int64_t n4 = n / 4;
    if (accumulate)
      hipLaunchKernelGGL(grad_update_f32_kernel<true>, dim3(grid_for(n4, 256)), dim3(256), 0, stream, dst.data_ptr<float>(), src.data_ptr<float>(), s, n4);
    else
      hipLaunchKernelGGL(grad_update_f32_kernel<false>, dim3(grid_for(n4, 256)), dim3(256), 0, stream, dst.data_ptr<float>(), src.data_ptr<float>(), s, n4);
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
}
