// Upcast of low-precision stored weights into a compute-dtype scratch tensor (layerwise casting).
//
// The reference's LayerwiseCastingHook (`/root/reference/src/accelerate/hooks.py:757-783`) calls `module.to(compute)`
// before every forward and `module.to(storage)` after it: two elementwise passes over the weights per forward, and the
// storage copy is rebuilt each time. Here the storage tensor stays resident (fp8 e4m3 / e5m2, fp16 or bf16) and each
// forward reads it once into a compute-dtype scratch tensor (bf16 / fp16 / fp32) that is dropped after the forward:
// one pass, half the HBM traffic of the reference's pair, no downcast at all. All of a module's parameters go in one
// launch (a small per-tensor table in kernel arguments). fp8 decodes use gfx950's OCP-format converts
// (v_cvt_pk_f32_fp8 / _bf8), 8 elements per lane per step.
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include "common.h"

namespace acc {

namespace {

enum : int { kF8E4M3 = 0, kF8E5M2 = 1, kF16 = 2, kBF16 = 3, kF32 = 4 };

constexpr int kMaxCastTensors = 8;

struct CastTable {
  const void* src[kMaxCastTensors];
  void* dst[kMaxCastTensors];
  long n[kMaxCastTensors];
  long block0[kMaxCastTensors + 1];  // first workgroup of tensor t (prefix sums), block0[count] = grid
  int count;
};

__device__ __forceinline__ void decode8(const void* src, long i, int st, float (&v)[8]) {
  if (st == kF8E4M3 || st == kF8E5M2) {
    const uint2 w = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(src) + i);
    const int lo = (int)w.x, hi = (int)w.y;
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2 a, b, c, d;
    if (st == kF8E4M3) {
      a = __builtin_amdgcn_cvt_pk_f32_fp8(lo, false); b = __builtin_amdgcn_cvt_pk_f32_fp8(lo, true);
      c = __builtin_amdgcn_cvt_pk_f32_fp8(hi, false); d = __builtin_amdgcn_cvt_pk_f32_fp8(hi, true);
    } else {
      a = __builtin_amdgcn_cvt_pk_f32_bf8(lo, false); b = __builtin_amdgcn_cvt_pk_f32_bf8(lo, true);
      c = __builtin_amdgcn_cvt_pk_f32_bf8(hi, false); d = __builtin_amdgcn_cvt_pk_f32_bf8(hi, true);
    }
    v[0] = a[0]; v[1] = a[1]; v[2] = b[0]; v[3] = b[1]; v[4] = c[0]; v[5] = c[1]; v[6] = d[0]; v[7] = d[1];
  } else if (st == kBF16) {
    const bf16x8 w = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16_t*>(src) + i);
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = bf2f(w.v[u]);
  } else if (st == kF16) {
    const uint4 w = *reinterpret_cast<const uint4*>(reinterpret_cast<const __half*>(src) + i);
    const __half* h = reinterpret_cast<const __half*>(&w);
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __half2float(h[u]);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src) + i);
    const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src) + i + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

__device__ __forceinline__ float decode1(const void* src, long i, int st) {
  if (st == kF8E4M3 || st == kF8E5M2) {
    const int b = reinterpret_cast<const uint8_t*>(src)[i];
    return st == kF8E4M3 ? __builtin_amdgcn_cvt_pk_f32_fp8(b, false)[0] : __builtin_amdgcn_cvt_pk_f32_bf8(b, false)[0];
  }
  if (st == kBF16) return bf2f(reinterpret_cast<const bf16_t*>(src)[i]);
  if (st == kF16) return __half2float(reinterpret_cast<const __half*>(src)[i]);
  return reinterpret_cast<const float*>(src)[i];
}

template <int DT>
__device__ __forceinline__ void store8(void* dst, long i, const float (&v)[8]) {
  if constexpr (DT == kBF16) {
    bf16x8 w;
#pragma unroll
    for (int u = 0; u < 8; ++u) w.v[u] = f2bf(v[u]);
    *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16_t*>(dst) + i) = w;
  } else if constexpr (DT == kF16) {
    uint4 w;
    __half* h = reinterpret_cast<__half*>(&w);
#pragma unroll
    for (int u = 0; u < 8; ++u) h[u] = __float2half(v[u]);
    *reinterpret_cast<uint4*>(reinterpret_cast<__half*>(dst) + i) = w;
  } else {
    float* p = reinterpret_cast<float*>(dst) + i;
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <int DT>
__device__ __forceinline__ void store1(void* dst, long i, float v) {
  if constexpr (DT == kBF16) reinterpret_cast<bf16_t*>(dst)[i] = f2bf(v);
  else if constexpr (DT == kF16) reinterpret_cast<__half*>(dst)[i] = __float2half(v);
  else reinterpret_cast<float*>(dst)[i] = v;
}

constexpr int kCastThreads = 256;
constexpr long kCastPerBlock = 8L * kCastThreads * 4;  // 4 steps of 8 elements per lane

// Workgroup b belongs to the tensor t with block0[t] <= b < block0[t + 1]; it converts elements
// [(b - block0[t]) * kCastPerBlock, +kCastPerBlock) of it. Every pointer is 16-B aligned (checked on the host) and the
// per-step index is a multiple of 8, so the 8-wide loads / stores stay aligned; the last partial group goes element by
// element.
template <int ST, int DT>
__global__ __launch_bounds__(kCastThreads) void upcast_multi_kernel(const CastTable tab) {
  int t = 0;
  while (t + 1 < tab.count && (long)blockIdx.x >= tab.block0[t + 1]) ++t;
  ACC_CHECK_OR_RETURN((long)blockIdx.x >= tab.block0[t] && (long)blockIdx.x < tab.block0[t + 1], kChkCastTable);
  const long n = tab.n[t];
  const long base = ((long)blockIdx.x - tab.block0[t]) * kCastPerBlock;
  const void* src = tab.src[t];
  void* dst = tab.dst[t];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const long i = base + ((long)s * kCastThreads + threadIdx.x) * 8;
    if (i + 8 <= n) {
      float v[8];
      decode8(src, i, ST, v);
      store8<DT>(dst, i, v);
    } else if (i < n) {
      for (long j = i; j < n; ++j) store1<DT>(dst, j, decode1(src, j, ST));
    }
  }
}

int code_of(at::ScalarType t) {
  switch (t) {
    case at::kFloat8_e4m3fn: return kF8E4M3;
    case at::kFloat8_e5m2: return kF8E5M2;
    case at::kHalf: return kF16;
    case at::kBFloat16: return kBF16;
    case at::kFloat: return kF32;
    default: return -1;
  }
}

}  // namespace

}  // namespace acc

using namespace acc;

ACC_DEBUG_TAKE_FN(acc_dbg_take_cast)

// dsts[i] = srcs[i] converted to dsts[i]'s dtype, all pairs in ONE launch (same source dtype and same destination dtype
// across the list; at most 8 tensors). Sources fp8 e4m3 / e5m2, fp16, bf16 or fp32; destinations bf16, fp16 or fp32.
// Returns false (nothing launched) for inputs outside that: the caller casts with torch instead.
bool upcast_multi(std::vector<torch::Tensor> srcs, std::vector<torch::Tensor> dsts) {
  if (srcs.empty() || srcs.size() != dsts.size() || srcs.size() > (size_t)kMaxCastTensors) return false;
  const int st = code_of(srcs[0].scalar_type()), dt = code_of(dsts[0].scalar_type());
  if (st < 0 || !(dt == kBF16 || dt == kF16 || dt == kF32)) return false;
  CastTable tab{};
  long blocks = 0;
  for (size_t k = 0; k < srcs.size(); ++k) {
    const auto& s = srcs[k];
    const auto& d = dsts[k];
    if (!s.is_cuda() || !d.is_cuda() || !s.is_contiguous() || !d.is_contiguous() || s.numel() != d.numel()) return false;
    if (code_of(s.scalar_type()) != st || code_of(d.scalar_type()) != dt) return false;
    if ((reinterpret_cast<uintptr_t>(s.data_ptr()) & 15) || (reinterpret_cast<uintptr_t>(d.data_ptr()) & 15)) return false;
    tab.src[k] = s.data_ptr();
    tab.dst[k] = d.data_ptr();
    tab.n[k] = s.numel();
    tab.block0[k] = blocks;
    blocks += (s.numel() + kCastPerBlock - 1) / kCastPerBlock;
  }
  tab.count = (int)srcs.size();
  tab.block0[tab.count] = blocks;
  if (blocks == 0) return true;
  if (blocks >= (1L << 31)) return false;
  auto stream = at::hip::getCurrentHIPStream();
#define ACC_UPCAST(S, D) hipLaunchKernelGGL((upcast_multi_kernel<S, D>), dim3((unsigned)blocks), dim3(kCastThreads), 0, stream, tab)
#define ACC_UPCAST_DT(S)                   \
  if (dt == kBF16) ACC_UPCAST(S, kBF16);   \
  else if (dt == kF16) ACC_UPCAST(S, kF16); \
  else ACC_UPCAST(S, kF32);
  switch (st) {
    case kF8E4M3: ACC_UPCAST_DT(kF8E4M3) break;
    case kF8E5M2: ACC_UPCAST_DT(kF8E5M2) break;
    case kF16: ACC_UPCAST_DT(kF16) break;
    case kBF16: ACC_UPCAST_DT(kBF16) break;
    default: ACC_UPCAST_DT(kF32) break;
  }
#undef ACC_UPCAST_DT
#undef ACC_UPCAST
  return true;
}
