// Token <-> expert-row movement of the MoE layer (models/moe.py, `_RouteDispatch` / `_RouteCombine`).
//
// Routing gives every (token t, slot k) exactly one row pos[t*K + k] of the routed buffer [R, H] (expert segments
// padded to 64 rows; the pad rows belong to no slot). Both directions are therefore plain row copies with unique
// destinations, or per-token sums over K rows — no atomics:
//   scatter: dst[pos[j]] = (w ? w[j] : 1) * src[j / K]         (dispatch; the combine's backward to the expert rows)
//            with DOT also dotw[j] = <src[j / K], y[pos[j]]>      (the combine's backward to the routing weights)
//   gather : out[t] = sum_k (w ? w[t*K + k] : 1) * src[pos[t*K + k]]   (combine; the dispatch's backward)
// fp32 accumulation, one bf16 rounding per output. One wave per row (scatter) / token (gather), 16-B accesses.
// Replaces torch index_copy / index_select / bf16 index_add (an atomic bf16 read-modify-write per element, ~0.6 TB/s
// on the Mixtral combine) in the non-expert-parallel path.
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include "common.h"

using namespace acc;

namespace {

constexpr int kWaves = 4;  // waves per 256-thread workgroup

template <bool SCALE, bool DOT>
__global__ __launch_bounds__(256) void moe_scatter_kernel(const bf16_t* __restrict__ src, const int64_t* __restrict__ pos,
                                                          const float* __restrict__ w, bf16_t* __restrict__ dst,
                                                          const bf16_t* __restrict__ y, float* __restrict__ dotw,
                                                          long nslots, int K, int H, long R) {
  const long j = (long)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= nslots) return;  // wave-uniform; no barriers in this kernel
  const long r = pos[j];
  ACC_CHECK_OR_RETURN(r >= 0 && r < R, kChkRoutePos);
  const float s = SCALE ? w[j] : 1.f;
  const bf16x8* sp = reinterpret_cast<const bf16x8*>(src + (j / K) * (long)H);
  bf16x8* dp = reinterpret_cast<bf16x8*>(dst + r * (long)H);
  const bf16x8* yp = DOT ? reinterpret_cast<const bf16x8*>(y + r * (long)H) : nullptr;
  float acc = 0.f;
  for (int c = lane; c < H / 8; c += 64) {
    const bf16x8 a = sp[c];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.v[e] = SCALE ? f2bf(bf2f(a.v[e]) * s) : a.v[e];
    dp[c] = o;
    if (DOT) {
      const bf16x8 b = yp[c];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc = fmaf(bf2f(a.v[e]), bf2f(b.v[e]), acc);
    }
  }
  if (DOT) {
    acc = wave_sum(acc);
    if (lane == 0) dotw[j] = acc;
  }
}

template <bool SCALE>
__global__ __launch_bounds__(256) void moe_gather_kernel(const bf16_t* __restrict__ src, const int64_t* __restrict__ pos,
                                                         const float* __restrict__ w, bf16_t* __restrict__ out, long T,
                                                         int K, int H, long R) {
  const long t = (long)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  constexpr int kMaxK = 8;
  const bf16x8* rows[kMaxK];
  float sc[kMaxK];
#pragma unroll
  for (int k = 0; k < kMaxK; ++k) {
    if (k < K) {
      const long r = pos[t * K + k];
      ACC_CHECK_OR_RETURN(r >= 0 && r < R, kChkRoutePos);
      rows[k] = reinterpret_cast<const bf16x8*>(src + r * (long)H);
      sc[k] = SCALE ? w[t * K + k] : 1.f;
    }
  }
  bf16x8* op = reinterpret_cast<bf16x8*>(out + t * (long)H);
  for (int c = lane; c < H / 8; c += 64) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) {
      if (k < K) {
        const bf16x8 a = rows[k][c];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(bf2f(a.v[e]), sc[k], acc[e]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.v[e] = f2bf(acc[e]);
    op[c] = o;
  }
}

void check_rows(const torch::Tensor& x, const char* name) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 2 && x.size(1) % 8 == 0,
              name, ": contiguous 2-D bf16 HIP tensor with a multiple of 8 columns expected");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0, name, " must be 16-byte aligned");
}

}  // namespace

ACC_DEBUG_TAKE_FN(acc_dbg_take_moe_route)

// dst[pos[j]] = w[j] * src[j / K] for every slot j (w optional); with y and dotw also dotw[j] = <src[j / K], y[pos[j]]>.
// Rows of dst that no slot names are left untouched (the caller zeroes them).
void moe_scatter_rows(torch::Tensor src, torch::Tensor pos, c10::optional<torch::Tensor> w, torch::Tensor dst,
                      c10::optional<torch::Tensor> y, c10::optional<torch::Tensor> dotw, int64_t K) {
  check_rows(src, "moe_scatter_rows: src");
  check_rows(dst, "moe_scatter_rows: dst");
  const long T = src.size(0), H = src.size(1), R = dst.size(0), nslots = pos.numel();
  TORCH_CHECK(K >= 1 && nslots == T * K && dst.size(1) == H, "moe_scatter_rows: shapes");
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == at::kLong && pos.is_contiguous(), "moe_scatter_rows: pos must be int64");
  const bool scale = w.has_value(), dot = y.has_value();
  if (scale) TORCH_CHECK(w->is_cuda() && w->scalar_type() == at::kFloat && w->is_contiguous() && w->numel() == nslots, "moe_scatter_rows: w fp32 [T*K]");
  TORCH_CHECK(dot == dotw.has_value() && (!dot || scale), "moe_scatter_rows: y and dotw go together, with w");
  if (dot) {
    check_rows(*y, "moe_scatter_rows: y");
    TORCH_CHECK(y->size(0) == R && y->size(1) == H && dotw->is_cuda() && dotw->scalar_type() == at::kFloat &&
                    dotw->is_contiguous() && dotw->numel() == nslots, "moe_scatter_rows: y / dotw shapes");
  }
  if (nslots == 0) return;
  const dim3 grid((nslots + kWaves - 1) / kWaves);
  auto stream = at::hip::getCurrentHIPStream();
  const bf16_t* sp = reinterpret_cast<const bf16_t*>(src.data_ptr());
  bf16_t* dp = reinterpret_cast<bf16_t*>(dst.data_ptr());
  const int64_t* pp = pos.data_ptr<int64_t>();
  const float* wp = scale ? w->data_ptr<float>() : nullptr;
  if (dot)
    hipLaunchKernelGGL((moe_scatter_kernel<true, true>), grid, dim3(256), 0, stream, sp, pp, wp, dp,
                       reinterpret_cast<const bf16_t*>(y->data_ptr()), dotw->data_ptr<float>(), nslots, (int)K, (int)H, R);
  else if (scale)
    hipLaunchKernelGGL((moe_scatter_kernel<true, false>), grid, dim3(256), 0, stream, sp, pp, wp, dp, nullptr, nullptr,
                       nslots, (int)K, (int)H, R);
  else
    hipLaunchKernelGGL((moe_scatter_kernel<false, false>), grid, dim3(256), 0, stream, sp, pp, nullptr, dp, nullptr,
                       nullptr, nslots, (int)K, (int)H, R);
}

// out[t] = sum_k w[t*K + k] * src[pos[t*K + k]] (w optional: plain sum), out [T, H] bf16.
torch::Tensor moe_gather_rows(torch::Tensor src, torch::Tensor pos, c10::optional<torch::Tensor> w, int64_t T, int64_t K) {
  check_rows(src, "moe_gather_rows: src");
  TORCH_CHECK(K >= 1 && K <= 8 && pos.numel() == T * K, "moe_gather_rows: 1 <= K <= 8 and pos [T*K]");
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == at::kLong && pos.is_contiguous(), "moe_gather_rows: pos must be int64");
  const bool scale = w.has_value();
  if (scale) TORCH_CHECK(w->is_cuda() && w->scalar_type() == at::kFloat && w->is_contiguous() && w->numel() == T * K, "moe_gather_rows: w fp32 [T*K]");
  const long H = src.size(1), R = src.size(0);
  auto out = torch::empty({T, H}, src.options());
  if (T == 0) return out;
  const dim3 grid((T + kWaves - 1) / kWaves);
  auto stream = at::hip::getCurrentHIPStream();
  const bf16_t* sp = reinterpret_cast<const bf16_t*>(src.data_ptr());
  bf16_t* op = reinterpret_cast<bf16_t*>(out.data_ptr());
  if (scale)
    hipLaunchKernelGGL((moe_gather_kernel<true>), grid, dim3(256), 0, stream, sp, pos.data_ptr<int64_t>(), w->data_ptr<float>(),
                       op, T, (int)K, (int)H, R);
  else
    hipLaunchKernelGGL((moe_gather_kernel<false>), grid, dim3(256), 0, stream, sp, pos.data_ptr<int64_t>(), nullptr, op, T,
                       (int)K, (int)H, R);
  return out;
}
