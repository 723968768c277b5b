// Memory-bound fused kernels for the transformer block (bf16 activations, fp32 math):
//   * RMSNorm forward (optionally fused with the residual add) and backward (dx + dweight),
//   * SwiGLU forward/backward on the fused [gate | up] projection output,
//   * rotary embedding (rotate-half convention) applied in place to the Q and K heads of a fused QKV buffer.
// All loads/stores are 16 B per lane (8 x bf16); one row per workgroup for the row-wise kernels.
// fp8 producer amax: given an `amax_part` buffer, each kernel also writes the max |output| of every workgroup (of the
// bf16 values it stores, so the result equals a separate amax pass bit for bit); `amax_finalize` folds the partials
// into the fp32 [1] amax the fp8 cast and GEMM read. That replaces a full re-read of the tensor by the amax kernel.
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"
#include <cstdlib>

using namespace acc;

namespace {

constexpr int kNormThreads = 256;

template <int VPT>
__global__ __launch_bounds__(kNormThreads) void rmsnorm_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, const bf16_t* __restrict__ w,
    bf16_t* __restrict__ y, bf16_t* __restrict__ res_out, float* __restrict__ rstd_out, int H, float eps,
    float* __restrict__ amax_part) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = H >> 3;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)row * H);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nvec) {
      bf16x8 a = xr[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = bf2f(a.v[j]);
      if (res != nullptr) {
        bf16x8 b = reinterpret_cast<const bf16x8*>(res + (size_t)row * H)[c];
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s.v[j] = f2bf(v[i][j] + bf2f(b.v[j]));
          v[i][j] = bf2f(s.v[j]);  // normalise exactly what is stored in the residual stream
        }
        reinterpret_cast<bf16x8*>(res_out + (size_t)row * H)[c] = s;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float r = rsqrtf(ss / (float)H + eps);
  if (threadIdx.x == 0) rstd_out[row] = r;
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(w);
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + (size_t)row * H);
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nvec) {
      bf16x8 ww = wr[c], o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o.v[j] = f2bf(v[i][j] * r * bf2f(ww.v[j]));
        m = fmaxf(m, fabsf(bf2f(o.v[j])));
      }
      yr[c] = o;
    }
  }
  if (amax_part != nullptr) {
    m = block_max(m, scratch);
    if (threadIdx.x == 0) amax_part[row] = m;
  }
}

// dx = rstd * (dy*w - xhat * mean(dy*w*xhat)) (+ dres); per-block partial dweight in fp32.
template <int VPT>
__global__ __launch_bounds__(kNormThreads) void rmsnorm_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
    const float* __restrict__ rstd, const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
    float* __restrict__ dw_part, int T, int H, float* __restrict__ amax_part) {
  __shared__ float scratch[2][kNormThreads / 64];  // wave partials, alternating per row (one barrier per row)
  float m = 0.f;
  const int nvec = H >> 3;
  float wv[VPT][8], dwacc[VPT][8];
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(w);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = 0.f;
    if (c < nvec) {
      bf16x8 ww = wr[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) wv[i][j] = bf2f(ww.v[j]);
    }
  }
  // The next row's x / dy / dres / rstd are loaded while this row is reduced and written: one block walks T / grid
  // rows in sequence, and without the prefetch every row paid a full HBM latency after the previous row's barrier.
  // Only up to VPT = 2 (H <= 4096): wider rows would lose the second resident block per CU to the extra registers.
  constexpr bool kPrefetch = VPT <= 2;
  bf16x8 xa[VPT] = {}, xd[VPT] = {}, xr[VPT] = {};
  float rn = 0.f;
  auto load_row = [&](int rw) {
    rn = rstd[rw];
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * kNormThreads;
      if (c < nvec) {
        xa[i] = reinterpret_cast<const bf16x8*>(x + (size_t)rw * H)[c];
        xd[i] = reinterpret_cast<const bf16x8*>(dy + (size_t)rw * H)[c];
        if (dres != nullptr) xr[i] = reinterpret_cast<const bf16x8*>(dres + (size_t)rw * H)[c];
      }
    }
  };
  if (kPrefetch && (int)blockIdx.x < T) load_row(blockIdx.x);
  int parity = 0;
  for (int row = blockIdx.x; row < T; row += gridDim.x, parity ^= 1) {
    float r;
    bf16x8 ca[VPT], cd[VPT], cr[VPT];
    if constexpr (kPrefetch) {
      r = rn;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        ca[i] = xa[i];
        cd[i] = xd[i];
        cr[i] = xr[i];
      }
      if (row + (int)gridDim.x < T) load_row(row + gridDim.x);
    } else {
      r = rstd[row];
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int c = threadIdx.x + i * kNormThreads;
        if (c < nvec) {
          ca[i] = reinterpret_cast<const bf16x8*>(x + (size_t)row * H)[c];
          cd[i] = reinterpret_cast<const bf16x8*>(dy + (size_t)row * H)[c];
          if (dres != nullptr) cr[i] = reinterpret_cast<const bf16x8*>(dres + (size_t)row * H)[c];
        }
      }
    }
    float xh[VPT][8], g[VPT][8];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * kNormThreads;
      if (c < nvec) {
        const bf16x8 a = ca[i];
        const bf16x8 d = cd[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = bf2f(a.v[j]) * r;
          const float dd = bf2f(d.v[j]);
          g[i][j] = dd * wv[i][j];
          dwacc[i][j] += dd * xh[i][j];
          dot += g[i][j] * xh[i][j];
        }
      }
    }
    {  // block sum in one barrier: the row after next writes this parity's slots only after the next row's barrier
      dot = wave_sum(dot);
      if ((threadIdx.x & 63) == 0) scratch[parity][threadIdx.x >> 6] = dot;
      __syncthreads();
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < kNormThreads / 64; ++k) t += scratch[parity][k];
      dot = t / (float)H;
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * kNormThreads;
      if (c < nvec) {
        bf16x8 o;
        const bf16x8 rr = cr[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float val = r * (g[i][j] - xh[i][j] * dot);
          if (dres != nullptr) val += bf2f(rr.v[j]);
          o.v[j] = f2bf(val);
          m = fmaxf(m, fabsf(bf2f(o.v[j])));
        }
        reinterpret_cast<bf16x8*>(dx + (size_t)row * H)[c] = o;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nvec) {
      float4* dst = reinterpret_cast<float4*>(dw_part + (size_t)blockIdx.x * H + c * 8);
      dst[0] = make_float4(dwacc[i][0], dwacc[i][1], dwacc[i][2], dwacc[i][3]);
      dst[1] = make_float4(dwacc[i][4], dwacc[i][5], dwacc[i][6], dwacc[i][7]);
    }
  }
  if (amax_part != nullptr) {
    m = block_max(m, &scratch[0][0]);
    if (threadIdx.x == 0) amax_part[blockIdx.x] = m;
  }
}

// Column sum of the [P, H] fp32 partials → dweight (bf16 or fp32 output). 256 threads = 32 columns x 8 row
// groups; each row group strides over the partial rows, then the 8 partial sums are combined through LDS.
__device__ __forceinline__ float as_float(float v) { return v; }
__device__ __forceinline__ float as_float(bf16_t v) { return bf2f(v); }

// ACC: add into `out` (a weight-gradient slot that already holds earlier micro-batches' gradient) instead of
// overwriting it.
template <typename OutT, bool ACC = false>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, OutT* __restrict__ out, int P, int H) {
  __shared__ float red[8][33];
  const int c = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + c;
  // eight independent partial sums: eight loads in flight per lane (one dependent chain left the kernel latency-bound,
  // 18 us for 8 MB of partials)
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < H) {
    int p = rg;
    for (; p + 56 < P; p += 64) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += part[(size_t)(p + 8 * u) * H + col];
    }
    for (; p < P; p += 8) acc[0] += part[(size_t)p * H + col];
  }
  const float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  red[rg][c] = s;
  __syncthreads();
  if (rg == 0 && col < H) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += red[g][c];
    if (ACC) t += as_float(out[col]);
    out[col] = from_f<OutT>(t);
  }
}

// ---------------------------------------------------------------------------------------------------
// SwiGLU on a fused [T, 2F] buffer: gate = gu[:, :F], up = gu[:, F:]; h = silu(gate) * up.
// ---------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ h, long T,
                                                         int F, float* __restrict__ amax_part) {
  __shared__ float scratch[16];
  float m = 0.f;
  const long nvec_row = F >> 3;
  const long total = T * nvec_row;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const long row = idx / nvec_row, c = idx - row * nvec_row;
    const bf16x8 g = reinterpret_cast<const bf16x8*>(gu + row * 2 * F)[c];
    const bf16x8 u = reinterpret_cast<const bf16x8*>(gu + row * 2 * F + F)[c];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g.v[j]);
      const float s = gf / (1.f + __expf(-gf));
      o.v[j] = f2bf(s * bf2f(u.v[j]));
      m = fmaxf(m, fabsf(bf2f(o.v[j])));
    }
    reinterpret_cast<bf16x8*>(h + row * F)[c] = o;
  }
  if (amax_part != nullptr) {
    m = block_max(m, scratch);
    if (threadIdx.x == 0) amax_part[blockIdx.x] = m;
  }
}

// dgate = dh * up * sig * (1 + g*(1-sig)), dup = dh * silu(g). Written into dgu [T, 2F].
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dh,
                                                         bf16_t* __restrict__ dgu, long T, int F,
                                                         float* __restrict__ amax_part) {
  __shared__ float scratch[16];
  float m = 0.f;
  const long nvec_row = F >> 3;
  const long total = T * nvec_row;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const long row = idx / nvec_row, c = idx - row * nvec_row;
    const bf16x8 g = reinterpret_cast<const bf16x8*>(gu + row * 2 * F)[c];
    const bf16x8 u = reinterpret_cast<const bf16x8*>(gu + row * 2 * F + F)[c];
    const bf16x8 d = reinterpret_cast<const bf16x8*>(dh + row * F)[c];
    bf16x8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g.v[j]), uf = bf2f(u.v[j]), df = bf2f(d.v[j]);
      const float sig = 1.f / (1.f + __expf(-gf));
      const float silu = gf * sig;
      og.v[j] = f2bf(df * uf * sig * (1.f + gf * (1.f - sig)));
      ou.v[j] = f2bf(df * silu);
      m = fmaxf(m, fmaxf(fabsf(bf2f(og.v[j])), fabsf(bf2f(ou.v[j]))));
    }
    reinterpret_cast<bf16x8*>(dgu + row * 2 * F)[c] = og;
    reinterpret_cast<bf16x8*>(dgu + row * 2 * F + F)[c] = ou;
  }
  if (amax_part != nullptr) {
    m = block_max(m, scratch);
    if (threadIdx.x == 0) amax_part[blockIdx.x] = m;
  }
}

// ---------------------------------------------------------------------------------------------------
// RoPE on qkv [T, (Hq + 2*Hkv) * D] (rotate-half pairs (i, i + D/2)); heads [0, Hq + Hkv) are rotated (Q and K),
// V passes through. cos/sin tables are fp32 [S, D/2]; position = pos[t] (or t % S). sign = +1 forward, -1 backward
// (inverse rotation of the incoming gradient). Out of place (src != dst: one read + one write of the whole row, V
// copied) or in place (src == dst, heads_iter = n_rot_heads: V never touched).
// ---------------------------------------------------------------------------------------------------
// W pairs per thread step (W bf16 = 8 or 16 B of each half): 16-B accesses whenever D / 2 is a multiple of 8.
template <int W>
__global__ void rope_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, const float* __restrict__ cosb,
                            const float* __restrict__ sinb, const int64_t* __restrict__ pos, long T, int S,
                            int n_rot_heads, int heads_iter, int n_heads_total, int D, float sign) {
  using vec = typename std::conditional<W == 8, bf16x8, bf16x4>::type;
  const int half = D >> 1;
  const int nvec = half / W;
  const long per_row = (long)heads_iter * nvec;
  const long total = T * per_row;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const long t = idx / per_row;
    const int rem = (int)(idx - t * per_row);
    const int h = rem / nvec, c = rem - h * nvec;
    const long off = (t * n_heads_total + h) * (long)D;
    const vec a = reinterpret_cast<const vec*>(src + off)[c];
    const vec b = reinterpret_cast<const vec*>(src + off + half)[c];
    vec oa = a, ob = b;
    if (h < n_rot_heads) {
      const long p = pos != nullptr ? pos[t] : (t % S);
      ACC_CHECK(p >= 0 && p < S, kChkRopePos);  // debug build: a position past the cos / sin table
      if (ACC_DEBUG_BUILD && (p < 0 || p >= S)) continue;
      float cc[W], ss[W];
#pragma unroll
      for (int q = 0; q < W / 4; ++q) {
        const float4 cs = reinterpret_cast<const float4*>(cosb + p * half)[c * (W / 4) + q];
        const float4 sn = reinterpret_cast<const float4*>(sinb + p * half)[c * (W / 4) + q];
        cc[4 * q] = cs.x; cc[4 * q + 1] = cs.y; cc[4 * q + 2] = cs.z; cc[4 * q + 3] = cs.w;
        ss[4 * q] = sn.x * sign; ss[4 * q + 1] = sn.y * sign; ss[4 * q + 2] = sn.z * sign; ss[4 * q + 3] = sn.w * sign;
      }
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const float x1 = bf2f(a.v[j]), x2 = bf2f(b.v[j]);
        oa.v[j] = f2bf(x1 * cc[j] - x2 * ss[j]);
        ob.v[j] = f2bf(x2 * cc[j] + x1 * ss[j]);
      }
    }
    reinterpret_cast<vec*>(dst + off)[c] = oa;
    reinterpret_cast<vec*>(dst + off + half)[c] = ob;
  }
}

// max over n per-workgroup partials -> out[0] (one 1024-thread workgroup; n is at most a few thousand)
__global__ __launch_bounds__(1024) void amax_finalize_kernel(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float scratch[16];
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) m = fmaxf(m, part[i]);
  m = block_max(m, scratch);
  if (threadIdx.x == 0) out[0] = m;
}

inline int grid_for(long work, int threads) {
  long g = (work + threads - 1) / threads;
  if (g > 256 * 8) g = 256 * 8;  // 8 resident blocks per CU, grid-stride the rest
  if (g < 1) g = 1;
  return (int)g;
}

void check_bf16_cuda(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a HIP tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// Partial-max buffer for a producer kernel with `blocks` workgroups (nullptr when no amax is requested).
struct AmaxOut {
  torch::Tensor part;
  float* out = nullptr;
  float* ptr() const { return out ? part.data_ptr<float>() : nullptr; }
  AmaxOut(const c10::optional<torch::Tensor>& amax, long blocks, const torch::Tensor& like) {
    if (!amax.has_value()) return;
    TORCH_CHECK(amax->is_cuda() && amax->scalar_type() == at::kFloat && amax->numel() >= 1, "amax must be a fp32 [1] HIP tensor");
    part = torch::empty({std::max<long>(blocks, 1)}, like.options().dtype(torch::kFloat32));
    out = amax->data_ptr<float>();
  }
  void finalize(long blocks) const {
    if (out == nullptr) return;
    if (blocks <= 0) {
      hipMemsetAsync(out, 0, sizeof(float), at::hip::getCurrentHIPStream());
      return;
    }
    hipLaunchKernelGGL(amax_finalize_kernel, dim3(1), dim3(1024), 0, at::hip::getCurrentHIPStream(), part.data_ptr<float>(),
                       (int)blocks, out);
  }
};

}  // namespace

ACC_DEBUG_TAKE_FN(acc_dbg_take_norm_act)

// ----------------------------------------------------------------------------------------- host API
std::vector<torch::Tensor> rmsnorm_fwd(torch::Tensor x, c10::optional<torch::Tensor> residual, torch::Tensor w,
                                       double eps, c10::optional<torch::Tensor> amax) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "weight");
  const int H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && H <= 8 * 256 * 8, "rmsnorm: hidden size must be a multiple of 8 and <= 16384");
  const long T = x.numel() / H;
  auto y = torch::empty_like(x);
  auto rstd = torch::empty({T}, x.options().dtype(torch::kFloat32));
  torch::Tensor res_out;
  const bf16_t* resp = nullptr;
  bf16_t* resop = nullptr;
  if (residual.has_value()) {
    check_bf16_cuda(*residual, "residual");
    res_out = torch::empty_like(x);
    resp = reinterpret_cast<const bf16_t*>(residual->data_ptr());
    resop = reinterpret_cast<bf16_t*>(res_out.data_ptr());
  }
  const AmaxOut am(amax, T, x);
  if (T == 0) {
    am.finalize(0);
    return {y, rstd, res_out};
  }
  auto stream = at::hip::getCurrentHIPStream();
  const int vpt = (H / 8 + kNormThreads - 1) / kNormThreads;
#define LAUNCH_FWD(V)                                                                                             \
  hipLaunchKernelGGL(rmsnorm_fwd_kernel<V>, dim3(T), dim3(kNormThreads), 0, stream,                              \
                     reinterpret_cast<const bf16_t*>(x.data_ptr()), resp, reinterpret_cast<const bf16_t*>(w.data_ptr()), \
                     reinterpret_cast<bf16_t*>(y.data_ptr()), resop, rstd.data_ptr<float>(), H, (float)eps, am.ptr())
  if (vpt <= 1) LAUNCH_FWD(1);
  else if (vpt <= 2) LAUNCH_FWD(2);
  else if (vpt <= 4) LAUNCH_FWD(4);
  else LAUNCH_FWD(8);
#undef LAUNCH_FWD
  am.finalize(T);
  return {y, rstd, res_out};
}

// dw_out: write dweight straight into this [H] fp32 / bf16 tensor (an FSDP weight-gradient slot; `accumulate` adds to
// it) instead of a new bf16 tensor that autograd would then add into the slot.
std::vector<torch::Tensor> rmsnorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor rstd,
                                       c10::optional<torch::Tensor> dres, c10::optional<torch::Tensor> amax,
                                       c10::optional<torch::Tensor> dw_out, bool accumulate) {
  check_bf16_cuda(dy, "dy");
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "weight");
  const int H = x.size(-1);
  const long T = x.numel() / H;
  auto dx = torch::empty_like(x);
  // workgroups (each walks T / P rows, one row prefetched): ACCELERATE_RMSNORM_BWD_BLOCKS, default 512
  static const long bwd_blocks = [] { const char* e = std::getenv("ACCELERATE_RMSNORM_BWD_BLOCKS"); return e ? std::atol(e) : 512L; }();
  const int P = (int)std::min<long>(T > 0 ? T : 1, bwd_blocks);
  auto part = torch::empty({P, H}, x.options().dtype(torch::kFloat32));
  torch::Tensor dw;
  if (dw_out.has_value()) {
    dw = *dw_out;
    TORCH_CHECK(dw.is_cuda() && dw.is_contiguous() && dw.numel() == H &&
                    (dw.scalar_type() == at::kFloat || dw.scalar_type() == at::kBFloat16),
                "rmsnorm_bwd: dw_out must be a contiguous fp32 / bf16 HIP tensor of H elements");
  } else {
    dw = torch::empty({H}, w.options());
    accumulate = false;
  }
  auto stream = at::hip::getCurrentHIPStream();
  const bf16_t* dresp = nullptr;
  if (dres.has_value()) {
    check_bf16_cuda(*dres, "dres");
    dresp = reinterpret_cast<const bf16_t*>(dres->data_ptr());
  }
  const AmaxOut am(amax, P, x);
  if (T == 0) {
    if (!accumulate) dw.zero_();
    am.finalize(0);
    return {dx, dw};
  }
  const int vpt = (H / 8 + kNormThreads - 1) / kNormThreads;
#define LAUNCH_BWD(V)                                                                                             \
  hipLaunchKernelGGL(rmsnorm_bwd_kernel<V>, dim3(P), dim3(kNormThreads), 0, stream,                              \
                     reinterpret_cast<const bf16_t*>(dy.data_ptr()), reinterpret_cast<const bf16_t*>(x.data_ptr()), \
                     reinterpret_cast<const bf16_t*>(w.data_ptr()), rstd.data_ptr<float>(), dresp,               \
                     reinterpret_cast<bf16_t*>(dx.data_ptr()), part.data_ptr<float>(), (int)T, H, am.ptr())
  if (vpt <= 1) LAUNCH_BWD(1);
  else if (vpt <= 2) LAUNCH_BWD(2);
  else if (vpt <= 4) LAUNCH_BWD(4);
  else LAUNCH_BWD(8);
#undef LAUNCH_BWD
  const dim3 cgrid((H + 31) / 32);
  if (dw.scalar_type() == at::kFloat) {
    if (accumulate) hipLaunchKernelGGL((colsum_kernel<float, true>), cgrid, dim3(256), 0, stream, part.data_ptr<float>(), dw.data_ptr<float>(), P, H);
    else hipLaunchKernelGGL((colsum_kernel<float, false>), cgrid, dim3(256), 0, stream, part.data_ptr<float>(), dw.data_ptr<float>(), P, H);
  } else {
    bf16_t* o = reinterpret_cast<bf16_t*>(dw.data_ptr());
    if (accumulate) hipLaunchKernelGGL((colsum_kernel<bf16_t, true>), cgrid, dim3(256), 0, stream, part.data_ptr<float>(), o, P, H);
    else hipLaunchKernelGGL((colsum_kernel<bf16_t, false>), cgrid, dim3(256), 0, stream, part.data_ptr<float>(), o, P, H);
  }
  am.finalize(P);
  return {dx, dw};
}

torch::Tensor swiglu_fwd(torch::Tensor gu, c10::optional<torch::Tensor> amax) {
  check_bf16_cuda(gu, "gate_up");
  const int F = gu.size(-1) / 2;
  TORCH_CHECK(F % 8 == 0, "swiglu: intermediate size must be a multiple of 8");
  const long T = gu.numel() / (2 * F);
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto h = torch::empty(sizes, gu.options());
  const long work = T * (F / 8);
  const int g = grid_for(work, 256);
  const AmaxOut am(amax, g, gu);
  if (work == 0) {
    am.finalize(0);
    return h;
  }
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(g), dim3(256), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16_t*>(gu.data_ptr()), reinterpret_cast<bf16_t*>(h.data_ptr()), T, F, am.ptr());
  am.finalize(g);
  return h;
}

torch::Tensor swiglu_bwd(torch::Tensor gu, torch::Tensor dh, c10::optional<torch::Tensor> amax) {
  check_bf16_cuda(gu, "gate_up");
  check_bf16_cuda(dh, "dh");
  const int F = gu.size(-1) / 2;
  const long T = gu.numel() / (2 * F);
  auto dgu = torch::empty_like(gu);
  const long work = T * (F / 8);
  const int g = grid_for(work, 256);
  const AmaxOut am(amax, g, gu);
  if (work == 0) {
    am.finalize(0);
    return dgu;
  }
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(g), dim3(256), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16_t*>(gu.data_ptr()), reinterpret_cast<const bf16_t*>(dh.data_ptr()),
                     reinterpret_cast<bf16_t*>(dgu.data_ptr()), T, F, am.ptr());
  am.finalize(g);
  return dgu;
}

static void rope_launch(const torch::Tensor& src, torch::Tensor& dst, const torch::Tensor& cos, const torch::Tensor& sin,
                        const c10::optional<torch::Tensor>& pos, int64_t n_rot_heads, int64_t n_heads_total,
                        int64_t head_dim, double sign) {
  check_bf16_cuda(src, "qkv");
  check_bf16_cuda(dst, "out");
  TORCH_CHECK(src.numel() == dst.numel(), "rope: src / dst size mismatch");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat, "rope tables must be fp32");
  TORCH_CHECK(head_dim % 8 == 0, "rope: head_dim must be a multiple of 8");
  TORCH_CHECK(src.numel() % (n_heads_total * head_dim) == 0 && n_rot_heads <= n_heads_total, "rope: bad head counts");
  const long T = src.numel() / (n_heads_total * head_dim);
  const int S = cos.size(0);
  TORCH_CHECK(cos.numel() >= (long)S * (head_dim / 2) && sin.numel() == cos.numel(), "rope: tables must be [S, D/2]");
  const int64_t* posp = nullptr;
  if (pos.has_value()) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->numel() == T, "rope: positions must be int64 [T]");
    posp = pos->data_ptr<int64_t>();
  }
  const bool inplace = src.data_ptr() == dst.data_ptr();
  const int heads_iter = (int)(inplace ? n_rot_heads : n_heads_total);
  const bool wide = (head_dim / 2) % 8 == 0;
  const long work = T * heads_iter * (head_dim / (wide ? 16 : 8));
  if (work == 0) return;
#define ROPE_GO(W_)                                                                                                  \
  hipLaunchKernelGGL(rope_kernel<W_>, dim3(grid_for(work, 256)), dim3(256), 0, at::hip::getCurrentHIPStream(),      \
                     reinterpret_cast<const bf16_t*>(src.data_ptr()), reinterpret_cast<bf16_t*>(dst.data_ptr()),   \
                     cos.data_ptr<float>(), sin.data_ptr<float>(), posp, T, S, (int)n_rot_heads, heads_iter,       \
                     (int)n_heads_total, (int)head_dim, (float)sign)
  if (wide) ROPE_GO(8);
  else ROPE_GO(4);
#undef ROPE_GO
}

void rope_inplace(torch::Tensor qkv, torch::Tensor cos, torch::Tensor sin, c10::optional<torch::Tensor> pos,
                  int64_t n_rot_heads, int64_t n_heads_total, int64_t head_dim, double sign) {
  TORCH_CHECK(qkv.is_contiguous(), "rope_inplace: qkv must be contiguous");
  rope_launch(qkv, qkv, cos, sin, pos, n_rot_heads, n_heads_total, head_dim, sign);
}

// Out-of-place RoPE: a new contiguous tensor (one pass over src instead of clone + in-place rotation).
torch::Tensor rope_out(torch::Tensor src, torch::Tensor cos, torch::Tensor sin, c10::optional<torch::Tensor> pos,
                       int64_t n_rot_heads, int64_t n_heads_total, int64_t head_dim, double sign) {
  auto s = src.contiguous();
  auto out = torch::empty_like(s);
  rope_launch(s, out, cos, sin, pos, n_rot_heads, n_heads_total, head_dim, sign);
  return out;
}

// ------------------------------------------------------------------------------------------------ transpose
// out[c, r] = in[r, c] for a row-major bf16 [R, C]. Used to hand the weight-gradient GEMM a token-contiguous copy of
// the layer input (parallel/fsdp.py), which moves that GEMM from the slow both-token-major layout to the
// dgrad-class layout, and for the MoE expert stacks.
//
// 128 x 128 tile per 256-thread workgroup (R, C multiples of 128): every thread moves 8 rows x 16 B in (coalesced
// 256-B row segments), the tile sits in LDS as 256-B rows with the 16-B chunk XOR-swizzled by the row's 8-row block,
// then every thread takes one 8 x 8 block back with eight ds_read_b128 (conflict-free under the swizzle), turns it in
// registers (v_perm) and writes eight 16-B pieces; the 16 threads sharing an output row write 256 contiguous bytes.
// R or C not a multiple of 128 (but of 64) take the 64 x 64 LDS-element kernel below.
namespace {
__device__ __forceinline__ unsigned lo_pair(unsigned a, unsigned b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }
__device__ __forceinline__ unsigned hi_pair(unsigned a, unsigned b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

__global__ __launch_bounds__(256) void transpose128_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                                int R, int C) {
  __shared__ __attribute__((aligned(16))) uint4 tile[128 * 16];  // 128 rows x 16 chunks of 16 B
  const int tid = threadIdx.x;
  const long tr = (long)blockIdx.y * 128, tc = (long)blockIdx.x * 128;
  in += (long)blockIdx.z * R * C;  // batched [E, R, C] -> [E, C, R]
  out += (long)blockIdx.z * R * C;
  // load: thread -> chunk (tid & 15) of rows (tid >> 4) + 16 p
  {
    const int ch = tid & 15;
    uint4 v[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int row = (tid >> 4) + 16 * p;
      v[p] = *reinterpret_cast<const uint4*>(in + (tr + row) * C + tc + ch * 8);
    }
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int row = (tid >> 4) + 16 * p;
      tile[row * 16 + (ch ^ ((row >> 3) & 15))] = v[p];
    }
  }
  __syncthreads();
  // turn: thread -> 8 x 8 block (row block rb, column chunk cb); lanes with consecutive rb share an output row
  const int rb = tid & 15, cb = tid >> 4;
  unsigned x[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 t = tile[(rb * 8 + i) * 16 + (cb ^ rb)];
    x[i][0] = t.x; x[i][1] = t.y; x[i][2] = t.z; x[i][3] = t.w;
  }
  // output row j = column cb*8 + j: elements x[0..7][j]; dword k packs rows 2k, 2k+1
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint4 w;
    unsigned d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      d[k] = (j & 1) ? hi_pair(x[2 * k][j >> 1], x[2 * k + 1][j >> 1]) : lo_pair(x[2 * k][j >> 1], x[2 * k + 1][j >> 1]);
    w.x = d[0]; w.y = d[1]; w.z = d[2]; w.w = d[3];
    *reinterpret_cast<uint4*>(out + (tc + cb * 8 + j) * R + tr + rb * 8) = w;
  }
}

// 64 x 64 fallback: the turn done element-wise through a padded LDS tile (row pitch 72 elements).
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out, int R,
                                                             int C) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[64][72];
  const int tr = blockIdx.y * 64, tc = blockIdx.x * 64, tid = threadIdx.x, ch = tid & 7;
  in += (long)blockIdx.z * R * C;
  out += (long)blockIdx.z * R * C;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = (tid >> 3) + 32 * p;
    *reinterpret_cast<bf16x8*>(&tile[row][ch * 8]) = *reinterpret_cast<const bf16x8*>(in + (long)(tr + row) * C + tc + ch * 8);
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = (tid >> 3) + 32 * p;
    bf16x8 w;
#pragma unroll
    for (int j = 0; j < 8; ++j) w.v[j] = tile[ch * 8 + j][c];
    *reinterpret_cast<bf16x8*>(out + (long)(tc + c) * R + tr + ch * 8) = w;
  }
}
}  // namespace

// [R, C] -> [C, R], or batched [E, R, C] -> [E, C, R].
torch::Tensor transpose_bf16(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && (x.dim() == 2 || x.dim() == 3) && x.is_contiguous(),
              "transpose_bf16: 2-D or 3-D contiguous bf16 HIP tensor expected");
  const int E = x.dim() == 3 ? x.size(0) : 1, R = x.size(-2), C = x.size(-1);
  TORCH_CHECK(R % 64 == 0 && C % 64 == 0, "transpose_bf16: both dims must be multiples of 64");
  auto out = x.dim() == 3 ? torch::empty({E, C, R}, x.options()) : torch::empty({C, R}, x.options());
  if (x.numel() == 0) return out;
  static const bool use128 = [] { const char* e = std::getenv("ACCELERATE_TRANSPOSE128"); return !e || e[0] != '0'; }();
  if (use128 && R % 128 == 0 && C % 128 == 0)
    hipLaunchKernelGGL(transpose128_bf16_kernel, dim3(C / 128, R / 128, E), dim3(256), 0, at::hip::getCurrentHIPStream(),
                       reinterpret_cast<const bf16_t*>(x.data_ptr()), reinterpret_cast<bf16_t*>(out.data_ptr()), R, C);
  else
    hipLaunchKernelGGL(transpose_bf16_kernel, dim3(C / 64, R / 64, E), dim3(256), 0, at::hip::getCurrentHIPStream(),
                       reinterpret_cast<const bf16_t*>(x.data_ptr()), reinterpret_cast<bf16_t*>(out.data_ptr()), R, C);
  return out;
}
