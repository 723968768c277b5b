// Loss and optimizer kernels:
//   * cross-entropy over bf16 logits [T, V] (fwd: per-row loss + logsumexp; bwd: softmax - onehot written
//     IN PLACE over the logits so the 2 GB logits buffer of a Llama-3 step is reused as its gradient),
//   * multi-tensor fused Adam/AdamW (one launch per parameter group over a chunked tensor list; optional bf16
//     shadow write of the updated parameter for the FSDP all-gather),
//   * multi-tensor L2 norm (two-pass, deterministic) and device-side clip scaling (no host sync).
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"
#include <cstdlib>
#include <type_traits>

using namespace acc;

namespace {

constexpr int kXentThreads = 512;

__global__ __launch_bounds__(kXentThreads) void xent_fwd_kernel(const bf16_t* __restrict__ logits,
                                                                 const int64_t* __restrict__ labels,
                                                                 float* __restrict__ loss, float* __restrict__ lse_out,
                                                                 long V, int ignore_index) {
  __shared__ float scratch[16];
  const long row = blockIdx.x;
  const bf16_t* x = logits + row * V;
  const long nvec = V >> 3;
  float m = -INFINITY, s = 0.f;
  for (long c = threadIdx.x; c < nvec; c += kXentThreads) {
    const bf16x8 a = reinterpret_cast<const bf16x8*>(x)[c];
    float f[8];
    float lm = m;
#pragma unroll
    for (int j = 0; j < 8; ++j) { f[j] = bf2f(a.v[j]); lm = fmaxf(lm, f[j]); }
    s *= __expf(m - lm);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(f[j] - lm);
    m = lm;
  }
  for (long i = nvec * 8 + threadIdx.x; i < V; i += kXentThreads) {  // tail (V % 8)
    const float f = bf2f(x[i]);
    const float lm = fmaxf(m, f);
    s = s * __expf(m - lm) + __expf(f - lm);
    m = lm;
  }
  const float gm = block_max(m, scratch);
  float sa = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  sa = block_sum(sa, scratch);
  if (threadIdx.x == 0) {
    const float lse = gm + __logf(sa);
    lse_out[row] = lse;
    const int64_t lab = labels[row];
    ACC_CHECK(lab == ignore_index || (lab >= 0 && lab < V), kChkXentLabel);  // debug build: label outside the vocab
    const bool skip = lab == ignore_index || (ACC_DEBUG_BUILD && (lab < 0 || lab >= V));
    loss[row] = skip ? 0.f : (lse - bf2f(x[lab]));
  }
}

// grad = (softmax - onehot) * scale[0] for valid rows, 0 for ignored rows. May alias logits.
__global__ __launch_bounds__(kXentThreads) void xent_bwd_kernel(const bf16_t* logits, const int64_t* __restrict__ labels,
                                                                 const float* __restrict__ lse, const float* __restrict__ scale,
                                                                 bf16_t* grad, long V, int ignore_index) {
  const long row = blockIdx.x;
  const bf16_t* x = logits + row * V;
  bf16_t* g = grad + row * V;
  const int64_t lab = labels[row];
  const float sc = (lab == ignore_index) ? 0.f : scale[0];
  const float l = lse[row];
  const long nvec = V >> 3;
  for (long c = threadIdx.x; c < nvec; c += kXentThreads) {
    const bf16x8 a = reinterpret_cast<const bf16x8*>(x)[c];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(bf2f(a.v[j]) - l);
      if (c * 8 + j == lab) p -= 1.f;
      o.v[j] = f2bf(p * sc);
    }
    reinterpret_cast<bf16x8*>(g)[c] = o;
  }
  for (long i = nvec * 8 + threadIdx.x; i < V; i += kXentThreads) {
    float p = __expf(bf2f(x[i]) - l);
    if (i == lab) p -= 1.f;
    g[i] = f2bf(p * sc);
  }
}

// ------------------------------------------------------------------------------------------------
// Multi-tensor apply
// ------------------------------------------------------------------------------------------------
// amax (Adam only, optional): an fp32 slot receiving max |bf16(updated p)| over the tensor by atomicMax on its bits (the
// caller zeroes it first). The FSDP engine points it at a weight's fp8 all-gather amax, so the per-step re-quantisation
// needs no second read of the bf16 shards (parallel/fsdp.py refresh_fp8).
struct TensorMeta {
  int64_t p, g, m, v, shadow, n, amax;
};

constexpr int kMTThreads = 256;
constexpr int kChunk = 8192;  // elements per workgroup (32 per lane)

__device__ __forceinline__ int find_tensor(const int64_t* __restrict__ block_prefix, int ntensors, int64_t b) {
  int lo = 0, hi = ntensors - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (block_prefix[mid] <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

template <typename T> struct Vec4;
template <> struct Vec4<float> {
  static __device__ __forceinline__ void load(const float* p, float (&o)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&o)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  }
  static constexpr int kAlign = 16;
};
template <> struct Vec4<bf16_t> {
  static __device__ __forceinline__ void load(const bf16_t* p, float (&o)[4]) {
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = bf2f(v.v[j]);
  }
  static __device__ __forceinline__ void store(bf16_t* p, const float (&o)[4]) {
    bf16x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v.v[j] = f2bf(o[j]);
    *reinterpret_cast<bf16x4*>(p) = v;
  }
  static constexpr int kAlign = 8;
};

// Global-address-space (MODE 1) and global non-temporal (MODE 2) forms of Vec4 for the optimizer, which streams every
// state tensor exactly once per step (ACCELERATE_ADAM_NT=1 / 2 (default); 0 = Vec4's generic-pointer flat accesses).
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef unsigned int nt_u2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) nt_f4 g_f4;
typedef __attribute__((address_space(1))) nt_u2 g_u2;
template <int MODE, typename T>
__device__ __forceinline__ void ld4(const T* p, float (&o)[4]) {
  if constexpr (MODE == 0) {
    Vec4<T>::load(p, o);
  } else if constexpr (std::is_same<T, float>::value) {
    const g_f4* q = (const g_f4*)p;
    const nt_f4 v = MODE == 2 ? __builtin_nontemporal_load(q) : *q;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    const g_u2* q = (const g_u2*)p;
    const nt_u2 v = MODE == 2 ? __builtin_nontemporal_load(q) : *q;
    o[0] = bf2f((bf16_t)(v.x & 0xffffu)); o[1] = bf2f((bf16_t)(v.x >> 16));
    o[2] = bf2f((bf16_t)(v.y & 0xffffu)); o[3] = bf2f((bf16_t)(v.y >> 16));
  }
}
template <int MODE, typename T>
__device__ __forceinline__ void st4(T* p, const float (&o)[4]) {
  if constexpr (MODE == 0) {
    Vec4<T>::store(p, o);
  } else if constexpr (std::is_same<T, float>::value) {
    const nt_f4 v = {o[0], o[1], o[2], o[3]};
    if constexpr (MODE == 2) __builtin_nontemporal_store(v, (g_f4*)p);
    else *(g_f4*)p = v;
  } else {
    nt_u2 v;
    v.x = (unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16);
    v.y = (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16);
    if constexpr (MODE == 2) __builtin_nontemporal_store(v, (g_u2*)p);
    else *(g_u2*)p = v;
  }
}

struct AdamHyper {
  float lr, beta1, beta2, eps, wd, bc1, bc2_sqrt;
  int adamw;
};

__device__ __forceinline__ void adam_elem(float& pf, float gf, float& mf, float& vf, const AdamHyper& h) {
  if (!h.adamw) gf += h.wd * pf;
  mf = h.beta1 * mf + (1.f - h.beta1) * gf;
  vf = h.beta2 * vf + (1.f - h.beta2) * gf * gf;
  if (h.adamw) pf *= 1.f - h.lr * h.wd;
  pf -= (h.lr / h.bc1) * mf / (sqrtf(vf) / h.bc2_sqrt + h.eps);
}

// Each lane owns 4 consecutive elements per iteration; 16-B (fp32) / 8-B (bf16) vector accesses when every
// operand of the tensor is aligned (chunk starts are multiples of kChunk elements, so the base decides).
template <typename P, typename G, typename S, int NT = 0>
__global__ __launch_bounds__(kMTThreads) void adam_mt_kernel(const TensorMeta* __restrict__ meta,
                                                             const int64_t* __restrict__ block_prefix, int ntensors,
                                                             AdamHyper h, const float* __restrict__ grad_scale) {
  const int t = find_tensor(block_prefix, ntensors, blockIdx.x);
  // debug build: the block maps to a listed tensor and a chunk inside it (block-uniform)
  ACC_CHECK_OR_RETURN(t >= 0 && t < ntensors && (int64_t)(blockIdx.x - block_prefix[t]) * kChunk < meta[t].n, kChkMtChunk);
  const TensorMeta tm = meta[t];
  const int64_t start = (int64_t)(blockIdx.x - block_prefix[t]) * kChunk;
  const int64_t end = min(start + (int64_t)kChunk, tm.n);
  P* p = reinterpret_cast<P*>(tm.p);
  const G* g = reinterpret_cast<const G*>(tm.g);
  S* m = reinterpret_cast<S*>(tm.m);
  S* v = reinterpret_cast<S*>(tm.v);
  bf16_t* sh = reinterpret_cast<bf16_t*>(tm.shadow);
  unsigned int* amax = reinterpret_cast<unsigned int*>(tm.amax);  // block-uniform
  float am = 0.f;
  const float gs = grad_scale != nullptr ? grad_scale[0] : 1.f;
  const bool aligned = (tm.p % Vec4<P>::kAlign == 0) && (tm.g % Vec4<G>::kAlign == 0) &&
                       (tm.m % Vec4<S>::kAlign == 0) && (tm.v % Vec4<S>::kAlign == 0) && (tm.shadow % 8 == 0);
  if (aligned) {
    const int64_t vend = start + ((end - start) & ~int64_t(3));
    for (int64_t i = start + (int64_t)threadIdx.x * 4; i < vend; i += (int64_t)kMTThreads * 4) {
      float pf[4], gf[4], mf[4], vf[4];
      ld4<NT>(p + i, pf);
      ld4<NT>(g + i, gf);
      ld4<NT>(m + i, mf);
      ld4<NT>(v + i, vf);
#pragma unroll
      for (int j = 0; j < 4; ++j) adam_elem(pf[j], gf[j] * gs, mf[j], vf[j], h);
      st4<NT>(p + i, pf);
      st4<NT>(m + i, mf);
      st4<NT>(v + i, vf);
      if (sh != nullptr) st4<NT == 2 ? 1 : NT>(sh + i, pf);  // the shadow is read again soon (all-gather / forward)
      if (amax != nullptr) {
#pragma unroll
        for (int j = 0; j < 4; ++j) am = fmaxf(am, fabsf(bf2f(f2bf(pf[j]))));
      }
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += kMTThreads) {
      float pf = to_f<P>(p[i]), mf = to_f<S>(m[i]), vf = to_f<S>(v[i]);
      adam_elem(pf, to_f<G>(g[i]) * gs, mf, vf, h);
      p[i] = from_f<P>(pf); m[i] = from_f<S>(mf); v[i] = from_f<S>(vf);
      if (sh != nullptr) sh[i] = f2bf(pf);
      if (amax != nullptr) am = fmaxf(am, fabsf(bf2f(f2bf(pf))));
    }
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += kMTThreads) {
      float pf = to_f<P>(p[i]), mf = to_f<S>(m[i]), vf = to_f<S>(v[i]);
      adam_elem(pf, to_f<G>(g[i]) * gs, mf, vf, h);
      p[i] = from_f<P>(pf); m[i] = from_f<S>(mf); v[i] = from_f<S>(vf);
      if (sh != nullptr) sh[i] = f2bf(pf);
      if (amax != nullptr) am = fmaxf(am, fabsf(bf2f(f2bf(pf))));
    }
  }
  if (amax != nullptr) {  // block-uniform: every thread reaches the barriers
    __shared__ float scratch[16];
    am = block_max(am, scratch);
    if (threadIdx.x == 0) atomicMax(amax, __float_as_uint(am));  // non-negative floats order like their bits
  }
}

template <typename G>
__global__ __launch_bounds__(kMTThreads) void sqnorm_mt_kernel(const TensorMeta* __restrict__ meta,
                                                               const int64_t* __restrict__ block_prefix, int ntensors,
                                                               float* __restrict__ partial) {
  __shared__ float scratch[16];
  const int t = find_tensor(block_prefix, ntensors, blockIdx.x);
  const TensorMeta tm = meta[t];
  const int64_t start = (int64_t)(blockIdx.x - block_prefix[t]) * kChunk;
  const int64_t end = min(start + (int64_t)kChunk, tm.n);
  const G* g = reinterpret_cast<const G*>(tm.g);
  float acc = 0.f;
  for (int64_t i = start + threadIdx.x; i < end; i += kMTThreads) {
    const float f = to_f<G>(g[i]);
    acc += f * f;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

__global__ void sum_partials_kernel(const float* __restrict__ partial, int n, float* __restrict__ out, int accumulate) {
  __shared__ float scratch[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partial[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + acc : acc;
}

// g *= min(1, max_norm / (sqrt(total_sq) + 1e-6)), all on device.
template <typename G>
__global__ __launch_bounds__(kMTThreads) void clip_mt_kernel(const TensorMeta* __restrict__ meta,
                                                             const int64_t* __restrict__ block_prefix, int ntensors,
                                                             const float* __restrict__ total_sq, float max_norm) {
  const int t = find_tensor(block_prefix, ntensors, blockIdx.x);
  const TensorMeta tm = meta[t];
  const int64_t start = (int64_t)(blockIdx.x - block_prefix[t]) * kChunk;
  const int64_t end = min(start + (int64_t)kChunk, tm.n);
  const float norm = sqrtf(total_sq[0]);
  const float coef = fminf(1.f, max_norm / (norm + 1e-6f));
  if (coef >= 1.f) return;
  G* g = reinterpret_cast<G*>(tm.g);
  for (int64_t i = start + threadIdx.x; i < end; i += kMTThreads) g[i] = from_f<G>(to_f<G>(g[i]) * coef);
}

// AMP unscale + overflow check (torch GradScaler's `_amp_foreach_non_finite_check_and_unscale_`): g *= inv_scale in
// place; any non-finite result sets found_inf[0] = 1. The flag is written with a plain store by every workgroup that
// saw one (all write the same value), so no atomics and no extra pass.
template <typename G>
__global__ __launch_bounds__(kMTThreads) void unscale_mt_kernel(const TensorMeta* __restrict__ meta,
                                                                const int64_t* __restrict__ block_prefix, int ntensors,
                                                                const float* __restrict__ inv_scale, float* __restrict__ found_inf) {
  const int t = find_tensor(block_prefix, ntensors, blockIdx.x);
  const TensorMeta tm = meta[t];
  const int64_t start = (int64_t)(blockIdx.x - block_prefix[t]) * kChunk;
  const int64_t end = min(start + (int64_t)kChunk, tm.n);
  const float inv = inv_scale[0];
  G* g = reinterpret_cast<G*>(tm.g);
  bool bad = false;
  for (int64_t i = start + threadIdx.x; i < end; i += kMTThreads) {
    const float v = to_f<G>(g[i]) * inv;
    bad |= !isfinite(v);
    g[i] = from_f<G>(v);
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) found_inf[0] = 1.f;
}

}  // namespace

ACC_DEBUG_TAKE_FN(acc_dbg_take_xent_optim)

#ifdef ACC_DEBUG_BOUNDS
namespace {
// Self-test of the check mechanism itself: every lane past `n` reports a failed bounds check instead of writing.
__global__ void acc_dbg_selftest_kernel(float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  ACC_CHECK_OR_RETURN(i < n, kChkSelfTest);
  out[i] = 1.f;
}
}  // namespace
#endif

// debug build: launch a kernel whose grid overshoots `out` by `overshoot` elements (the check must catch it and no
// write may land past the end); release build: a no-op returning false.
bool debug_selftest(torch::Tensor out, int64_t overshoot) {
#ifdef ACC_DEBUG_BOUNDS
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous(), "debug_selftest: fp32 HIP tensor");
  const int n = (int)out.numel(), total = n + (int)overshoot;
  hipLaunchKernelGGL(acc_dbg_selftest_kernel, dim3((total + 255) / 256), dim3(256), 0, at::hip::getCurrentHIPStream(),
                     out.data_ptr<float>(), n);
  return true;
#else
  (void)out;
  (void)overshoot;
  return false;
#endif
}

// ----------------------------------------------------------------------------------------- host API
std::vector<torch::Tensor> xent_fwd(torch::Tensor logits, torch::Tensor labels, int64_t ignore_index) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kBFloat16 && logits.is_contiguous(), "xent: logits must be contiguous bf16 on GPU");
  TORCH_CHECK(labels.scalar_type() == at::kLong, "xent: labels must be int64");
  const long V = logits.size(-1);
  const long T = logits.numel() / V;
  TORCH_CHECK(labels.numel() == T, "xent: labels must have one entry per logits row");
  auto loss = torch::empty({T}, logits.options().dtype(torch::kFloat32));
  auto lse = torch::empty({T}, logits.options().dtype(torch::kFloat32));
  if (T == 0) return {loss, lse};
  hipLaunchKernelGGL(xent_fwd_kernel, dim3(T), dim3(kXentThreads), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16_t*>(logits.data_ptr()), labels.contiguous().data_ptr<int64_t>(),
                     loss.data_ptr<float>(), lse.data_ptr<float>(), V, (int)ignore_index);
  return {loss, lse};
}

// Writes the gradient into `out` (may be `logits` itself for an in-place backward).
void xent_bwd(torch::Tensor logits, torch::Tensor labels, torch::Tensor lse, torch::Tensor scale, torch::Tensor out,
              int64_t ignore_index) {
  const long V = logits.size(-1);
  const long T = logits.numel() / V;
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == at::kBFloat16 && out.numel() == logits.numel(), "xent_bwd: bad out");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.is_cuda(), "xent_bwd: scale must be a fp32 device scalar");
  if (T == 0) return;
  hipLaunchKernelGGL(xent_bwd_kernel, dim3(T), dim3(kXentThreads), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16_t*>(logits.data_ptr()), labels.contiguous().data_ptr<int64_t>(),
                     lse.data_ptr<float>(), scale.data_ptr<float>(), reinterpret_cast<bf16_t*>(out.data_ptr()), V,
                     (int)ignore_index);
}

// `meta` is an int64 device tensor [ntensors, 6] (p, g, m, v, shadow, n); `block_prefix` int64 [ntensors + 1].
// dtype codes: 0 = fp32, 1 = bf16.
void adam_multi_tensor(torch::Tensor meta, torch::Tensor block_prefix, int64_t nblocks, int64_t pdtype, int64_t gdtype,
                       int64_t sdtype, double lr, double beta1, double beta2, double eps, double wd, double bc1,
                       double bc2_sqrt, bool adamw, c10::optional<torch::Tensor> grad_scale) {
  TORCH_CHECK(meta.dim() == 2 && meta.size(1) == sizeof(TensorMeta) / 8, "multi_tensor: meta must be [n, 7] int64");
  const int nt = meta.size(0);
  if (nt == 0 || nblocks == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const TensorMeta* mp = reinterpret_cast<const TensorMeta*>(meta.data_ptr<int64_t>());
  const int64_t* bp = block_prefix.data_ptr<int64_t>();
  const float* gsp = grad_scale.has_value() ? grad_scale->data_ptr<float>() : nullptr;
  AdamHyper hyper{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (float)bc1, (float)bc2_sqrt, (int)adamw};
  // default 2 (global non-temporal): tools/bench_adam.py at Llama-3-8B scale, 26.6 ms vs 26.9-27.7 (flat) and 27.4-27.6
  // (global, temporal) per step, two interleaved rounds on one box
  static const int adam_nt = [] { const char* e = std::getenv("ACCELERATE_ADAM_NT"); return e != nullptr ? std::atoi(e) : 2; }();
#define ADAM_LAUNCH(P, G, S)                                                                                            \
  if (adam_nt == 2) hipLaunchKernelGGL((adam_mt_kernel<P, G, S, 2>), dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, hyper, gsp); \
  else if (adam_nt == 1) hipLaunchKernelGGL((adam_mt_kernel<P, G, S, 1>), dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, hyper, gsp); \
  else hipLaunchKernelGGL((adam_mt_kernel<P, G, S>), dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, hyper, gsp)
  if (pdtype == 0 && gdtype == 0 && sdtype == 0) { ADAM_LAUNCH(float, float, float); }
  else if (pdtype == 0 && gdtype == 1 && sdtype == 0) { ADAM_LAUNCH(float, bf16_t, float); }
  else if (pdtype == 1 && gdtype == 1 && sdtype == 1) { ADAM_LAUNCH(bf16_t, bf16_t, bf16_t); }
  else if (pdtype == 1 && gdtype == 1 && sdtype == 0) { ADAM_LAUNCH(bf16_t, bf16_t, float); }
  else if (pdtype == 0 && gdtype == 0 && sdtype == 1) { ADAM_LAUNCH(float, float, bf16_t); }  // fp32 master, bf16 m / v
  else if (pdtype == 0 && gdtype == 1 && sdtype == 1) { ADAM_LAUNCH(float, bf16_t, bf16_t); }
  else TORCH_CHECK(false, "adam_multi_tensor: unsupported dtype combination");
#undef ADAM_LAUNCH
}

int64_t multi_tensor_chunk() { return kChunk; }

// Accumulates the squared L2 norm of the listed grads into out[0] (out is fp32 [1], zeroed by caller
// or accumulated when `accumulate`).
void sqnorm_multi_tensor(torch::Tensor meta, torch::Tensor block_prefix, int64_t nblocks, int64_t gdtype, torch::Tensor out,
                         bool accumulate) {
  TORCH_CHECK(meta.dim() == 2 && meta.size(1) == sizeof(TensorMeta) / 8, "multi_tensor: meta must be [n, 7] int64");
  const int nt = meta.size(0);
  auto stream = at::hip::getCurrentHIPStream();
  if (nt == 0 || nblocks == 0) {
    if (!accumulate) out.zero_();
    return;
  }
  auto partial = torch::empty({nblocks}, out.options());
  const TensorMeta* mp = reinterpret_cast<const TensorMeta*>(meta.data_ptr<int64_t>());
  const int64_t* bp = block_prefix.data_ptr<int64_t>();
  if (gdtype == 0)
    hipLaunchKernelGGL(sqnorm_mt_kernel<float>, dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, partial.data_ptr<float>());
  else
    hipLaunchKernelGGL(sqnorm_mt_kernel<bf16_t>, dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, partial.data_ptr<float>());
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(1024), 0, stream, partial.data_ptr<float>(), (int)nblocks,
                     out.data_ptr<float>(), (int)accumulate);
}

void clip_multi_tensor(torch::Tensor meta, torch::Tensor block_prefix, int64_t nblocks, int64_t gdtype, torch::Tensor total_sq,
                       double max_norm) {
  TORCH_CHECK(meta.dim() == 2 && meta.size(1) == sizeof(TensorMeta) / 8, "multi_tensor: meta must be [n, 7] int64");
  const int nt = meta.size(0);
  if (nt == 0 || nblocks == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const TensorMeta* mp = reinterpret_cast<const TensorMeta*>(meta.data_ptr<int64_t>());
  const int64_t* bp = block_prefix.data_ptr<int64_t>();
  if (gdtype == 0)
    hipLaunchKernelGGL(clip_mt_kernel<float>, dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, total_sq.data_ptr<float>(), (float)max_norm);
  else
    hipLaunchKernelGGL(clip_mt_kernel<bf16_t>, dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, total_sq.data_ptr<float>(), (float)max_norm);
}

// grads *= inv_scale[0]; found_inf[0] = 1 if any result is inf / NaN (found_inf is NOT cleared here: torch semantics).
void unscale_multi_tensor(torch::Tensor meta, torch::Tensor block_prefix, int64_t nblocks, int64_t gdtype, torch::Tensor inv_scale,
                          torch::Tensor found_inf) {
  TORCH_CHECK(meta.dim() == 2 && meta.size(1) == sizeof(TensorMeta) / 8, "multi_tensor: meta must be [n, 7] int64");
  const int nt = meta.size(0);
  if (nt == 0 || nblocks == 0) return;
  TORCH_CHECK(inv_scale.scalar_type() == at::kFloat && found_inf.scalar_type() == at::kFloat, "unscale: fp32 scale / flag");
  auto stream = at::hip::getCurrentHIPStream();
  const TensorMeta* mp = reinterpret_cast<const TensorMeta*>(meta.data_ptr<int64_t>());
  const int64_t* bp = block_prefix.data_ptr<int64_t>();
  if (gdtype == 0)
    hipLaunchKernelGGL(unscale_mt_kernel<float>, dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, inv_scale.data_ptr<float>(),
                       found_inf.data_ptr<float>());
  else
    hipLaunchKernelGGL(unscale_mt_kernel<bf16_t>, dim3(nblocks), dim3(kMTThreads), 0, stream, mp, bp, nt, inv_scale.data_ptr<float>(),
                       found_inf.data_ptr<float>());
}
