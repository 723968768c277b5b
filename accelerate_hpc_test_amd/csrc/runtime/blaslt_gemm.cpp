// Weight-gradient GEMM with an fp32 destination, straight on hipBLASLt with per-shape algorithm search.
//
//   out[N, K] (+)= dy[T, N]^T . x[T, K]        dy, x: row-major bf16; out: row-major fp32 (the FSDP fp32 grad shard)
//
// Why: at FSDP world size 1 the weight gradients are written in fp32 directly into the grad shard (no bf16 buffer and
// no bf16 -> fp32 pass). torch's `mm(..., out_dtype=float32)` reaches hipBLASLt through its default heuristic only
// (TunableOp does not cover mixed-precision outputs) and lands on a depth-32 tile for these NT shapes. Here the first
// call of each (T, N, K) asks hipBLASLt for its candidate algorithms, times them on a scratch output, and caches the
// fastest; every later call is one hipblasLtMatmul on the current HIP stream. Column-major view used for the call:
//   D (K x N, ld K) = X (K x T, ld K, op N) . DY^T (DY: N x T, ld N, op T), beta = accumulate ? 1 : 0.
// With `x_t` the layer input arrives as its token-contiguous copy xT [K, T] (the FSDP / DDP engines keep that copy
// for this GEMM): X is then the column-major T x K matrix (ld T) taken with op T.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

constexpr size_t kWorkspace = size_t(64) << 20;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  bool ok = false;
  float ms = 0.f;
  int candidates = 0;
  int64_t T = 0;  // the token count the layouts (and the timed search) were built for
};

// power-of-two buckets from 256: problems within a factor of two share one timed search (variable-length batches would
// otherwise search — and synchronise inside backward — once per distinct token count, and grow the cache without bound)
int64_t dim_bucket(int64_t x) {
  int64_t b = 256;
  while (b < x) b <<= 1;
  return b;
}

struct State {
  hipblasLtHandle_t handle = nullptr;
  torch::Tensor workspace;  // of the first stream that called
  // one workspace per HIP stream: GEMMs enqueued on different streams (MoE experts spread over side streams) run
  // concurrently, and a shared workspace would be written by both
  std::map<hipStream_t, torch::Tensor> stream_ws;
  std::map<std::tuple<int64_t, int64_t, int64_t, int, int>, Plan> plans;  // (T bucket, N, K, device, x_t | dy_t << 1)
  std::mutex mu;
};

State& state() {
  static State s;
  return s;
}

bool check(hipblasStatus_t st) { return st == HIPBLAS_STATUS_SUCCESS; }

// How many of hipBLASLt's heuristic candidates a searched plan times (ACCELERATE_BLASLT_CANDIDATES, default 32): the
// search runs once per problem (bucket), at its first call.
int search_width() {
  static const int n = [] {
    const char* e = std::getenv("ACCELERATE_BLASLT_CANDIDATES");
    const int v = e ? std::atoi(e) : 32;
    return v < 1 ? 1 : (v > 512 ? 512 : v);
  }();
  return n;
}

// Workspace of `stream` (call with s.mu held).
void* workspace_for(State& s, hipStream_t stream, const torch::Tensor& like) {
  auto it = s.stream_ws.find(stream);
  if (it == s.stream_ws.end()) {
    torch::Tensor ws = s.stream_ws.empty() && s.workspace.defined()
                           ? s.workspace
                           : torch::empty({(int64_t)kWorkspace}, like.options().dtype(torch::kUInt8));
    it = s.stream_ws.emplace(stream, ws).first;
  }
  return it->second.data_ptr();
}

// Time every usable heuristic candidate (`run_i(i)` launches candidate i on the scratch operands and returns false when
// hipBLASLt rejects it): one warm-up and `reps` back-to-back runs each, then the 4 fastest again with 4 x `reps` runs,
// so that one lucky measurement does not pick the plan (with three runs per candidate a wider search mostly found the
// luckiest timing, profiles/r4_llama8b_step.md). Returns the winner's index (-1 if none ran) and its ms per run.
template <class RunI>
int search_best(const std::vector<hipblasLtMatmulHeuristicResult_t>& res, int got, RunI run_i, hipStream_t stream,
                int reps, float& ms_out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time = [&](int i, int n) -> float {
    if (!run_i(i)) return -1.f;
    hipEventRecord(e0, stream);
    for (int r = 0; r < n; ++r) run_i(i);
    hipEventRecord(e1, stream);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / n;
  };
  std::vector<std::pair<float, int>> first;
  for (int i = 0; i < got; ++i) {
    if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > kWorkspace) continue;
    const float ms = time(i, reps);
    if (ms >= 0.f) first.emplace_back(ms, i);
  }
  std::sort(first.begin(), first.end());
  int best = -1;
  float best_ms = 1e30f;
  for (size_t k = 0; k < first.size() && k < 4; ++k) {
    const float ms = time(first[k].second, 4 * reps);
    if (ms >= 0.f && ms < best_ms) {
      best_ms = ms;
      best = first[k].second;
    }
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  ms_out = best_ms;
  return best;
}

// dy_t: dy arrives transposed ([N, T], token-contiguous), so both operands are contraction-contiguous (the TN class of
// the forward GEMMs) instead of dy being read across its rows.
bool build_plan(State& s, Plan& p, int64_t T, int64_t N, int64_t K, bool x_t, bool dy_t, hipStream_t stream,
                const torch::Tensor& like) {
  const hipblasOperation_t ta = x_t ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = dy_t ? HIPBLAS_OP_N : HIPBLAS_OP_T;
  if (!check(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F))) return false;
  if (!check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)))) return false;
  if (!check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)))) return false;
  if (!check(x_t ? hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, T, K, T)
                 : hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, T, K))) return false;
  if (!check(dy_t ? hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, T, N, T)
                  : hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, N, T, N))) return false;
  if (!check(hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_32F, K, N, K))) return false;
  hipblasLtMatmulPreference_t pref;
  if (!check(hipblasLtMatmulPreferenceCreate(&pref))) return false;
  uint64_t ws = kWorkspace;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(search_width());
  int got = 0;
  const bool okh = check(hipblasLtMatmulAlgoGetHeuristic(s.handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, (int)res.size(),
                                                         res.data(), &got));
  hipblasLtMatmulPreferenceDestroy(pref);
  if (!okh || got <= 0) return false;
  p.candidates = got;
  // time every candidate on scratch operands of the real shape (beta = 0, so nothing real is touched)
  auto a = torch::empty({T, K}, like.options().dtype(torch::kBFloat16)).normal_();
  auto b = torch::empty({T, N}, like.options().dtype(torch::kBFloat16)).normal_();
  auto d = torch::empty({N, K}, like.options().dtype(torch::kFloat32));
  const float one = 1.f, zero = 0.f;
  auto run_i = [&](int i) {
    return check(hipblasLtMatmul(s.handle, p.desc, &one, a.data_ptr(), p.la, b.data_ptr(), p.lb, &zero, d.data_ptr(), p.lc,
                             d.data_ptr(), p.lc, &res[i].algo, workspace_for(s, stream, like), kWorkspace, stream));
  };
  float best = 0.f;
  const int bi = search_best(res, got, run_i, stream, 3, best);
  if (bi >= 0) {
    p.algo = res[bi].algo;
    p.ok = true;
  }
  p.ms = best;
  p.T = T;
  return p.ok;
}

// Token count T of a bucket whose plan was searched on another T: per-call layouts (host objects), the bucket's algorithm
// when hipBLASLt supports it for this problem, else the heuristic's first choice — no timing, no synchronisation.
bool run_wgrad_other_t(State& s, Plan& plan, int64_t T, int64_t N, int64_t K, bool x_t, bool dy_t, const void* x,
                       const void* dy, void* out, float beta, void* ws, hipStream_t stream) {
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  bool ok = check(x_t ? hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, T, K, T) : hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, T, K)) &&
            check(dy_t ? hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, T, N, T) : hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, N, T, N)) &&
            check(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, K, N, K));
  const float one = 1.f;
  hipblasLtMatmulAlgo_t algo = plan.algo;
  if (ok) {
    size_t wsz = 0;
    if (hipblaslt_ext::matmulIsAlgoSupported(s.handle, plan.desc, (void*)&one, la, lb, (void*)&beta, lc, lc, algo, wsz) !=
            HIPBLAS_STATUS_SUCCESS || wsz > kWorkspace) {
      hipblasLtMatmulPreference_t pref;
      ok = check(hipblasLtMatmulPreferenceCreate(&pref));
      if (ok) {
        uint64_t wsl = kWorkspace;
        hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsl, sizeof(wsl));
        hipblasLtMatmulHeuristicResult_t r;
        int got = 0;
        ok = check(hipblasLtMatmulAlgoGetHeuristic(s.handle, plan.desc, la, lb, lc, lc, pref, 1, &r, &got)) && got > 0 &&
             r.state == HIPBLAS_STATUS_SUCCESS;
        if (ok) algo = r.algo;
        hipblasLtMatmulPreferenceDestroy(pref);
      }
    }
  }
  if (ok)
    ok = check(hipblasLtMatmul(s.handle, plan.desc, &one, x, la, dy, lb, &beta, out, lc, out, lc, &algo, ws, kWorkspace, stream));
  if (la) hipblasLtMatrixLayoutDestroy(la);
  if (lb) hipblasLtMatrixLayoutDestroy(lb);
  if (lc) hipblasLtMatrixLayoutDestroy(lc);
  return ok;
}

}  // namespace

// Returns false (and does nothing) when hipBLASLt offers no working algorithm: the caller falls back to torch.
bool blaslt_wgrad_f32(torch::Tensor dy, torch::Tensor x, torch::Tensor out, bool accumulate, bool x_t, bool dy_t) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && out.is_cuda(), "blaslt_wgrad_f32: HIP tensors expected");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kFloat,
              "blaslt_wgrad_f32: bf16 operands and an fp32 output expected");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && out.dim() == 2 && dy.is_contiguous() && x.is_contiguous() && out.is_contiguous(),
              "blaslt_wgrad_f32: 2-D contiguous tensors expected");
  const int64_t T = dy_t ? dy.size(1) : dy.size(0), N = dy_t ? dy.size(0) : dy.size(1), K = x_t ? x.size(0) : x.size(1);
  TORCH_CHECK((x_t ? x.size(1) : x.size(0)) == T && out.size(0) == N && out.size(1) == K, "blaslt_wgrad_f32: shape mismatch");
  State& s = state();
  hipStream_t stream = at::hip::getCurrentHIPStream();
  Plan* plan = nullptr;
  void* ws = nullptr;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.handle == nullptr) {
      if (!check(hipblasLtCreate(&s.handle))) return false;
      s.workspace = torch::empty({(int64_t)kWorkspace}, out.options().dtype(torch::kUInt8));
    }
    const int dev = out.get_device();
    auto key = std::make_tuple(dim_bucket(T), N, K, dev, (int)x_t | ((int)dy_t << 1));
    auto it = s.plans.find(key);
    if (it == s.plans.end()) {
      Plan p;
      build_plan(s, p, T, N, K, x_t, dy_t, stream, out);
      it = s.plans.emplace(key, p).first;
    }
    plan = &it->second;
    ws = workspace_for(s, stream, out);
    if (plan->ok && plan->T != T)
      return run_wgrad_other_t(s, *plan, T, N, K, x_t, dy_t, x.data_ptr(), dy.data_ptr(), out.data_ptr(), accumulate ? 1.f : 0.f,
                               ws, stream);
  }
  if (!plan->ok) return false;
  const float one = 1.f, beta = accumulate ? 1.f : 0.f;
  return check(hipblasLtMatmul(s.handle, plan->desc, &one, x.data_ptr(), plan->la, dy.data_ptr(), plan->lb, &beta,
                               out.data_ptr(), plan->lc, out.data_ptr(), plan->lc, &plan->algo, ws, kWorkspace, stream));
}

// ------------------------------------------------------------------------------------------------ bf16 dgrad, NN layout
// dx[T, K] = dy[T, N] . W[N, K] with both operands row-major as the autograd graph holds them (no transposed weight
// copy). Column-major view: D (K x T, ld K) = A (W: K x N, ld K, op N) . B (dy: N x T, ld N, op N). torch's matmul
// reaches hipBLASLt's first heuristic choice for this NN class only; here the candidates are timed once per
// (power-of-two T bucket, N, K) as for the weight gradient above, and other token counts of a bucket reuse the winner
// (or the heuristic's first choice where it does not apply) without a search.
namespace {

struct DgState {
  std::map<std::tuple<int64_t, int64_t, int64_t, int>, Plan> plans;
};

DgState& dgstate() {
  static DgState s;
  return s;
}

bool dg_layouts(int64_t T, int64_t N, int64_t K, hipblasLtMatrixLayout_t* la, hipblasLtMatrixLayout_t* lb,
                hipblasLtMatrixLayout_t* lc) {
  return check(hipblasLtMatrixLayoutCreate(la, HIP_R_16BF, K, N, K)) && check(hipblasLtMatrixLayoutCreate(lb, HIP_R_16BF, N, T, N)) &&
         check(hipblasLtMatrixLayoutCreate(lc, HIP_R_16BF, K, T, K));
}

bool build_dg_plan(State& s, Plan& p, int64_t T, int64_t N, int64_t K, hipStream_t stream, const torch::Tensor& like) {
  const hipblasOperation_t op = HIPBLAS_OP_N;
  if (!check(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F))) return false;
  if (!check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &op, sizeof(op)))) return false;
  if (!check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &op, sizeof(op)))) return false;
  if (!dg_layouts(T, N, K, &p.la, &p.lb, &p.lc)) return false;
  hipblasLtMatmulPreference_t pref;
  if (!check(hipblasLtMatmulPreferenceCreate(&pref))) return false;
  uint64_t ws = kWorkspace;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(search_width());
  int got = 0;
  const bool okh = check(hipblasLtMatmulAlgoGetHeuristic(s.handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, (int)res.size(),
                                                         res.data(), &got));
  hipblasLtMatmulPreferenceDestroy(pref);
  if (!okh || got <= 0) return false;
  p.candidates = got;
  auto w = torch::empty({N, K}, like.options().dtype(torch::kBFloat16)).normal_();
  auto dy = torch::empty({T, N}, like.options().dtype(torch::kBFloat16)).normal_();
  auto d = torch::empty({T, K}, like.options().dtype(torch::kBFloat16));
  const float one = 1.f, zero = 0.f;
  auto run_i = [&](int i) {
    return check(hipblasLtMatmul(s.handle, p.desc, &one, w.data_ptr(), p.la, dy.data_ptr(), p.lb, &zero, d.data_ptr(), p.lc,
                             d.data_ptr(), p.lc, &res[i].algo, workspace_for(s, stream, like), kWorkspace, stream));
  };
  float best = 0.f;
  const int bi = search_best(res, got, run_i, stream, 3, best);
  if (bi >= 0) {
    p.algo = res[bi].algo;
    p.ok = true;
  }
  p.ms = best;
  p.T = T;
  return p.ok;
}

}  // namespace

// Returns false (nothing launched) when hipBLASLt offers no algorithm: the caller falls back to torch.
bool blaslt_dgrad_bf16(torch::Tensor dy, torch::Tensor w, torch::Tensor out) {
  TORCH_CHECK(dy.is_cuda() && w.is_cuda() && out.is_cuda() && dy.scalar_type() == at::kBFloat16 &&
                  w.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
              "blaslt_dgrad_bf16: bf16 HIP tensors expected");
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 2 && out.dim() == 2 && dy.is_contiguous() && w.is_contiguous() && out.is_contiguous(),
              "blaslt_dgrad_bf16: 2-D contiguous tensors expected");
  const int64_t T = dy.size(0), N = dy.size(1), K = w.size(1);
  TORCH_CHECK(w.size(0) == N && out.size(0) == T && out.size(1) == K, "blaslt_dgrad_bf16: shape mismatch");
  State& s = state();
  hipStream_t stream = at::hip::getCurrentHIPStream();
  std::lock_guard<std::mutex> lk(s.mu);
  if (s.handle == nullptr) {
    if (!check(hipblasLtCreate(&s.handle))) return false;
    s.workspace = torch::empty({(int64_t)kWorkspace}, out.options().dtype(torch::kUInt8));
  }
  auto key = std::make_tuple(dim_bucket(T), N, K, (int)out.get_device());
  auto& plans = dgstate().plans;
  auto it = plans.find(key);
  if (it == plans.end()) {
    Plan p;
    build_dg_plan(s, p, T, N, K, stream, out);
    it = plans.emplace(key, p).first;
  }
  Plan& plan = it->second;
  if (!plan.ok) return false;
  void* ws = workspace_for(s, stream, out);
  const float one = 1.f, zero = 0.f;
  if (plan.T == T)
    return check(hipblasLtMatmul(s.handle, plan.desc, &one, w.data_ptr(), plan.la, dy.data_ptr(), plan.lb, &zero,
                                 out.data_ptr(), plan.lc, out.data_ptr(), plan.lc, &plan.algo, ws, kWorkspace, stream));
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  bool ok = dg_layouts(T, N, K, &la, &lb, &lc);
  hipblasLtMatmulAlgo_t algo = plan.algo;
  if (ok) {
    size_t wsz = 0;
    if (hipblaslt_ext::matmulIsAlgoSupported(s.handle, plan.desc, (void*)&one, la, lb, (void*)&zero, lc, lc, algo, wsz) !=
            HIPBLAS_STATUS_SUCCESS || wsz > kWorkspace) {
      hipblasLtMatmulPreference_t pref;
      ok = check(hipblasLtMatmulPreferenceCreate(&pref));
      if (ok) {
        uint64_t wsl = kWorkspace;
        hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsl, sizeof(wsl));
        hipblasLtMatmulHeuristicResult_t r;
        int got = 0;
        ok = check(hipblasLtMatmulAlgoGetHeuristic(s.handle, plan.desc, la, lb, lc, lc, pref, 1, &r, &got)) && got > 0 &&
             r.state == HIPBLAS_STATUS_SUCCESS;
        if (ok) algo = r.algo;
        hipblasLtMatmulPreferenceDestroy(pref);
      }
    }
  }
  if (ok)
    ok = check(hipblasLtMatmul(s.handle, plan.desc, &one, w.data_ptr(), la, dy.data_ptr(), lb, &zero, out.data_ptr(), lc,
                               out.data_ptr(), lc, &algo, ws, kWorkspace, stream));
  if (la) hipblasLtMatrixLayoutDestroy(la);
  if (lb) hipblasLtMatrixLayoutDestroy(lb);
  if (lc) hipblasLtMatrixLayoutDestroy(lc);
  return ok;
}

// ------------------------------------------------------------------------------------------------ fp8, per-tensor
// C[M, N] (=|+=) alpha * sa * sb * (A[M, K] . B[N, K]^T)   A, B: row-major (K-contiguous) e4m3 / e5m2; sa, sb: device
// fp32 [1] scale factors read by the kernel (Fp8Linear passes each operand's amax and folds 1 / (qmax_a * qmax_b)
// into alpha, so no scale arithmetic runs on the device); C: row-major bf16 or fp32, accumulated with beta = 1.
// This is the per-tensor-scaled fp8 GEMM the reference reaches through torchao -> torch._scaled_mm -> hipBLASLt;
// measured on MI355X it runs the Llama-3-8B linear shapes at 2.7-3.4 PF/s (profiles/r3_gemm_fp8_library.md), so the
// per-tensor path uses it. Column-major view: D (N x M, ld N) = op_T(B: K x N, ld K) . op_N(A: K x M, ld K) — the TN
// form hipBLASLt's fp8 kernels are built for. Per (M, N, K, dtypes, output) the candidates are timed once.
namespace {

struct F8Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  bool ok = false;
  float ms = 0.f;
  int candidates = 0;
  int64_t M = 0, K = 0;  // the problem the layouts (and the timed search) were built for
};

constexpr size_t kMaxExactF8 = 64;

using F8Key = std::tuple<int64_t, int64_t, int64_t, int64_t, int64_t, int, int, int, int>;

struct F8State {
  // exact problems: (M, N, K, lda, ldb, dtype A, dtype B, fp32 out, device)
  std::map<F8Key, F8Plan> plans;
  // problems whose M or K changes from call to call (MoE expert segments): (M bucket, N, K bucket, lda, ldb, ...),
  // searched once on the first problem of the bucket
  std::map<F8Key, F8Plan> dyn_plans;
  int64_t dyn_calls = 0, dyn_reused = 0, dyn_heuristic = 0;
};

F8State& f8state() {
  static F8State s;
  return s;
}

hipDataType f8type(at::ScalarType t) { return t == at::kFloat8_e5m2 ? HIP_R_8F_E5M2 : HIP_R_8F_E4M3; }

bool set_scales(hipblasLtMatmulDesc_t desc, const void* sa, const void* sb) {
  // hipBLASLt's matA is B (weights / second operand), matB is A
  return check(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_A_SCALE_POINTER, &sb, sizeof(sb))) &&
         check(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_B_SCALE_POINTER, &sa, sizeof(sa)));
}

bool build_f8_plan(State& s, F8Plan& p, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, at::ScalarType ta_,
                   at::ScalarType tb_, bool out_f32, hipStream_t stream, const torch::Tensor& like) {
  const hipblasOperation_t opA = HIPBLAS_OP_T, opB = HIPBLAS_OP_N;
  const hipDataType dt = out_f32 ? HIP_R_32F : HIP_R_16BF;
  if (!check(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F))) return false;
  if (!check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)))) return false;
  if (!check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)))) return false;
  if (!check(hipblasLtMatrixLayoutCreate(&p.la, f8type(tb_), K, N, ldb))) return false;
  if (!check(hipblasLtMatrixLayoutCreate(&p.lb, f8type(ta_), K, M, lda))) return false;
  if (!check(hipblasLtMatrixLayoutCreate(&p.lc, dt, N, M, N))) return false;
  auto one_t = torch::ones({2}, like.options().dtype(torch::kFloat32));
  if (!set_scales(p.desc, one_t.data_ptr<float>(), one_t.data_ptr<float>() + 1)) return false;
  hipblasLtMatmulPreference_t pref;
  if (!check(hipblasLtMatmulPreferenceCreate(&pref))) return false;
  uint64_t ws = kWorkspace;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(search_width());
  int got = 0;
  const bool okh = check(hipblasLtMatmulAlgoGetHeuristic(s.handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, (int)res.size(),
                                                         res.data(), &got));
  hipblasLtMatmulPreferenceDestroy(pref);
  if (!okh || got <= 0) return false;
  p.candidates = got;
  auto a = torch::empty({M, lda}, like.options().dtype(torch::kUInt8)).random_(0, 64);  // small finite fp8 values
  auto b = torch::empty({N, ldb}, like.options().dtype(torch::kUInt8)).random_(0, 64);
  auto d = torch::empty({M, N}, like.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16));
  const float one = 1.f, zero = 0.f;
  auto run_i = [&](int i) {
    return check(hipblasLtMatmul(s.handle, p.desc, &one, b.data_ptr(), p.la, a.data_ptr(), p.lb, &zero, d.data_ptr(), p.lc,
                             d.data_ptr(), p.lc, &res[i].algo, workspace_for(s, stream, like), kWorkspace, stream));
  };
  float best = 0.f;
  const int bi = search_best(res, got, run_i, stream, 3, best);
  if (bi >= 0) {
    p.algo = res[bi].algo;
    p.ok = true;
  }
  p.ms = best;
  p.M = M;
  p.K = K;
  return p.ok;
}

// Run problem (M, K) of a dynamic family with the bucket plan's descriptor: the bucket's searched algorithm when
// hipBLASLt supports it for this exact problem, else the heuristic's first choice (neither path times anything or
// synchronises). The layouts are per call (host-side objects, read at enqueue).
bool run_dynamic(State& s, F8State& fs, F8Plan& plan, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                 at::ScalarType ta_, at::ScalarType tb_, bool out_f32, const void* a, const void* b, void* out,
                 float alpha, float beta, void* ws, hipStream_t stream) {
  if (M == plan.M && K == plan.K)
    return check(hipblasLtMatmul(s.handle, plan.desc, &alpha, b, plan.la, a, plan.lb, &beta, out, plan.lc, out, plan.lc,
                                 &plan.algo, ws, kWorkspace, stream));
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  bool ok = check(hipblasLtMatrixLayoutCreate(&la, f8type(tb_), K, N, ldb)) &&
            check(hipblasLtMatrixLayoutCreate(&lb, f8type(ta_), K, M, lda)) &&
            check(hipblasLtMatrixLayoutCreate(&lc, out_f32 ? HIP_R_32F : HIP_R_16BF, N, M, N));
  hipblasLtMatmulAlgo_t algo = plan.algo;
  if (ok) {
    size_t ws = 0;
    ++fs.dyn_calls;
    if (hipblaslt_ext::matmulIsAlgoSupported(s.handle, plan.desc, &alpha, la, lb, &beta, lc, lc, algo, ws) ==
            HIPBLAS_STATUS_SUCCESS && ws <= kWorkspace) {
      ++fs.dyn_reused;
    } else {
      hipblasLtMatmulPreference_t pref;
      ok = check(hipblasLtMatmulPreferenceCreate(&pref));
      if (ok) {
        uint64_t wsl = kWorkspace;
        hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsl, sizeof(wsl));
        hipblasLtMatmulHeuristicResult_t r;
        int got = 0;
        ok = check(hipblasLtMatmulAlgoGetHeuristic(s.handle, plan.desc, la, lb, lc, lc, pref, 1, &r, &got)) && got > 0 &&
             r.state == HIPBLAS_STATUS_SUCCESS;
        if (ok) algo = r.algo;
        hipblasLtMatmulPreferenceDestroy(pref);
        ++fs.dyn_heuristic;
      }
    }
  }
  if (ok)
    ok = check(hipblasLtMatmul(s.handle, plan.desc, &alpha, b, la, a, lb, &beta, out, lc, out, lc, &algo, ws, kWorkspace,
                               stream));
  if (la) hipblasLtMatrixLayoutDestroy(la);
  if (lb) hipblasLtMatrixLayoutDestroy(lb);
  if (lc) hipblasLtMatrixLayoutDestroy(lc);
  return ok;
}

}  // namespace

// Returns false (nothing launched) when hipBLASLt has no working algorithm for the problem; the caller then uses the
// hand-written MX-MFMA kernel. `dynamic`: M and / or K change from call to call (MoE expert segments) — one timed
// search per power-of-two bucket of (M, K), every other problem of the bucket reuses that algorithm (or, where it does
// not apply, hipBLASLt's first heuristic choice) without a search or a host synchronisation.
bool blaslt_fp8_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor sa, torch::Tensor sb, double alpha, torch::Tensor out,
                     bool accumulate, bool dynamic) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda() && sa.is_cuda() && sb.is_cuda(), "blaslt_fp8_gemm: HIP tensors expected");
  const auto ta = a.scalar_type(), tb = b.scalar_type();
  TORCH_CHECK((ta == at::kFloat8_e4m3fn || ta == at::kFloat8_e5m2) && (tb == at::kFloat8_e4m3fn || tb == at::kFloat8_e5m2),
              "blaslt_fp8_gemm: e4m3 / e5m2 operands expected");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "blaslt_fp8_gemm: bf16 / fp32 output");
  TORCH_CHECK(sa.scalar_type() == at::kFloat && sb.scalar_type() == at::kFloat && sa.numel() >= 1 && sb.numel() >= 1,
              "blaslt_fp8_gemm: fp32 scale tensors expected");
  // A and B may be row slices / column windows of larger row-major matrices (leading dimension = stride(0), e.g. an
  // expert's token range of a transposed activation for the MoE weight gradient); C is contiguous
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1 &&
                  a.stride(0) >= a.size(1) && b.stride(0) >= b.size(1) && out.is_contiguous(),
              "blaslt_fp8_gemm: 2-D row-major operands (unit column stride) and a contiguous output expected");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  const int64_t lda = a.stride(0), ldb = b.stride(0);
  TORCH_CHECK(b.size(1) == K && out.size(0) == M && out.size(1) == N, "blaslt_fp8_gemm: shape mismatch");
  const bool out_f32 = out.scalar_type() == at::kFloat;
  State& s = state();
  F8State& fs = f8state();
  hipStream_t stream = at::hip::getCurrentHIPStream();
  F8Plan* plan = nullptr;
  void* ws = nullptr;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.handle == nullptr) {
      if (!check(hipblasLtCreate(&s.handle))) return false;
      s.workspace = torch::empty({(int64_t)kWorkspace}, out.options().dtype(torch::kUInt8));
    }
    // exact-problem searches are capped: past kMaxExactF8 distinct problems (variable-length batches) every new
    // problem joins the power-of-two bucket family instead of getting a timed search of its own
    if (!dynamic && fs.plans.size() >= kMaxExactF8 &&
        fs.plans.find(std::make_tuple(M, N, K, lda, ldb, (int)ta, (int)tb, (int)out_f32, (int)out.get_device())) == fs.plans.end())
      dynamic = true;
    auto& table = dynamic ? fs.dyn_plans : fs.plans;
    auto key = dynamic ? std::make_tuple(dim_bucket(M), N, dim_bucket(K), lda, ldb, (int)ta, (int)tb, (int)out_f32, (int)out.get_device())
                       : std::make_tuple(M, N, K, lda, ldb, (int)ta, (int)tb, (int)out_f32, (int)out.get_device());
    auto it = table.find(key);
    if (it == table.end()) {
      F8Plan p;
      build_f8_plan(s, p, M, N, K, lda, ldb, ta, tb, out_f32, stream, out);
      it = table.emplace(key, p).first;
    }
    plan = &it->second;
    if (!plan->ok) return false;
    if (!set_scales(plan->desc, sa.data_ptr(), sb.data_ptr())) return false;
    ws = workspace_for(s, stream, out);
    if (dynamic)
      return run_dynamic(s, fs, *plan, M, N, K, lda, ldb, ta, tb, out_f32, a.data_ptr(), b.data_ptr(), out.data_ptr(),
                         (float)alpha, accumulate ? 1.f : 0.f, ws, stream);
    // enqueued while the lock is held: the scale pointers just written into the shared descriptor belong to THIS call
    // (another thread using the same plan could otherwise overwrite them before hipblasLtMatmul reads them)
    const float al = (float)alpha, beta = accumulate ? 1.f : 0.f;
    return check(hipblasLtMatmul(s.handle, plan->desc, &al, b.data_ptr(), plan->la, a.data_ptr(), plan->lb, &beta,
                                 out.data_ptr(), plan->lc, out.data_ptr(), plan->lc, &plan->algo, ws, kWorkspace, stream));
  }
}

// ------------------------------------------------------------------------------------------------ MXFP8 (block scales)
// C[M, N] (=|+=) (A[M, K] . B[N, K]^T) with one e8m0 scale per 32-element K block of every row of A and B
// (HIPBLASLT_MATMUL_MATRIX_SCALE_VEC32_UE8M0); sa / sb are the scale tensors in the layout hipBLASLt reads (the caller
// converts from the quantiser's grouped layout). Same TN mapping and per-problem algorithm timing as the per-tensor
// runner above. Returns false when hipBLASLt has no MX algorithm for the problem.
namespace {

struct MxState {
  std::map<std::tuple<int64_t, int64_t, int64_t, int, int, int, int>, F8Plan> plans;
};

MxState& mxstate() {
  static MxState s;
  return s;
}

bool set_mx_scales(hipblasLtMatmulDesc_t desc, const void* sa, const void* sb) {
  const int32_t mode = HIPBLASLT_MATMUL_MATRIX_SCALE_VEC32_UE8M0;
  return check(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_A_SCALE_MODE, &mode, sizeof(mode))) &&
         check(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_B_SCALE_MODE, &mode, sizeof(mode))) &&
         set_scales(desc, sa, sb);
}

bool build_mx_plan(State& s, F8Plan& p, int64_t M, int64_t N, int64_t K, at::ScalarType ta_, at::ScalarType tb_,
                   bool out_f32, hipStream_t stream, const torch::Tensor& like) {
  const hipblasOperation_t opA = HIPBLAS_OP_T, opB = HIPBLAS_OP_N;
  const hipDataType dt = out_f32 ? HIP_R_32F : HIP_R_16BF;
  if (!check(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F))) return false;
  if (!check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)))) return false;
  if (!check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)))) return false;
  if (!check(hipblasLtMatrixLayoutCreate(&p.la, f8type(tb_), K, N, K))) return false;
  if (!check(hipblasLtMatrixLayoutCreate(&p.lb, f8type(ta_), K, M, K))) return false;
  if (!check(hipblasLtMatrixLayoutCreate(&p.lc, dt, N, M, N))) return false;
  auto sa_s = torch::full({M * K / 32}, 127, like.options().dtype(torch::kUInt8));
  auto sb_s = torch::full({N * K / 32}, 127, like.options().dtype(torch::kUInt8));
  if (!set_mx_scales(p.desc, sa_s.data_ptr(), sb_s.data_ptr())) return false;
  hipblasLtMatmulPreference_t pref;
  if (!check(hipblasLtMatmulPreferenceCreate(&pref))) return false;
  uint64_t ws = kWorkspace;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(8);  // the heuristic's first 8: some MX candidates are very slow
  int got = 0;
  const bool okh = check(hipblasLtMatmulAlgoGetHeuristic(s.handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, (int)res.size(),
                                                         res.data(), &got));
  hipblasLtMatmulPreferenceDestroy(pref);
  if (!okh || got <= 0) return false;
  p.candidates = got;
  auto a = torch::empty({M, K}, like.options().dtype(torch::kUInt8)).random_(0, 64);
  auto b = torch::empty({N, K}, like.options().dtype(torch::kUInt8)).random_(0, 64);
  auto d = torch::empty({M, N}, like.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16));
  const float one = 1.f, zero = 0.f;
  auto run_i = [&](int i) {
    return check(hipblasLtMatmul(s.handle, p.desc, &one, b.data_ptr(), p.la, a.data_ptr(), p.lb, &zero, d.data_ptr(), p.lc,
                             d.data_ptr(), p.lc, &res[i].algo, workspace_for(s, stream, like), kWorkspace, stream));
  };
  float best = 0.f;
  const int bi = search_best(res, got, run_i, stream, 2, best);
  if (bi >= 0) {
    p.algo = res[bi].algo;
    p.ok = true;
  }
  p.ms = best;
  p.M = M;
  p.K = K;
  return p.ok;
}

}  // namespace

bool blaslt_mx_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor sa, torch::Tensor sb, torch::Tensor out,
                    bool accumulate) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda() && sa.is_cuda() && sb.is_cuda(), "blaslt_mx_gemm: HIP tensors");
  const auto ta = a.scalar_type(), tb = b.scalar_type();
  TORCH_CHECK((ta == at::kFloat8_e4m3fn || ta == at::kFloat8_e5m2) && (tb == at::kFloat8_e4m3fn || tb == at::kFloat8_e5m2),
              "blaslt_mx_gemm: e4m3 / e5m2 operands expected");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && out.is_contiguous() &&
                  sa.is_contiguous() && sb.is_contiguous() && sa.scalar_type() == at::kByte && sb.scalar_type() == at::kByte,
              "blaslt_mx_gemm: contiguous operands, uint8 e8m0 scales");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && out.size(0) == M && out.size(1) == N && K % 32 == 0 && sa.numel() == M * K / 32 &&
                  sb.numel() == N * K / 32, "blaslt_mx_gemm: shape mismatch");
  const bool out_f32 = out.scalar_type() == at::kFloat;
  TORCH_CHECK(out_f32 || out.scalar_type() == at::kBFloat16, "blaslt_mx_gemm: bf16 / fp32 output");
  State& s = state();
  hipStream_t stream = at::hip::getCurrentHIPStream();
  F8Plan* plan = nullptr;
  void* ws = nullptr;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.handle == nullptr) {
      if (!check(hipblasLtCreate(&s.handle))) return false;
      s.workspace = torch::empty({(int64_t)kWorkspace}, out.options().dtype(torch::kUInt8));
    }
    auto key = std::make_tuple(M, N, K, (int)ta, (int)tb, (int)out_f32, (int)out.get_device());
    auto& plans = mxstate().plans;
    auto it = plans.find(key);
    if (it == plans.end()) {
      F8Plan p;
      build_mx_plan(s, p, M, N, K, ta, tb, out_f32, stream, out);
      it = plans.emplace(key, p).first;
    }
    plan = &it->second;
    if (!plan->ok) return false;
    if (!set_mx_scales(plan->desc, sa.data_ptr(), sb.data_ptr())) return false;
    ws = workspace_for(s, stream, out);
    const float one = 1.f, beta = accumulate ? 1.f : 0.f;  // enqueued under the lock (scale pointers, as above)
    return check(hipblasLtMatmul(s.handle, plan->desc, &one, b.data_ptr(), plan->la, a.data_ptr(), plan->lb, &beta,
                                 out.data_ptr(), plan->lc, out.data_ptr(), plan->lc, &plan->algo, ws, kWorkspace, stream));
  }
}

// [(M, N, K, candidates, best ms)] of every fp8 problem searched so far.
std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t, double>> blaslt_fp8_plans() {
  std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t, double>> out;
  State& s = state();
  std::lock_guard<std::mutex> lk(s.mu);
  for (auto& kv : f8state().plans)
    out.emplace_back(std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first), kv.second.candidates,
                     kv.second.ok ? kv.second.ms : -1.0);
  return out;
}

// (bucket searches, dynamic calls on a non-representative problem, of which the bucket algorithm was reused, of
// which the heuristic choice ran)
std::vector<int64_t> blaslt_fp8_dynamic_stats() {
  State& s = state();
  std::lock_guard<std::mutex> lk(s.mu);
  F8State& fs = f8state();
  return {(int64_t)fs.dyn_plans.size(), fs.dyn_calls, fs.dyn_reused, fs.dyn_heuristic};
}

// [(T, N, K, candidates, best ms)] of every shape searched so far (diagnostics / bench logs).
std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t, double>> blaslt_wgrad_plans() {
  std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t, double>> out;
  State& s = state();
  std::lock_guard<std::mutex> lk(s.mu);
  for (auto& kv : s.plans)
    out.emplace_back(std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first), kv.second.candidates,
                     kv.second.ok ? kv.second.ms : -1.0);
  return out;
}
