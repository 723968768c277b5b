// Grouped GEMMs for Mixture-of-Experts layers (bf16 and MX-fp8) driven by a DEVICE-side segment table: one launch
// per projection and direction, no host synchronisation, no per-expert launch loop.
//
// Tokens are sorted by expert into one buffer in which every expert's segment starts at a multiple of 64 rows (the
// few pad rows are zero). `seg[0..E]` (int32, device) holds the segment boundaries in rows. Two modes:
//   GROUP_M  (forward / dgrad):  C[r, :] = A[r, :] . B_e^T        for rows r of segment e      A [R, K], B [E, N, K]
//   GROUP_K  (weight gradient):  C_e     = A[:, seg_e] . B[:, seg_e]^T  (K restricted to segment e)  C [E, M, N]
// Both operands are K-contiguous ("TN"); the layer produces the transposed copies it needs (the fp8 cast kernel writes
// both layouts in one pass, weights are transposed once per step).
//
// The main loop is the MX-fp8 GEMM v3 structure (csrc/kernels/fp8.hip): 256x256 tile, 4 waves of 128x128 (one per
// SIMD, accumulators in AGPRs), BK = 64 bytes per K-tile, a 4-deep LDS ring filled by buffer_load ... lds off SGPR
// descriptors, one counted vmcnt + barrier per K-tile placed mid-tile, fragment reads and DMA interleaved with the
// MFMAs, branch-free loop. K-tiles past a segment's end are staged from an out-of-range soffset, so the hardware range
// check feeds zeros and the loop needs no tail handling. bf16 uses v_mfma_f32_32x32x16_bf16 twice per 64-byte K-tile
// on the same fragments (the two 16-B halves of each lane's 32 bytes; A and B use the same k permutation).
//
// GROUP_M: the grid is sized on the host from an upper bound (ceil(R / 256) + E + 1 row tiles x N tiles); each
// workgroup finds its (expert, row tile) by a scalar walk over seg[]; the spare workgroups zero the rows past seg[E]
// and exit before touching LDS. Output rows past a segment's end are not written (they belong to the next expert).
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"
#include <type_traits>

using namespace acc;

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GG_BM = 256, GG_BN = 256, GG_BK = 64;  // BK in bytes
constexpr int GG_TILE = (GG_BM + GG_BN) * GG_BK;
constexpr int GG_BOFF = GG_BM * GG_BK;
constexpr int kModeM = 1, kModeK = 2;
constexpr int kBf16 = -1;  // operand "format" for bf16 (fp8 formats: 0 = e4m3, 1 = e5m2)

__device__ __forceinline__ int gg_swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

struct GGArgs {
  const uint8_t* A;
  const uint8_t* B;
  void* C;
  const int* seg;       // [E + 1] segment boundaries (rows of A for GROUP_M, K positions for GROUP_K)
  const float* sa;      // A scale: [1] (fp8 amax-derived inverse scale, or 1)
  const float* sb;      // B scale: [E] for GROUP_M (per-expert weight), [1] for GROUP_K
  float smul;
  int R;                // GROUP_M: rows of A / C.  GROUP_K: M (rows of A, C_e)
  int N;                // columns of C
  int K;                // GROUP_M: K (elements).  GROUP_K: total K length of A / B rows (elements)
  int E;
  int accum;
};

template <int FA, int FB, bool OUT_F32, int MODE>
__global__ __launch_bounds__(256, 1) void grouped_gemm_kernel(GGArgs p) {
  __shared__ __attribute__((aligned(1024))) uint8_t ring0[GG_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring1[GG_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring2[GG_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring3[GG_TILE];
  constexpr bool BF = FA == kBf16;
  constexpr int ES = BF ? 2 : 1;  // element size
  constexpr int TI = 4, TJ = 4, DPW = 4;
  const int tiles_n = p.N / GG_BN;
  const int Kb = p.K * ES;  // row length in bytes (GROUP_M: of A and B_e; GROUP_K: of A and B)

  // ---- tile -> (expert, output rows, K range)
  int e = 0, row0 = 0, row_end = 0, tn = 0, k_base = 0, nk = 0;
  const uint8_t* Bp = p.B;
  if constexpr (MODE == kModeM) {
    const int mt = blockIdx.x / tiles_n;
    tn = (blockIdx.x % tiles_n) * GG_BN;
    int acc = 0;
    e = -1;
    for (int i = 0; i < p.E; ++i) {  // wave-uniform scalar walk over the segment table
      const int lo = p.seg[i], hi = p.seg[i + 1];
      // debug build: segments are ordered and inside the routed buffer (a bad table would read / write past it)
      ACC_CHECK_OR_RETURN(lo >= 0 && hi >= lo && hi <= p.R, kChkGroupSeg);
      const int nt = (hi - lo + GG_BM - 1) / GG_BM;
      if (e < 0 && mt < acc + nt) {
        e = i;
        row0 = lo + (mt - acc) * GG_BM;
        row_end = hi;
      }
      acc += nt;
    }
    if (e < 0) {
      // past the last real tile (uniform, before any LDS / barrier): the spare row tiles zero the buffer's tail rows
      // [seg[E], R), so every row of the output is defined (fp8 amax / casts run over the whole buffer)
      const int r0 = p.seg[p.E] + (mt - acc) * GG_BM;
      if (p.accum || r0 >= p.R) return;
      constexpr int esz = OUT_F32 ? 4 : 2, cpr = GG_BN * esz / 16;  // 16-B chunks per tile row
      const int rows = min(GG_BM, p.R - r0);
      uint8_t* base = reinterpret_cast<uint8_t*>(p.C) + ((long)r0 * p.N + tn) * esz;
      for (int c = threadIdx.x; c < rows * cpr; c += 256)
        *reinterpret_cast<uint4*>(base + (long)(c / cpr) * p.N * esz + (c % cpr) * 16) = make_uint4(0, 0, 0, 0);
      return;
    }
    Bp = p.B + (long)e * p.N * Kb;
    nk = Kb / GG_BK;
  } else {
    const int tiles_m = p.R / GG_BM;
    const int per = tiles_m * tiles_n;
    e = blockIdx.x / per;
    const int t = blockIdx.x % per;
    row0 = (t / tiles_n) * GG_BM;
    row_end = row0 + GG_BM;
    tn = (t % tiles_n) * GG_BN;
    k_base = p.seg[e] * ES;
    nk = (p.seg[e + 1] - p.seg[e]) * ES / GG_BK;
  }
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int wv = __builtin_amdgcn_readfirstlane(wave);
  unsigned voff[DPW];
#pragma unroll
  for (int t = 0; t < DPW; ++t) {
    const int row = (wv * DPW + t) * 16 + (lane >> 2);
    voff[t] = (unsigned)(row * Kb + gg_swz(row, lane & 3) * 16);
  }
  // A panel: rows [row0, row0 + 256) (GROUP_M: clipped to the buffer, the range check zero-fills the rest)
  const long a_rows = MODE == kModeM ? (long)min(GG_BM, p.R - row0) : (long)GG_BM;
  const auto a_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (long)row0 * Kb), (short)0, (int)(a_rows * Kb), 0x00020000);
  const auto b_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(Bp + (long)tn * Kb), (short)0, GG_BN * Kb, 0x00020000);
  auto stage = [&](int kt, uint8_t* base) {
    const int so = kt < nk ? k_base + kt * GG_BK : 0x40000000;  // past the segment: zeros, no memory traffic
#pragma unroll
    for (int t = 0; t < DPW; ++t) {
      const int blk = wv * DPW + t;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rs, base + blk * 1024, 16, voff[t], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rs, base + GG_BOFF + blk * 1024, 16, voff[t], so, 0, 0);
    }
  };
  const int sw = (r >> 2) & 3;
  const int lo0 = ((2 * hf) ^ sw) * 16, lo1 = ((2 * hf + 1) ^ sw) * 16;
  const int arow = (wm + r) * GG_BK, brow = GG_BOFF + (wn + r) * GG_BK;
  auto frag = [&](const uint8_t* q) -> v8i {
    const uint4 lo = *reinterpret_cast<const uint4*>(q + lo0);
    const uint4 hi = *reinterpret_cast<const uint4*>(q + lo1);
    v8i v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };
  auto load = [&](const uint8_t* img, v8i (&fa)[TI], v8i (&fb)[TJ]) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[j] = frag(img + brow + j * 32 * GG_BK);
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[i] = frag(img + arow + i * 32 * GG_BK);
  };
  auto mma = [&](const v8i& b, const v8i& a, f32x16& c) {
    if constexpr (BF) {  // the lane's two 16-B halves are two k-slices of 8 bf16
      typedef int v4i __attribute__((ext_vector_type(4)));
      const v4i b0 = {b[0], b[1], b[2], b[3]}, b1 = {b[4], b[5], b[6], b[7]};
      const v4i a0 = {a[0], a[1], a[2], a[3]}, a1 = {a[4], a[5], a[6], a[7]};
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, b0), __builtin_bit_cast(v8bf, a0), c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, b1), __builtin_bit_cast(v8bf, a1), c, 0, 0, 0);
    } else {
      c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a, c, FB, FA, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
    }
  };
  auto mfma_rows = [&](const v8i (&fa)[TI], const v8i (&fb)[TJ], int i0) {
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) mma(fb[j], fa[i], acc[i][j]);  // acc = C^T tile (lane <-> m, regs <-> n)
  };
  constexpr int MF = BF ? 2 : 1;  // MFMAs per (i, j) per K-tile

  stage(0, ring0);
  stage(1, ring1);
  stage(2, ring2);
  stage(3, ring3);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  v8i xa[TI], xb[TJ], ya[TI], yb[TJ];
  load(ring0, xa, xb);
  auto step = [&](int t, uint8_t* slot, const uint8_t* nslot, v8i (&ca)[TI], v8i (&cb)[TJ], v8i (&na)[TI], v8i (&nb)[TJ]) {
    mfma_rows(ca, cb, 0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stage(t + 4, slot);
    load(nslot, na, nb);
    mfma_rows(ca, cb, 2);
#pragma unroll
    for (int k = 0; k < 8 * MF; ++k) {
      if (k % MF == 0) {
        __builtin_amdgcn_sched_group_barrier(0x10, 1, 0);   // VMEM (buffer_load ... lds)
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
      }
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);      // MFMA
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // K-tiles past nk read zeros, so running whole groups of four is exact
  for (int t = 0; t < nk; t += 4) {
    step(t, ring0, ring1, xa, xb, ya, yb);
    step(t + 1, ring1, ring2, ya, yb, xa, xb);
    step(t + 2, ring2, ring3, xa, xb, ya, yb);
    step(t + 3, ring3, ring0, ya, yb, xa, xb);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const float s = p.sa[0] * (MODE == kModeM ? p.sb[e] : p.sb[0]) * p.smul;
  const int N = p.N;
  void* Cb = MODE == kModeK ? (void*)(reinterpret_cast<uint8_t*>(p.C) + (long)e * p.R * N * (OUT_F32 ? 4 : 2)) : p.C;
  auto epilogue = [&](auto acc_in) {
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int m = row0 + wm + i * 32 + r;
      if (MODE == kModeM && m >= row_end) continue;
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = tn + wn + j * 32 + 8 * g + 4 * hf;
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = acc[i][j][4 * g + u] * s;
          if constexpr (OUT_F32) {
            float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(Cb) + (long)m * N + n);
            if constexpr (decltype(acc_in)::value) {
              const float4 o = *cp4;
              v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
            }
            *cp4 = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(Cb) + (long)m * N + n);
            if constexpr (decltype(acc_in)::value) {
              const bf16x4 o = *cp4;
#pragma unroll
              for (int u = 0; u < 4; ++u) v[u] += bf2f(o.v[u]);
            }
            bf16x4 w;
#pragma unroll
            for (int u = 0; u < 4; ++u) w.v[u] = f2bf(v[u]);
            *cp4 = w;
          }
        }
    }
  };
  if (p.accum) epilogue(std::true_type{});
  else epilogue(std::false_type{});
}

int fmt_of(const torch::Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return kBf16;
  if (t.scalar_type() == at::kFloat8_e4m3fn) return 0;
  if (t.scalar_type() == at::kFloat8_e5m2) return 1;
  TORCH_CHECK(false, "grouped_gemm: operands must be bf16, float8_e4m3fn or float8_e5m2");
  return 0;
}

}  // namespace

ACC_DEBUG_TAKE_FN(acc_dbg_take_grouped_gemm)

// mode 1 (GROUP_M): a [R, K], b [E, N, K], out [R, N]; seg [E+1] row boundaries.
// mode 2 (GROUP_K): a [M, Ktot], b [N, Ktot], out [E, M, N]; seg [E+1] K boundaries.
// sa: [1]; sb: [E] (mode 1) or [1] (mode 2). C = (A . B^T) * sa * sb * smul (+ out when accumulate).
// Segment starts (and, for mode 2, lengths) must be multiples of 64 elements; M, N multiples of 256, K (mode 1) of 256.
void grouped_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor out, torch::Tensor seg, int64_t mode, torch::Tensor sa,
                  torch::Tensor sb, double smul, bool accumulate) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda() && seg.is_cuda(), "grouped_gemm: HIP tensors expected");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && out.is_contiguous() && seg.is_contiguous(), "grouped_gemm: contiguous");
  TORCH_CHECK(seg.scalar_type() == at::kInt && seg.dim() == 1 && seg.numel() >= 2, "grouped_gemm: seg must be int32 [E+1]");
  TORCH_CHECK(sa.scalar_type() == at::kFloat && sb.scalar_type() == at::kFloat, "grouped_gemm: fp32 scales");
  const int fa = fmt_of(a), fb = fmt_of(b);
  TORCH_CHECK((fa == kBf16) == (fb == kBf16), "grouped_gemm: both operands bf16 or both fp8");
  const bool of32 = out.scalar_type() == at::kFloat;
  TORCH_CHECK(of32 || out.scalar_type() == at::kBFloat16, "grouped_gemm: out must be fp32 or bf16");
  const int E = seg.numel() - 1;
  GGArgs p{};
  p.A = reinterpret_cast<const uint8_t*>(a.data_ptr());
  p.B = reinterpret_cast<const uint8_t*>(b.data_ptr());
  p.C = out.data_ptr();
  p.seg = seg.data_ptr<int>();
  p.sa = sa.data_ptr<float>();
  p.sb = sb.data_ptr<float>();
  p.smul = (float)smul;
  p.E = E;
  p.accum = accumulate ? 1 : 0;
  const int es = fa == kBf16 ? 2 : 1;
  long grid = 0;
  if (mode == kModeM) {
    TORCH_CHECK(a.dim() == 2 && b.dim() == 3 && b.size(0) == E && b.size(2) == a.size(1), "grouped_gemm(M): a [R,K], b [E,N,K]");
    p.R = a.size(0);
    p.K = a.size(1);
    p.N = b.size(1);
    TORCH_CHECK(out.dim() == 2 && out.size(0) == p.R && out.size(1) == p.N, "grouped_gemm(M): out [R, N]");
    TORCH_CHECK(sb.numel() == E, "grouped_gemm(M): sb must hold one scale per expert");
    TORCH_CHECK(p.N % GG_BN == 0 && (p.K * es) % (4 * GG_BK) == 0, "grouped_gemm(M): N % 256, K bytes % 256");
    TORCH_CHECK((long)GG_BM * p.K * es < (1L << 30), "grouped_gemm(M): row panel too large");  // < the zero-fill soffset
    grid = ((long)(p.R + GG_BM - 1) / GG_BM + E + 1) * (p.N / GG_BN);  // real tiles + tail-zeroing tiles
  } else {
    TORCH_CHECK(mode == kModeK, "grouped_gemm: mode 1 (group rows) or 2 (group K)");
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "grouped_gemm(K): a [M,Ktot], b [N,Ktot]");
    p.R = a.size(0);
    p.N = b.size(0);
    p.K = a.size(1);
    TORCH_CHECK(out.dim() == 3 && out.size(0) == E && out.size(1) == p.R && out.size(2) == p.N, "grouped_gemm(K): out [E, M, N]");
    TORCH_CHECK(p.R % GG_BM == 0 && p.N % GG_BN == 0 && (p.K * es) % 16 == 0, "grouped_gemm(K): M, N % 256");
    TORCH_CHECK((long)GG_BM * p.K * es < (1L << 30), "grouped_gemm(K): row panel too large");
    grid = (long)E * (p.R / GG_BM) * (p.N / GG_BN);
  }
  if (grid == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
#define GG_LAUNCH(FA, FB, OF, MD) hipLaunchKernelGGL((grouped_gemm_kernel<FA, FB, OF, MD>), dim3(grid), dim3(256), 0, stream, p)
#define GG_OUT(FA, FB, MD) do { if (of32) GG_LAUNCH(FA, FB, true, MD); else GG_LAUNCH(FA, FB, false, MD); } while (0)
#define GG_FMT(MD)                                                              \
  do {                                                                          \
    if (fa == kBf16) GG_OUT(kBf16, kBf16, MD);                                  \
    else if (fa == 0 && fb == 0) GG_OUT(0, 0, MD);                              \
    else if (fa == 1 && fb == 0) GG_OUT(1, 0, MD);                              \
    else if (fa == 0 && fb == 1) GG_OUT(0, 1, MD);                              \
    else GG_OUT(1, 1, MD);                                                      \
  } while (0)
  if (mode == kModeM) GG_FMT(kModeM);
  else GG_FMT(kModeK);
#undef GG_FMT
#undef GG_OUT
#undef GG_LAUNCH
}

torch::Tensor transpose_bf16(torch::Tensor x);
torch::Tensor u8_transpose(torch::Tensor x);

// [E, R, C] -> [E, C, R] (bf16: 64x64 LDS tiles, 16-B accesses; 1-byte: 128x128 tiles, 4x4 register byte transposes).
torch::Tensor batched_transpose(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 3 && x.is_contiguous(), "batched_transpose: contiguous [E, R, C] HIP tensor");
  if (x.element_size() == 1) return u8_transpose(x);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "batched_transpose: bf16 or 1-byte elements");
  return transpose_bf16(x);
}
