// fp8 (OCP e4m3fn / e5m2, native on gfx950) training kernels:
//   * per-tensor amax (block max + one device-scope atomic max per workgroup),
//   * scale-and-cast to fp8 with saturation, optionally also writing the transposed copy needed by the
//     dgrad / wgrad GEMMs (transpose staged through LDS),
//   * fp8 GEMM  C[M,N] = (A[M,K] . B[N,K]^T) * sa * sb (+ bias)  on v_mfma_scale_f32_32x32x64_f8f6f4 with unit
//     block scales (the MX-scaled MFMA runs at 2x the bf16 MFMA rate; the per-tensor scales are applied in the
//     epilogue). 128x128 tile, BK = 64, 4 waves (2x2) of 64x64, LDS double buffer with XOR-swizzled 16-B chunks,
//     XCD-aware tile order.
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"
#include <cstdlib>
#include <type_traits>

using namespace acc;

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr float kE4M3Max = 448.f;
constexpr float kE5M2Max = 57344.f;

__global__ __launch_bounds__(1024) void amax_kernel(const bf16_t* __restrict__ x, long n, unsigned int* __restrict__ out) {
  __shared__ float scratch[16];
  float m = 0.f;
  const long nvec = n >> 3;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  // four independent 16-B loads in flight per lane per iteration (a single dependent load per trip left the
  // grid-stride loop latency-bound at ~3 TB/s)
  for (; i + 3 * stride < nvec; i += 4 * stride) {
    bf16x8 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = reinterpret_cast<const bf16x8*>(x)[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(bf2f(a[u].v[j])));
  }
  for (; i < nvec; i += stride) {
    const bf16x8 a = reinterpret_cast<const bf16x8*>(x)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(bf2f(a.v[j])));
  }
  for (long i = nvec * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(bf2f(x[i])));
  m = block_max(m, scratch);
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(m));  // non-negative floats order like their bits
}

template <bool E5M2>
__device__ __forceinline__ uint32_t cvt_pair(float a, float b) {
  const float mx = E5M2 ? kE5M2Max : kE4M3Max;
  a = fminf(fmaxf(a, -mx), mx);
  b = fminf(fmaxf(b, -mx), mx);
  if (E5M2) return (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false) & 0xffffu;
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false) & 0xffffu;
}

// Scale of a cast: FROM_AMAX ? qmax / max(amax, tiny) : t[0] * qmax (t = a plain scale tensor). Reading the
// scale straight from the amax buffer on the device keeps the scale arithmetic out of separate tiny launches.
__device__ __forceinline__ float cast_scale(const float* t, float qmax, bool from_amax) {
  return from_amax ? qmax / fmaxf(t[0], 1e-12f) : t[0] * qmax;
}

// 4x4 byte transpose of four dwords (w[i] = bytes of row i): returns in c[j] the four bytes of column j.
__device__ __forceinline__ void transpose4x4(const uint32_t w[4], uint32_t c[4]) {
  const uint32_t lo01 = __builtin_amdgcn_perm(w[1], w[0], 0x05010400u), hi01 = __builtin_amdgcn_perm(w[1], w[0], 0x07030602u);
  const uint32_t lo23 = __builtin_amdgcn_perm(w[3], w[2], 0x05010400u), hi23 = __builtin_amdgcn_perm(w[3], w[2], 0x07030602u);
  c[0] = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);
  c[1] = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
  c[2] = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
  c[3] = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
}

template <bool E5M2>
__device__ __forceinline__ uint32_t cvt4(const bf16_t* v, float s) {
  return cvt_pair<E5M2>(bf2f(v[0]) * s, bf2f(v[1]) * s) | (cvt_pair<E5M2>(bf2f(v[2]) * s, bf2f(v[3]) * s) << 16);
}

// y = sat(x * scale) as fp8 [M, N]; optionally yt = y^T [N, M]. One 128x128 tile per 256-thread workgroup:
// each thread converts 4 x 16 elements (two 16-B loads -> one 16-B store per row piece) into a padded LDS byte
// tile; the transposed copy is read back as 4-byte words, transposed 4x4 in registers (v_perm_b32) and written as
// 16-B rows of yt, 8 lanes per 128-B line. Partial edge tiles take a per-element path.
constexpr int kCT = 128, kCTP = kCT + 4;  // tile edge, padded LDS row pitch (bytes)
template <bool E5M2, bool TRANS>
__global__ __launch_bounds__(256) void cast_kernel(const bf16_t* __restrict__ x, const float* __restrict__ st, float qmax,
                                                   int from_amax, uint8_t* __restrict__ y, uint8_t* __restrict__ yt, int M,
                                                   int N) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kCT * kCTP];
  {  // batched [E, M, N] stacks (grid.z = E): matrix z and its own scale / amax slot; grid.z = 1 otherwise
    const long zo = (long)blockIdx.z * M * N;
    x += zo;
    y += zo;
    if (TRANS) yt += zo;
    st += blockIdx.z;
  }
  const int tm = blockIdx.y * kCT, tn = blockIdx.x * kCT;
  const float s = cast_scale(st, qmax, from_amax != 0);
  const int tid = threadIdx.x;
  const bool full = tm + kCT <= M && tn + kCT <= N && (N % 16) == 0 && (M % 16) == 0;
  if (!full) {  // edge tile
    for (int e = tid; e < kCT * kCT; e += 256) {
      const int r = e / kCT, c = e % kCT, gm = tm + r, gn = tn + c;
      if (gm < M && gn < N) {
        const uint8_t v = cvt_pair<E5M2>(bf2f(x[(long)gm * N + gn]) * s, 0.f) & 0xff;
        y[(long)gm * N + gn] = v;
        if (TRANS) yt[(long)gn * M + gm] = v;
      }
    }
    return;
  }
  // phase 1: rows r = tid/8 + 32p, 16 columns c = (tid%8)*16
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int r = (tid >> 3) + pass * 32, c = (tid & 7) * 16;
    const bf16_t* src = x + (long)(tm + r) * N + tn + c;
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(src);
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(src + 8);
    uint4 w;
    w.x = cvt4<E5M2>(a.v, s);
    w.y = cvt4<E5M2>(a.v + 4, s);
    w.z = cvt4<E5M2>(b.v, s);
    w.w = cvt4<E5M2>(b.v + 4, s);
    *reinterpret_cast<uint4*>(y + (long)(tm + r) * N + tn + c) = w;
    if (TRANS) {
      uint32_t* t = reinterpret_cast<uint32_t*>(tile + r * kCTP + c);
      t[0] = w.x; t[1] = w.y; t[2] = w.z; t[3] = w.w;
    }
  }
  if (!TRANS) return;
  __syncthreads();
  // phase 2: output rows n = n4 .. n4+3 (tile columns), 16 output bytes m16 .. m16+15 each
  const int m16 = (tid & 7) * 16, n4 = (tid >> 3) * 4;
  uint32_t col[4][4];  // col[j][q]: bytes m16+4q .. +3 of output row n4+j
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t w[4], c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = *reinterpret_cast<const uint32_t*>(tile + (m16 + 4 * q + i) * kCTP + n4);
    transpose4x4(w, c);
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j][q] = c[j];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    *reinterpret_cast<uint4*>(yt + (long)(tn + n4 + j) * M + tm + m16) = make_uint4(col[j][0], col[j][1], col[j][2], col[j][3]);
}


// ------------------------------------------------------------------------------------------------ FSDP fp8 all-gather
// The sharded flat buffer holds several weights back to back; each weight gets its own per-tensor scale. Segment k =
// elements [lo[k], hi[k]) of the flat bf16 shard. One workgroup per (segment, 64 Ki-element chunk): 16-B loads (8
// bf16 per lane per load, four in flight), the chunk's unaligned head / tail element-wise, and ONE atomic max per
// 128 KB chunk (a 4 Ki-element chunk made ~7.6k same-address atomics per weight and the kernel ran 7x under HBM speed).
constexpr long kSegChunk = 65536;

__global__ __launch_bounds__(256) void seg_amax_kernel(const bf16_t* __restrict__ x, const long* __restrict__ lo,
                                                       const long* __restrict__ hi, unsigned int* __restrict__ out) {
  __shared__ float scratch[16];
  const int k = blockIdx.y;
  const long a = lo[k] + (long)blockIdx.x * kSegChunk, b = min(hi[k], a + kSegChunk);
  if (a >= b) return;  // workgroup-uniform: past the end of a shorter segment
  const long a8 = min(b, (a + 7) & ~7L), b8 = max(a8, b & ~7L);
  float m = 0.f;
  const int tid = threadIdx.x;
  if (tid < a8 - a) m = fabsf(bf2f(x[a + tid]));
  if (tid < b - b8) m = fmaxf(m, fabsf(bf2f(x[b8 + tid])));
  const bf16x8* xv = reinterpret_cast<const bf16x8*>(x + a8);
  const long nv = (b8 - a8) >> 3;
  long i = tid;
  for (; i + 768 < nv; i += 1024) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = xv[i + 256 * u];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(bf2f(v[u].v[j])));
  }
  for (; i < nv; i += 256) {
    const bf16x8 v = xv[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(bf2f(v.v[j])));
  }
  m = block_max(m, scratch);
  if (tid == 0) atomicMax(out + k, __float_as_uint(m));
}

// y[i] = e4m3(sat(x[i] * 448 / amax[k])) for i in segment k: the same conversion as cast_kernel, so a weight cast from
// its shard with the all-reduced amax is bit-identical to the weight cast whole. 16-B loads, 8-B stores.
__global__ __launch_bounds__(256) void seg_cast_kernel(const bf16_t* __restrict__ x, const long* __restrict__ lo,
                                                       const long* __restrict__ hi, const float* __restrict__ amax,
                                                       float qmax, uint8_t* __restrict__ y) {
  const int k = blockIdx.y;
  const long a = lo[k] + (long)blockIdx.x * kSegChunk, b = min(hi[k], a + kSegChunk);
  if (a >= b) return;
  const float s = cast_scale(amax + k, qmax, true);
  const long a8 = min(b, (a + 7) & ~7L), b8 = max(a8, b & ~7L);
  const int tid = threadIdx.x;
  if (tid < a8 - a) y[a + tid] = cvt_pair<false>(bf2f(x[a + tid]) * s, 0.f) & 0xff;
  if (tid < b - b8) y[b8 + tid] = cvt_pair<false>(bf2f(x[b8 + tid]) * s, 0.f) & 0xff;
  const bf16x8* xv = reinterpret_cast<const bf16x8*>(x + a8);
  uint2* yv = reinterpret_cast<uint2*>(y + a8);
  const long nv = (b8 - a8) >> 3;
  long i = tid;
  for (; i + 768 < nv; i += 1024) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = xv[i + 256 * u];
#pragma unroll
    for (int u = 0; u < 4; ++u) yv[i + 256 * u] = make_uint2(cvt4<false>(v[u].v, s), cvt4<false>(v[u].v + 4, s));
  }
  for (; i < nv; i += 256) {
    const bf16x8 v = xv[i];
    yv[i] = make_uint2(cvt4<false>(v.v, s), cvt4<false>(v.v + 4, s));
  }
}

// y = x^T for a [R, C] byte matrix (fp8 weights: the K-major copy the dgrad GEMM reads). 128x128 tiles through a
// padded LDS tile; 4x4 byte transposes in registers (v_perm_b32), 16-B stores. Edge tiles per element.
__global__ __launch_bounds__(256) void u8_transpose_kernel(const uint8_t* __restrict__ x, uint8_t* __restrict__ y, int R, int C) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kCT * kCTP];
  const int tr = blockIdx.y * kCT, tc = blockIdx.x * kCT, tid = threadIdx.x;
  x += (long)blockIdx.z * R * C;  // batched [E, R, C] -> [E, C, R]
  y += (long)blockIdx.z * R * C;
  if (!(tr + kCT <= R && tc + kCT <= C && (R % 16) == 0 && (C % 16) == 0)) {
    for (int e = tid; e < kCT * kCT; e += 256) {
      const int r = tr + e / kCT, c = tc + e % kCT;
      if (r < R && c < C) y[(long)c * R + r] = x[(long)r * C + c];
    }
    return;
  }
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int r = (tid >> 3) + pass * 32, c = (tid & 7) * 16;
    const uint4 w = *reinterpret_cast<const uint4*>(x + (long)(tr + r) * C + tc + c);
    uint32_t* t = reinterpret_cast<uint32_t*>(tile + r * kCTP + c);
    t[0] = w.x; t[1] = w.y; t[2] = w.z; t[3] = w.w;
  }
  __syncthreads();
  const int m16 = (tid & 7) * 16, n4 = (tid >> 3) * 4;
  uint32_t col[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t w[4], c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = *reinterpret_cast<const uint32_t*>(tile + (m16 + 4 * q + i) * kCTP + n4);
    transpose4x4(w, c);
#pragma unroll
    for (int j = 0; j < 4; ++j) col[j][q] = c[j];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    *reinterpret_cast<uint4*>(y + (long)(tc + n4 + j) * R + tr + m16) = make_uint4(col[j][0], col[j][1], col[j][2], col[j][3]);
}

// ------------------------------------------------------------------------------------------------ MXFP8 quantisation
// OCP MX block scaling (TransformerEngine's MXFP8BlockScaling recipe): every 32 consecutive elements along a GEMM's
// reduction dimension share one e8m0 scale 2^(e - 127); the elements are stored as sat(x / 2^(e - 127)) in e4m3 / e5m2.
// e is rounded UP from amax / fp8_max, so the block's largest element never saturates. Scales are stored one byte per
// block in a grouped order that matches the GEMM's fragment ownership: within each row, the 8 blocks of a 256-element
// group g are laid out as [hf = 0: q = 0..3 | hf = 1: q = 0..3] for block 8 g + 2 q + hf, so one dword is one lane's
// scales for four 64-wide K-tiles. mx_pos maps a block index to its byte.
__device__ __forceinline__ int mx_pos(int b) { return (b & ~7) | ((b & 1) << 2) | ((b >> 1) & 3); }

template <bool E5M2, typename Get>
__device__ __forceinline__ void mx_quant_block(Get get, uint8_t* __restrict__ q, uint8_t* __restrict__ sc) {
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) m = fmaxf(m, fabsf(get(j)));
  const uint32_t bits = __float_as_uint(m * (1.f / (E5M2 ? kE5M2Max : kE4M3Max)));
  uint32_t e = bits >> 23;              // m >= 0: the biased exponent of amax / fp8_max ...
  if ((bits & 0x7fffffu) != 0) e += 1;  // ... rounded up to a power of two >= it
  e = min(e, 253u);
  const float inv = __uint_as_float((254u - e) << 23);  // 2^(127 - e); all-zero blocks get e = 0
  *sc = (uint8_t)e;
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    w[k] = cvt_pair<E5M2>(get(4 * k) * inv, get(4 * k + 1) * inv) | (cvt_pair<E5M2>(get(4 * k + 2) * inv, get(4 * k + 3) * inv) << 16);
  reinterpret_cast<uint4*>(q)[0] = make_uint4(w[0], w[1], w[2], w[3]);
  reinterpret_cast<uint4*>(q)[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// x [R, C] bf16 -> q [R, C] + s [R, C/32] (blocks along C) and, with COL, qt [C, R] + st [C, R/32] (= x^T quantised
// along R: the operand of the GEMMs that reduce over R). One 64x64 tile per 256-thread workgroup, staged once in LDS
// as fp32; waves 0-1 quantise its 128 row blocks, waves 2-3 its 128 column blocks.
constexpr int kMxT = 64;
template <bool E5M2, bool COL>
__global__ __launch_bounds__(256) void mx_quant_kernel(const bf16_t* __restrict__ x, int R, int C, uint8_t* __restrict__ q,
                                                       uint8_t* __restrict__ s, uint8_t* __restrict__ qt, uint8_t* __restrict__ st) {
  __shared__ float tile[kMxT][kMxT + 1];
  const int r0 = blockIdx.y * kMxT, c0 = blockIdx.x * kMxT, tid = threadIdx.x;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int idx = tid + p * 256, row = idx >> 3, ch = (idx & 7) * 8;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (long)(r0 + row) * C + c0 + ch);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[row][ch + j] = bf2f(v.v[j]);
  }
  __syncthreads();
  if (tid < 128) {
    const int row = tid >> 1, blk = tid & 1;
    mx_quant_block<E5M2>([&](int j) { return tile[row][blk * 32 + j]; }, q + (long)(r0 + row) * C + c0 + blk * 32,
                         s + (long)(r0 + row) * (C / 32) + mx_pos(c0 / 32 + blk));
  } else if (COL) {
    const int i = tid - 128, col = i >> 1, blk = i & 1;
    mx_quant_block<E5M2>([&](int j) { return tile[blk * 32 + j][col]; }, qt + (long)(c0 + col) * R + r0 + blk * 32,
                         st + (long)(c0 + col) * (R / 32) + mx_pos(r0 / 32 + blk));
  }
}

// ------------------------------------------------------------------------------------------------ GEMM
constexpr int BM = 128, BN = 128, BK = 64;  // BK in fp8 elements (= bytes)

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

template <int FA, int FB, bool OUT_F32>
__global__ __launch_bounds__(256, 2) void fp8_gemm_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                          const float* __restrict__ sa, const float* __restrict__ sb, float smul,
                                                          const bf16_t* __restrict__ bias, void* __restrict__ C, int M,
                                                          int N, int K, int accum) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2][2][BM * BK];  // [buf][A/B][rows * 64 B]
  const int tiles_n = N / BN;
  const int nwg = (M / BM) * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = (bid / tiles_n) * BM, tn = (bid % tiles_n) * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // staging: 128 rows x 4 chunks of 16 B per operand = 512 chunks -> 2 per thread per operand
  uint4 ra[2], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int c = tid + t * 256, row = c >> 2, ch = c & 3;
      ra[t] = *reinterpret_cast<const uint4*>(A + (long)(tm + row) * K + k0 + ch * 16);
      rb[t] = *reinterpret_cast<const uint4*>(B + (long)(tn + row) * K + k0 + ch * 16);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int c = tid + t * 256, row = c >> 2, ch = c & 3;
      *reinterpret_cast<uint4*>(&smem[buf][0][row * 64 + swz(row, ch) * 16]) = ra[t];
      *reinterpret_cast<uint4*>(&smem[buf][1][row * 64 + swz(row, ch) * 16]) = rb[t];
    }
  };
  auto frag = [&](int buf, int which, int row) -> v8i {
    const uint8_t* base = &smem[buf][which][row * 64];
    const uint4 lo = *reinterpret_cast<const uint4*>(base + swz(row, 2 * hf) * 16);
    const uint4 hi = *reinterpret_cast<const uint4*>(base + swz(row, 2 * hf + 1) * 16);
    v8i v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };

  const int nk = K / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);  // issue next tile's loads before the MFMAs (latency hidden)
    v8i af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = frag(cur, 0, wm + i * 32 + r);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = frag(cur, 1, wn + j * 32 + r);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)  // swapped operands: acc = C^T tile (lane <-> m, registers <-> n)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bfr[j], af[i], acc[i][j], FB, FA, 0, 0x7f7f7f7f, 0,
                                                                    0x7f7f7f7f);
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }
  const float s = sa[0] * sb[0] * smul;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = tm + wm + i * 32 + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = tn + wn + j * 32 + 8 * g + 4 * hf;
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          v[t] = acc[i][j][4 * g + t] * s;
          if (bias != nullptr) v[t] += bf2f(bias[n + t]);
        }
        if (OUT_F32) {
          float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (long)m * N + n);
          if (accum) {
            const float4 o = *cp4;
            v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
          }
          *cp4 = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(C) + (long)m * N + n);
          if (accum) {
            const bf16x4 o = *cp4;
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] += bf2f(o.v[t]);
          }
          bf16x4 w;
#pragma unroll
          for (int t = 0; t < 4; ++t) w.v[t] = f2bf(v[t]);
          *cp4 = w;
        }
      }
    }
}

// ------------------------------------------------------------------------------------------------ GEMM v2
// 256x256 output tile, BK = 128 fp8 bytes per K-step, MX-scaled 32x32x64 MFMA (2x the bf16 MFMA rate).
// Wave grid WM x WN (default 2 x 2 = 4 waves, one per SIMD, 128x128 outputs per wave: 256 accumulator registers
// in AGPRs, which only the full 512-entry register file of a one-wave-per-SIMD workgroup holds without spills).
// Operands are staged HBM/L2 -> LDS with global_load_lds_dwordx4 (no VGPR round trip, no ds_write): one
// wave-instruction fills 1 KiB = 8 rows x 128 B of the LDS image. The image is XOR-swizzled per 16-B chunk,
// chunk' = chunk ^ ((row >> 1) & 7), which makes every ds_read_b128 lane group of a 32x32x64 fragment read hit
// 16 distinct 16-B slots of the 256-B bank row (conflict-free); because a DMA writes lane-linearly, the swizzle
// is applied to each lane's *global source* address instead. Two LDS stages (2 x 64 KiB): the next K-step's
// DMA is in flight while the current one runs its MFMAs; one vmcnt(0) + barrier per K-step.
constexpr int V2_BM = 256, V2_BN = 256, V2_BK = 128;
constexpr int V2_STAGE = (V2_BM + V2_BN) * V2_BK;  // bytes per stage (A image then B image)

__device__ __forceinline__ int v2_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Body shared by the two wave layouts; each __global__ wrapper below fixes its own launch bounds (a
// template-dependent __launch_bounds__ on the kernel itself leaves the host stub undefined).
template <int FA, int FB, bool OUT_F32, int WM, int WN>
__device__ __forceinline__ void fp8_gemm_v2_body(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                 const float* __restrict__ sa, const float* __restrict__ sb, float smul,
                                                 const bf16_t* __restrict__ bias, void* __restrict__ C, int M, int N,
                                                 int K, int accum) {
  constexpr int NW = WM * WN;
  constexpr int TI = V2_BM / WM / 32, TJ = V2_BN / WN / 32;  // 32x32 MFMA tiles per wave along M / N
  constexpr int DPW = 32 / NW;                                 // 1-KiB DMA blocks per wave per operand
  // One static LDS object PER STAGE, each used with a compile-time identity (the K loop is unrolled by two):
  // the AMDGPU LDS lowering gives distinct objects distinct alias scopes, so hipcc can see that the DMA filling
  // one stage never feeds the ds_reads of the other and does not drain it (vmcnt(0)) before every K-step — which
  // it does for a single array indexed by a run-time stage number (checked in the .s).
  __shared__ __attribute__((aligned(1024))) uint8_t stage0[V2_STAGE];  // A 256x128 | B 256x128
  __shared__ __attribute__((aligned(1024))) uint8_t stage1[V2_STAGE];
  const int tiles_n = N / V2_BN;
  const int nwg = (M / V2_BM) * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = (bid / tiles_n) * V2_BM, tn = (bid % tiles_n) * V2_BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int wm = (wave / WN) * (V2_BM / WM), wn = (wave % WN) * (V2_BN / WN);

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // DMA assignment: each operand image is 256 rows = 32 blocks of 8 rows (1 KiB), DPW blocks per wave.
  // Lane l of an instruction covering rows [8b, 8b+8) writes LDS byte 16*l of that block, i.e. row 8b + l/8,
  // physical chunk l%8, which must hold logical chunk (l%8) ^ ((row>>1)&7).
  // Sources = wave-uniform tile base (SGPRs) + a 32-bit per-lane offset, identical for A and B (same K).
  const int lrow = lane >> 3, lpch = lane & 7;
  int voff[DPW];
#pragma unroll
  for (int t = 0; t < DPW; ++t) {
    const int row = (wave * DPW + t) * 8 + lrow;
    voff[t] = row * K + v2_swz(row, lpch) * 16;
  }
  const uint8_t* const a_tile = A + (long)tm * K;
  const uint8_t* const b_tile = B + (long)tn * K;
  auto stage = [&](int k0, uint8_t* base) {
    const uint8_t* a0 = a_tile + k0;
    const uint8_t* b0 = b_tile + k0;
#pragma unroll
    for (int t = 0; t < DPW; ++t) {
      const int blk = wave * DPW + t;  // 0..31
      __builtin_amdgcn_global_load_lds(a0 + voff[t], base + blk * 1024, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(b0 + voff[t], base + V2_BM * V2_BK + blk * 1024, 16, 0, 0);
    }
  };
  // Fragment rows are wm + 32 i + r (A) / wn + 32 j + r (B): the swizzle term (row >> 1) & 7 is (r >> 1) & 7 for
  // all of them, so each (ks, half) chunk has ONE per-lane offset and the fragment index is an immediate.
  const int sw = (r >> 1) & 7;
  int loff[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int p = 0; p < 2; ++p) loff[ks][p] = ((ks * 4 + 2 * hf + p) ^ sw) * 16;
  const int arow = (wm + r) * V2_BK, brow = V2_BM * V2_BK + (wn + r) * V2_BK;
  auto frag = [&](const uint8_t* img, int rowoff, int idx, int ks) -> v8i {
    const uint8_t* rp = img + rowoff + idx * 32 * V2_BK;
    const uint4 lo = *reinterpret_cast<const uint4*>(rp + loff[ks][0]);
    const uint4 hi = *reinterpret_cast<const uint4*>(rp + loff[ks][1]);
    v8i v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };

  auto compute = [&](const uint8_t* img) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // 8-wave layout (256 VGPRs per wave): keep each k-sub's fragment reads next to its MFMAs, hoisting the next
      // k-sub's reads would spill
      if (NW > 4) __builtin_amdgcn_sched_barrier(0);
      v8i af[TI], bfr[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = frag(img, brow, j, ks);
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = frag(img, arow, i, ks);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)  // swapped operands: acc holds the C^T tile (lane <-> m, registers <-> n)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bfr[j], af[i], acc[i][j], FB, FA, 0, 0x7f7f7f7f, 0,
                                                                      0x7f7f7f7f);
    }
  };
  auto retire = [&]() {  // this stage's DMA landed for every wave; every wave finished reading the other stage
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };

  const int nk = K / V2_BK;
  stage(0, stage0);
  retire();
  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    stage((kt + 1) * V2_BK, stage1);  // DMA of K-step kt+1 overlaps the MFMAs of kt
    compute(stage0);
    retire();
    if (kt + 2 < nk) stage((kt + 2) * V2_BK, stage0);
    compute(stage1);
    retire();
  }
  if (kt < nk) compute(stage0);  // odd number of K-steps: the last one was staged into stage0
  const float s = sa[0] * sb[0] * smul;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int m = tm + wm + i * 32 + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = tn + wn + j * 32 + 8 * g + 4 * hf;
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          v[t] = acc[i][j][4 * g + t] * s;
          if (bias != nullptr) v[t] += bf2f(bias[n + t]);
        }
        if (OUT_F32) {
          float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (long)m * N + n);
          if (accum) {
            const float4 o = *cp4;
            v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
          }
          *cp4 = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(C) + (long)m * N + n);
          if (accum) {
            const bf16x4 o = *cp4;
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] += bf2f(o.v[t]);
          }
          bf16x4 w;
#pragma unroll
          for (int t = 0; t < 4; ++t) w.v[t] = f2bf(v[t]);
          *cp4 = w;
        }
      }
    }
}

// 4 waves (one per SIMD, 128x128 per wave, 512-entry register file) and 8 waves (two per SIMD, 128x64 per wave).
template <int FA, int FB, bool OUT_F32>
__global__ __launch_bounds__(256, 1) void fp8_gemm_v2_w4_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                                const float* __restrict__ sa, const float* __restrict__ sb, float smul,
                                                                const bf16_t* __restrict__ bias, void* __restrict__ C, int M,
                                                                int N, int K, int accum) {
  fp8_gemm_v2_body<FA, FB, OUT_F32, 2, 2>(A, B, sa, sb, smul, bias, C, M, N, K, accum);
}

template <int FA, int FB, bool OUT_F32>
__global__ __launch_bounds__(512, 1) void fp8_gemm_v2_w8_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                                const float* __restrict__ sa, const float* __restrict__ sb, float smul,
                                                                const bf16_t* __restrict__ bias, void* __restrict__ C, int M,
                                                                int N, int K, int accum) {
  fp8_gemm_v2_body<FA, FB, OUT_F32, 2, 4>(A, B, sa, sb, smul, bias, C, M, N, K, accum);
}

// ------------------------------------------------------------------------------------------------ GEMM v3
// 256x256 output tile, 4 waves (2 x 2, one per SIMD: 128x128 per wave = 16 MX 32x32x64 accumulators in the 256
// AGPRs), BK = 64 fp8 bytes per K-tile (32 KiB of A+B), a FOUR-deep LDS ring filled by global_load_lds. Per K-tile t:
//   MFMAs on rows 0-63 of the wave's tile (fragments of t already in VGPRs)
//   s_waitcnt vmcnt(16)  -- only tile t+1 must have landed; t+2, t+3 stay in flight ACROSS the barrier
//   s_barrier            -- t+1 visible to every wave; every wave's reads of t retired (lgkmcnt(0) before it)
//   DMA of tile t+4 into t's slot and ds_reads of t+1's fragments into the second VGPR set, interleaved one DMA and
//   two ds_reads per MFMA with the MFMAs on rows 64-127
// so no K-tile starts with an exposed LDS-read latency or a drained DMA queue (v2's vmcnt(0) + barrier per K-step
// left the MFMA pipe idle for both at one wave per SIMD). Image rows are 64 B; the 16-B chunk swizzle
// c ^ ((row >> 2) & 3) makes every 16-lane ds_read_b128 group of a 32x32x64 fragment cover the 16 slots of a 256-B
// bank row.
constexpr int V3_BM = 256, V3_BN = 256, V3_BK = 64;
constexpr int V3_TILE = (V3_BM + V3_BN) * V3_BK;  // 32 KiB per K-tile: A 256x64 | B 256x64
constexpr int V3_BOFF = V3_BM * V3_BK;

__device__ __forceinline__ int v3_swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

// NW = 4: 2 x 2 waves of 128x128 (one per SIMD, accumulators in the 512-entry file); NW = 8: 2 x 4 waves of 128x64
// (two per SIMD, so one wave's DMA / LDS issue overlaps the other's MFMAs).
// vmcnt waits of the v3 ring (the count must be an immediate)
template <int N>
__device__ __forceinline__ void v3_wait() {
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 14) asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24) lgkmcnt(0)" ::: "memory");
  else static_assert(N < 0, "v3_wait: unsupported count");
}

// MX: the per-32-element e8m0 block scales of A [M, K/32] and B [N, K/32] (mx_quant's grouped layout, see below)
// feed the MFMA's own scale operands instead of unit scales; the per-tensor sa / sb are then unused.
template <int FA, int FB, bool OUT_F32, int NW, bool MX = false, bool UNSCALED = false>
__device__ __forceinline__ void fp8_gemm_v3_body(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                 const float* __restrict__ sa, const float* __restrict__ sb, float smul,
                                                 const bf16_t* __restrict__ bias, void* __restrict__ C, int M, int N,
                                                 int K, int accum, int group_m, const uint8_t* __restrict__ mxa = nullptr,
                                                 const uint8_t* __restrict__ mxb = nullptr) {
  // one LDS object per ring slot, each addressed with a compile-time identity (the loop is unrolled by the ring
  // depth): distinct objects carry distinct alias scopes, so hipcc does not drain the other slots' DMA (vmcnt(0))
  // before a slot's ds_reads
  __shared__ __attribute__((aligned(1024))) uint8_t ring0[V3_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring1[V3_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring2[V3_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring3[V3_TILE];
  constexpr int WN = NW / 2;                        // waves along N (2 along M)
  constexpr int TI = 4, TJ = 4 / (NW / 4);          // 32x32 tiles per wave along M / N
  constexpr int DPW = 16 / NW;                      // 1-KiB DMA blocks per wave per operand per K-tile
  constexpr int RD = 2 * (TI + TJ);                 // ds_read_b128 per wave per K-tile
  constexpr int HALF = 2 * TJ;                      // MFMAs per half K-tile
  const int tiles_n = N / V3_BN;
  const int nwg = (M / V3_BM) * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);  // each XCD gets a contiguous range of tile ids
  // tile id -> (row, col) in column-major groups of group_m tile rows: the ~32 tiles an XCD runs at once then cover
  // a group_m x (32 / group_m) block (A and B panels both re-read from that XCD's L2) instead of one row of 32
  // tiles, each with its own B panel
  int tile_m, tile_n;
  if (group_m > 1) {
    const int tiles_m = M / V3_BM, per_group = group_m * tiles_n;
    const int g = bid / per_group, first = g * group_m, rows = min(tiles_m - first, group_m), in = bid % per_group;
    tile_m = first + in % rows;
    tile_n = in / rows;
  } else {
    tile_m = bid / tiles_n;
    tile_n = bid % tiles_n;
  }
  const int tm = tile_m * V3_BM, tn = tile_n * V3_BN;
  // debug build: the tile and its K sweep stay inside A [M, K], B [N, K], C [M, N] (block-uniform)
  ACC_CHECK_OR_RETURN(tm + V3_BM <= M && tn + V3_BN <= N && K % 64 == 0 && bid < nwg, kChkGemmTile);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int wm = (wave / WN) * 128, wn = (wave % WN) * (V3_BN / WN);

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // DMA: each operand image is 256 rows x 64 B = 16 blocks of 16 rows (1 KiB), DPW per wave per operand. Lane l of a
  // block writes row 16 b + l / 4, physical chunk l % 4, which holds logical chunk (l % 4) ^ ((row >> 2) & 3).
  // buffer_load ... lds off one buffer descriptor per operand panel (SGPRs): the per-lane source offset is a
  // loop-invariant 32-bit VGPR and the K position rides in soffset, so staging costs no VALU address math (the
  // flat form needs a 64-bit VGPR address per instruction); out-of-range rows would read zeros, not fault.
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  unsigned voff[DPW];
#pragma unroll
  for (int t = 0; t < DPW; ++t) {
    const int row = (wv * DPW + t) * 16 + (lane >> 2);
    voff[t] = (unsigned)(row * K + v3_swz(row, lane & 3) * 16);
  }
  const auto a_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * K), (short)0, V3_BM * K, 0x00020000);
  const auto b_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * K), (short)0, V3_BN * K, 0x00020000);
  const int nk = K / V3_BK;
  // MX scales: lane (r, hf) of a 32x32x64 fragment holds K bytes 32 hf .. 32 hf + 31 of its row, i.e. exactly one
  // 32-element block, so its scale is one byte per fragment. mx_quant groups the scales of 4 K-tiles per row and half:
  // dword (row, g, hf) = the blocks 8 g + 2 q + hf, q = 0..3, one byte each — one buffer load per fragment row per 4
  // K-tiles (the ring loop's unroll), issued behind the DMA of step q = 0 and waited for with the ring's counts.
  constexpr int NS = MX ? TI + TJ : 0;  // scale loads per wave per 4 K-tiles
  const int kb = K / 32;
  unsigned sca[TI], scb[TJ], nsa[TI], nsb[TJ];
  const auto sa_rs = __builtin_amdgcn_make_buffer_rsrc(MX ? (void*)(mxa + (long)tm * kb) : (void*)A, (short)0, V3_BM * kb, 0x00020000);
  const auto sb_rs = __builtin_amdgcn_make_buffer_rsrc(MX ? (void*)(mxb + (long)tn * kb) : (void*)B, (short)0, V3_BN * kb, 0x00020000);
  const unsigned sv_a = (unsigned)((wm + r) * kb + hf * 4), sv_b = (unsigned)((wn + r) * kb + hf * 4);
  auto load_scales = [&](int g, unsigned (&la)[TI], unsigned (&lb)[TJ]) {
    if constexpr (MX) {
#pragma unroll
      for (int i = 0; i < TI; ++i) la[i] = __builtin_amdgcn_raw_buffer_load_b32(sa_rs, sv_a, i * 32 * kb + g * 8, 0);
#pragma unroll
      for (int j = 0; j < TJ; ++j) lb[j] = __builtin_amdgcn_raw_buffer_load_b32(sb_rs, sv_b, j * 32 * kb + g * 8, 0);
    }
  };
  // Past the last K-tile the DMA is still issued (so every wait below has ONE count and the loop body has no branch
  // for hipcc to sink the MFMAs across), but with an soffset beyond the descriptor: the hardware range check returns
  // zeros without touching memory, into a ring slot nobody reads again.
  auto stage = [&](int kt, uint8_t* base) {
    const int so = kt < nk ? kt * V3_BK : 0x40000000;
#pragma unroll
    for (int t = 0; t < DPW; ++t) {
      const int blk = wv * DPW + t;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rs, base + blk * 1024, 16, voff[t], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rs, base + V3_BOFF + blk * 1024, 16, voff[t], so, 0, 0);
    }
  };
  // fragment rows wm + 32 i + r / wn + 32 j + r all have (row >> 2) & 3 == (r >> 2) & 3
  const int sw = (r >> 2) & 3;
  // The MFMA's K order: lane (r, hf) supplies K 16 hf .. +15 in its first four registers and K 32 + 16 hf .. +15 in
  // the last four, and the block scale of lane (r, hf) covers K 32 hf .. 32 hf + 31. Reading the chunks hf and 2 + hf
  // keeps that K order equal to the memory order, so each 32-element memory block meets its own scale.
  const int lo0 = (hf ^ sw) * 16, lo1 = ((2 + hf) ^ sw) * 16;
  const int arow = (wm + r) * V3_BK, brow = V3_BOFF + (wn + r) * V3_BK;
  auto frag = [&](const uint8_t* p) -> v8i {
    const uint4 lo = *reinterpret_cast<const uint4*>(p + lo0);
    const uint4 hi = *reinterpret_cast<const uint4*>(p + lo1);
    v8i v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };
  auto load = [&](const uint8_t* img, v8i (&fa)[TI], v8i (&fb)[TJ]) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[j] = frag(img + brow + j * 32 * V3_BK);
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[i] = frag(img + arow + i * 32 * V3_BK);
  };
  auto mfma_rows = [&](const v8i (&fa)[TI], const v8i (&fb)[TJ], int i0, auto q) {
    constexpr int Q = decltype(q)::value;  // K-tile within the group of 4: byte Q of the scale dwords
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {  // swapped operands: acc holds the C^T tile (lane <-> m, registers <-> n)
        if constexpr (MX)  // op_sel picks byte Q of the scale dword in the MFMA itself (no VALU byte shifts)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fb[j], fa[i], acc[i][j], FB, FA, Q, (int)scb[j], Q,
                                                                      (int)sca[i]);
        else  // unit block scales; UNSCALED: scale operands 0 -> the plain v_mfma_f32_32x32x64_f8f6f4 (no ld_scale)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fb[j], fa[i], acc[i][j], FB, FA, 0,
                                                                      UNSCALED ? 0 : 0x7f7f7f7f, 0,
                                                                      UNSCALED ? 0 : 0x7f7f7f7f);
      }
  };

  // prologue: scales of K-tiles 0..3, tiles 0..3 in flight, wait for both and tile 0, read its fragments
  load_scales(0, sca, scb);
  __builtin_amdgcn_sched_barrier(0);  // the scale loads stay ahead of the DMA (their wait below is then free)
  stage(0, ring0);
  stage(1, ring1);
  stage(2, ring2);
  stage(3, ring3);
  if constexpr (NW == 4) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // 3 tiles x 2 DPW DMAs in flight
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (MX) {
    // consume the first scales here: a load still pending at the loop header (preheader path) would make hipcc wait
    // for it at the top of EVERY iteration, draining the DMA ring
#pragma unroll
    for (int i = 0; i < TI; ++i) asm volatile("" ::"v"(sca[i]));
#pragma unroll
    for (int j = 0; j < TJ; ++j) asm volatile("" ::"v"(scb[j]));
  }
  __builtin_amdgcn_sched_barrier(0);
  v8i xa[TI], xb[TJ], ya[TI], yb[TJ];
  load(ring0, xa, xb);

  // one K-tile: `cur` fragments (tile t, in VGPRs) -> MFMAs; `nxt` <- fragments of tile t+1 from slot `nslot`;
  // DMA of tile t+4 into `slot` (tile t's, free once every wave passed the barrier). Straight-line code only.
  const int ng = nk / 4;
  auto step = [&](int t, uint8_t* slot, const uint8_t* nslot, v8i (&ca)[TI], v8i (&cb)[TJ], v8i (&na)[TI], v8i (&nb)[TJ],
                  auto q) {
    constexpr int Q = decltype(q)::value;
    mfma_rows(ca, cb, 0, q);
    __builtin_amdgcn_sched_barrier(0);
    // tile t+1 landed (t+2, t+3 in flight). MX: the next group's scales, loaded behind tile t+4 - Q's DMA in step
    // Q = 0, stay in flight through Q = 1, 2 and have landed after the wait of Q = 3.
    constexpr int DMA2 = NW == 4 ? 16 : 8;  // two tiles' DMA
    v3_wait<(Q == 1 || Q == 2) ? DMA2 + NS : DMA2>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stage(t + 4, slot);
    if constexpr (Q == 0) load_scales(min(t / 4 + 1, ng - 1), nsa, nsb);  // the last group re-reads its own
    load(nslot, na, nb);  // past the last tile this reads a stale slot into registers nobody uses
    mfma_rows(ca, cb, 2, q);
    // issue order of this region: per MFMA one DMA and two fragment reads, so the reads of t+1 start right after the
    // barrier and their latency hides under this half's MFMAs (left alone, hipcc issues the MFMAs first)
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x10, 2 * DPW / HALF, 0);  // VMEM (buffer_load ... lds)
      __builtin_amdgcn_sched_group_barrier(0x100, RD / HALF, 0);      // DS read
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);                // MFMA
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;
  using Q2 = std::integral_constant<int, 2>;
  using Q3 = std::integral_constant<int, 3>;
  for (int t = 0; t < nk; t += 4) {  // nk % 4 == 0 (host check)
    step(t, ring0, ring1, xa, xb, ya, yb, Q0{});
    step(t + 1, ring1, ring2, ya, yb, xa, xb, Q1{});
    step(t + 2, ring2, ring3, xa, xb, ya, yb, Q2{});
    step(t + 3, ring3, ring0, ya, yb, xa, xb, Q3{});
    if constexpr (MX) {
#pragma unroll
      for (int i = 0; i < TI; ++i) sca[i] = nsa[i];
#pragma unroll
      for (int j = 0; j < TJ; ++j) scb[j] = nsb[j];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA left in flight past the loop

  const float s = MX ? smul : sa[0] * sb[0] * smul;
  // epilogue: bias / accumulate resolved once per kernel, not per element (per-element `if (bias)` became a branch
  // around every bias load)
  auto epilogue = [&](auto has_bias, auto acc_in) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int m = tm + wm + i * 32 + r;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = tn + wn + j * 32 + 8 * g + 4 * hf;
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = acc[i][j][4 * g + u] * s;
          if constexpr (decltype(has_bias)::value) {
            const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] += bf2f(b4.v[u]);
          }
          if constexpr (OUT_F32) {
            float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (long)m * N + n);
            if constexpr (decltype(acc_in)::value) {
              const float4 o = *cp4;
              v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
            }
            *cp4 = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(C) + (long)m * N + n);
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
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (bias != nullptr) {
    if (accum) epilogue(T_{}, T_{}); else epilogue(T_{}, F_{});
  } else {
    if (accum) epilogue(F_{}, T_{}); else epilogue(F_{}, F_{});
  }
}

template <int FA, int FB, bool OUT_F32, bool UNSCALED = false>
__global__ __launch_bounds__(256, 1) void fp8_gemm_v3_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                             const float* __restrict__ sa, const float* __restrict__ sb, float smul,
                                                             const bf16_t* __restrict__ bias, void* __restrict__ C, int M, int N,
                                                             int K, int accum, int group_m) {
  fp8_gemm_v3_body<FA, FB, OUT_F32, 4, false, UNSCALED>(A, B, sa, sb, smul, bias, C, M, N, K, accum, group_m);
}

// MXFP8 GEMM: v3 4-wave body with per-block e8m0 scales (xa: [M, K/32], xb: [N, K/32], grouped layout)
template <int FA, int FB, bool OUT_F32>
__global__ __launch_bounds__(256, 1) void mx_gemm_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                         const uint8_t* __restrict__ xa, const uint8_t* __restrict__ xb,
                                                         float smul, const bf16_t* __restrict__ bias, void* __restrict__ C,
                                                         int M, int N, int K, int accum, int group_m) {
  fp8_gemm_v3_body<FA, FB, OUT_F32, 4, true>(A, B, nullptr, nullptr, smul, bias, C, M, N, K, accum, group_m, xa, xb);
}

template <int FA, int FB, bool OUT_F32, bool UNSCALED = false>
__global__ __launch_bounds__(512, 1) void fp8_gemm_v3_w8_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                                const float* __restrict__ sa, const float* __restrict__ sb,
                                                                float smul, const bf16_t* __restrict__ bias, void* __restrict__ C,
                                                                int M, int N, int K, int accum, int group_m) {
  fp8_gemm_v3_body<FA, FB, OUT_F32, 8, false, UNSCALED>(A, B, sa, sb, smul, bias, C, M, N, K, accum, group_m);
}

// ------------------------------------------------------------------------------------------------ GEMM v6
// v3's tiling and 4-slot LDS ring (256x256, 4 waves of 128x128, 32x32x64 MFMA, BK 64) with the LDS-DMA issue spread
// over the whole K-tile. A buffer_load ... lds piece costs 60-185 issue cycles beside the MFMAs (MI355X constants), and
// v3 issued all 8 pieces of tile t+4 in the second half of tile t together with the 16 fragment reads of t+1: that half
// is issue-bound (8 x ~100 + 16 reads against 8 x 64 MFMA cycles) and the matrix pipe idles (PMC: 57 % MFMA busy vs
// hipBLASLt's 74 % at the same clock). Here tile t issues the pieces of tile t+3 into the slot tile t-1 left (free since
// the barrier of t-1): 4 with the first half's MFMAs, 4 with the second's. Two tiles stay in flight across each barrier.
template <int FA, int FB, bool OUT_F32, bool UNSCALED>
__global__ __launch_bounds__(256, 1) void fp8_gemm_v6_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                             const float* __restrict__ sa, const float* __restrict__ sb,
                                                             float smul, const bf16_t* __restrict__ bias, void* __restrict__ C,
                                                             int M, int N, int K, int accum, int group_m) {
  __shared__ __attribute__((aligned(1024))) uint8_t ring0[V3_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring1[V3_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring2[V3_TILE];
  __shared__ __attribute__((aligned(1024))) uint8_t ring3[V3_TILE];
  constexpr int TI = 4, TJ = 4, DPW = 4;
  const int tiles_n = N / V3_BN, tiles_m = M / V3_BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  int tile_m, tile_n;
  if (group_m > 1) {
    const int per_group = group_m * tiles_n;
    const int g = bid / per_group, first = g * group_m, rows = min(tiles_m - first, group_m), in = bid % per_group;
    tile_m = first + in % rows;
    tile_n = in / rows;
  } else {
    tile_m = bid / tiles_n;
    tile_n = bid % tiles_n;
  }
  const int tm = tile_m * V3_BM, tn = tile_n * V3_BN;
  ACC_CHECK_OR_RETURN(tm + V3_BM <= M && tn + V3_BN <= N && K % 256 == 0 && bid < nwg, kChkGemmTile);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;
  constexpr int SC = UNSCALED ? 0 : 0x7f7f7f7f;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int wv = __builtin_amdgcn_readfirstlane(wave);
  unsigned voff[DPW];
#pragma unroll
  for (int t = 0; t < DPW; ++t) {
    const int row = (wv * DPW + t) * 16 + (lane >> 2);
    voff[t] = (unsigned)(row * K + v3_swz(row, lane & 3) * 16);
  }
  const auto a_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * K), (short)0, V3_BM * K, 0x00020000);
  const auto b_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * K), (short)0, V3_BN * K, 0x00020000);
  const int nk = K / V3_BK;
  // half h of tile kt's pieces: A and B blocks 2h, 2h + 1 of this wave (zero-fill past the end, one count per wait)
  auto stage_half = [&](int kt, uint8_t* base, int h) {
    const int so = kt < nk ? kt * V3_BK : 0x40000000;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = 2 * h + u, blk = wv * DPW + t;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rs, base + blk * 1024, 16, voff[t], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rs, base + V3_BOFF + blk * 1024, 16, voff[t], so, 0, 0);
    }
  };
  const int sw = (r >> 2) & 3;
  const int lo0 = (hf ^ sw) * 16, lo1 = ((2 + hf) ^ sw) * 16;
  const int arow = (wm + r) * V3_BK, brow = V3_BOFF + (wn + r) * V3_BK;
  auto frag = [&](const uint8_t* p) -> v8i {
    const uint4 lo = *reinterpret_cast<const uint4*>(p + lo0);
    const uint4 hi = *reinterpret_cast<const uint4*>(p + lo1);
    v8i v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };
  auto load = [&](const uint8_t* img, v8i (&fa)[TI], v8i (&fb)[TJ]) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[j] = frag(img + brow + j * 32 * V3_BK);
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[i] = frag(img + arow + i * 32 * V3_BK);
  };
  auto mfma_rows = [&](const v8i (&fa)[TI], const v8i (&fb)[TJ], int i0) {
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fb[j], fa[i], acc[i][j], FB, FA, 0, SC, 0, SC);
  };

  // prologue: tiles 0..2 in flight, tile 0 landed, its fragments in registers
  stage_half(0, ring0, 0); stage_half(0, ring0, 1);
  stage_half(1, ring1, 0); stage_half(1, ring1, 1);
  stage_half(2, ring2, 0); stage_half(2, ring2, 1);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  v8i xa[TI], xb[TJ], ya[TI], yb[TJ];
  load(ring0, xa, xb);

  // tile t: `cur` fragments -> MFMAs; pieces of t+3 into `fill` (tile t-1's slot); fragments of t+1 from `nslot`
  auto step = [&](int t, const uint8_t* nslot, uint8_t* fill, v8i (&ca)[TI], v8i (&cb)[TJ], v8i (&na)[TI], v8i (&nb)[TJ]) {
    stage_half(t + 3, fill, 0);
    mfma_rows(ca, cb, 0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // one piece per two MFMAs
      __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");  // t+1 landed; t+2 and half of t+3 in flight
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stage_half(t + 3, fill, 1);
    load(nslot, na, nb);
    mfma_rows(ca, cb, 2);
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // per two MFMAs: one piece and four fragment reads
      __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int t = 0; t < nk; t += 4) {  // nk % 4 == 0 (host check)
    step(t, ring1, ring3, xa, xb, ya, yb);
    step(t + 1, ring2, ring0, ya, yb, xa, xb);
    step(t + 2, ring3, ring1, xa, xb, ya, yb);
    step(t + 3, ring0, ring2, ya, yb, xa, xb);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const float s = sa[0] * sb[0] * smul;
  auto epilogue = [&](auto has_bias, auto acc_in) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int m = tm + wm + i * 32 + r;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = tn + wn + j * 32 + 8 * g + 4 * hf;
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = acc[i][j][4 * g + u] * s;
          if constexpr (decltype(has_bias)::value) {
            const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] += bf2f(b4.v[u]);
          }
          if constexpr (OUT_F32) {
            float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (long)m * N + n);
            if constexpr (decltype(acc_in)::value) {
              const float4 o = *cp4;
              v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
            }
            *cp4 = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(C) + (long)m * N + n);
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
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (bias != nullptr) {
    if (accum) epilogue(T_{}, T_{}); else epilogue(T_{}, F_{});
  } else {
    if (accum) epilogue(F_{}, T_{}); else epilogue(F_{}, F_{});
  }
}

// ------------------------------------------------------------------------------------------------ GEMM v4
// 256x256 output tile, 4 waves (2 x 2, one per SIMD, 128x128 per wave), v_mfma 16x16x128 f8f6f4: 8 x 8 accumulator
// blocks of 4 registers (256 AGPR/VGPR). The 16x16 shape holds a higher clock under load than 32x32 at equal
// cycles per FLOP (MI355X DVFS give-back, item 7), and with unit block scales the scale operands can be dropped:
// UNSCALED passes scale 0, which hipcc lowers to the plain v_mfma_f32_16x16x128_f8f6f4 (no ld_scale prefix).
// BK = 128 fp8 bytes per K-step = one MFMA K. Two LDS slots of 64 KiB (A 256x128 | B 256x128) filled by
// buffer_load ... lds. Per K-step t (slot s = t % 2):
//   rows i = 0..5 of the wave's A blocks: A fragment i+1 read while the 8 MFMAs of row i run (B fragments of t are
//     already in registers)
//   vmcnt(0) + barrier: the DMA of t+1 (slot s^1, issued at the start of t) landed for every wave
//   rows i = 6, 7 + the B fragments and first A fragment of t+1 read from slot s^1 between their MFMAs
//   lgkmcnt(0) + barrier: every wave is done with slot s -> DMA of t+2 into slot s (interleaved with the next
//     step's first MFMAs)
// Image rows are 128 B; the 16-B chunk swizzle c ^ ((row >> 1) & 7) makes every 16-lane ds_read_b128 group of a
// 16x16x128 fragment read (lane (r, q): chunks q and q + 4 of row r) hit 16 distinct 16-B slots of the bank row.
constexpr int V4_BM = 256, V4_BN = 256, V4_BK = 128;
constexpr int V4_SLOT = (V4_BM + V4_BN) * V4_BK;  // 64 KiB
constexpr int V4_BOFF = V4_BM * V4_BK;

__device__ __forceinline__ int v4_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int FA, int FB, bool OUT_F32, bool UNSCALED>
__global__ __launch_bounds__(256, 1) void fp8_gemm_v4_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                             const float* __restrict__ sa, const float* __restrict__ sb,
                                                             float smul, const bf16_t* __restrict__ bias, void* __restrict__ C,
                                                             int M, int N, int K, int accum, int group_m) {
  __shared__ __attribute__((aligned(1024))) uint8_t slot0[V4_SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t slot1[V4_SLOT];
  const int tiles_n = N / V4_BN, tiles_m = M / V4_BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  int tile_m, tile_n;
  if (group_m > 1) {
    const int per_group = group_m * tiles_n;
    const int g = bid / per_group, first = g * group_m, rows = min(tiles_m - first, group_m), in = bid % per_group;
    tile_m = first + in % rows;
    tile_n = in / rows;
  } else {
    tile_m = bid / tiles_n;
    tile_n = bid % tiles_n;
  }
  const int tm = tile_m * V4_BM, tn = tile_n * V4_BN;
  ACC_CHECK_OR_RETURN(tm + V4_BM <= M && tn + V4_BN <= N && K % 256 == 0 && bid < nwg, kChkGemmTile);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r16 = lane & 15, q = lane >> 4;
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;
  constexpr int SC = UNSCALED ? 0 : 0x7f7f7f7f;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // DMA: each operand image = 32 blocks of 8 rows x 128 B (1 KiB); wave w fills blocks 8w .. 8w + 7 of both. Lane l
  // of a block writes row 8b + l / 8, physical chunk l % 8, which holds logical chunk (l % 8) ^ ((row >> 1) & 7).
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  unsigned voff[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int row = (wv * 8 + t) * 8 + (lane >> 3);
    voff[t] = (unsigned)(row * K + v4_swz(row, lane & 7) * 16);
  }
  const auto a_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * K), (short)0, V4_BM * K, 0x00020000);
  const auto b_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * K), (short)0, V4_BN * K, 0x00020000);
  const int nk = K / V4_BK;
  // past the last K-step the DMA still issues (one count for every wait) with an soffset beyond the descriptor: the
  // range check returns zeros into a slot nobody reads again
  auto stage = [&](int kt, uint8_t* base) {
    const int so = kt < nk ? kt * V4_BK : 0x40000000;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rs, base + (wv * 8 + t) * 1024, 16, voff[t], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rs, base + V4_BOFF + (wv * 8 + t) * 1024, 16, voff[t], so, 0, 0);
    }
  };
  // fragment rows (wm | wn) + 16 i + r16 share (row >> 1) & 7 == (r16 >> 1) & 7
  const int f = (r16 >> 1) & 7;
  const int lo = (q ^ f) * 16, hi = ((q + 4) ^ f) * 16;
  const int arow = (wm + r16) * V4_BK, brow = V4_BOFF + (wn + r16) * V4_BK;
  auto frag = [&](const uint8_t* p) -> v8i {
    const uint4 a = *reinterpret_cast<const uint4*>(p + lo);
    const uint4 b = *reinterpret_cast<const uint4*>(p + hi);
    v8i v;
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    return v;
  };
  auto mfma_row = [&](const v8i& af, const v8i (&bf)[8], int i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)  // swapped operands: acc holds C^T blocks (lane <-> m, registers <-> 4 n)
      acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af, acc[i][j], FB, FA, 0, SC, 0, SC);
  };

  stage(0, slot0);
  stage(1, slot1);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // slot 0 landed (this wave), slot 1 in flight
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  v8i bx[8], by[8], a0x, a0y;
#pragma unroll
  for (int j = 0; j < 8; ++j) bx[j] = frag(slot0 + brow + j * 16 * V4_BK);
  a0x = frag(slot0 + arow);

  // one K-step: `bc` / `a0c` = fragments of t (registers), `bn` / `a0n` <- fragments of t+1 from `nxt`
  auto step = [&](int t, uint8_t* cur, const uint8_t* nxt, v8i (&bc)[8], v8i (&bn)[8], v8i& a0c, v8i& a0n) {
    v8i ar[2];
    ar[0] = a0c;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      ar[(i + 1) & 1] = frag(cur + arow + (i + 1) * 16 * V4_BK);
      mfma_row(ar[i & 1], bc, i);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // t+1 landed (this wave's part)
    __builtin_amdgcn_s_barrier();                    // ... and every wave's
    __builtin_amdgcn_sched_barrier(0);
    ar[1] = frag(cur + arow + 7 * 16 * V4_BK);
#pragma unroll
    for (int j = 0; j < 8; ++j) bn[j] = frag(nxt + brow + j * 16 * V4_BK);
    a0n = frag(nxt + arow);
    mfma_row(ar[0], bc, 6);
    mfma_row(ar[1], bc, 7);
    // 16 MFMAs, 20 ds_reads: the reads of t+1 hide under this half's MFMAs
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);    // MFMA
    }
#pragma unroll
    for (int k = 4; k < 16; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of `cur` retired
    __builtin_amdgcn_s_barrier();                      // ... every wave's
    __builtin_amdgcn_sched_barrier(0);
    stage(t + 2, cur);
  };
  for (int t = 0; t < nk; t += 2) {  // nk even (host check: K % 256 == 0)
    step(t, slot0, slot1, bx, by, a0x, a0y);
    step(t + 1, slot1, slot0, by, bx, a0y, a0x);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-fill DMAs past the end retire before the exit

  const float s = sa[0] * sb[0] * smul;
  auto epilogue = [&](auto has_bias, auto acc_in) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = tm + wm + i * 16 + r16;
        const int n = tn + wn + j * 16 + 4 * q;
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = acc[i][j][u] * s;
        if constexpr (decltype(has_bias)::value) {
          const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] += bf2f(b4.v[u]);
        }
        if constexpr (OUT_F32) {
          float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (long)m * N + n);
          if constexpr (decltype(acc_in)::value) {
            const float4 o = *cp4;
            v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
          }
          *cp4 = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(C) + (long)m * N + n);
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
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (bias != nullptr) {
    if (accum) epilogue(T_{}, T_{}); else epilogue(T_{}, F_{});
  } else {
    if (accum) epilogue(F_{}, T_{}); else epilogue(F_{}, F_{});
  }
}

// ------------------------------------------------------------------------------------------------ GEMM v5
// v4's tiling (256x256, 4 waves of 128x128, 16x16x128 MFMA, BK 128, two 64 KiB slots) with ONE barrier per K-step and
// no register double buffer of the B fragments (v4's two B sets + prefetched A pushed hipcc into ~600 AGPR<->VGPR
// moves per loop trip). Per K-step t (slot s = t % 2):
//   DMA of t+1 into slot s^1 (free: every wave passed the barrier that ended t-1), interleaved with the first rows'
//     MFMAs;
//   B fragments of t (8 x 2 ds_read_b128) read at the step's start, A fragments streamed one row ahead;
//   vmcnt(0) + barrier at the end: t+1 landed for every wave, every wave is done reading slot s.
template <int FA, int FB, bool OUT_F32, bool UNSCALED>
__global__ __launch_bounds__(256, 1) void fp8_gemm_v5_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                             const float* __restrict__ sa, const float* __restrict__ sb,
                                                             float smul, const bf16_t* __restrict__ bias, void* __restrict__ C,
                                                             int M, int N, int K, int accum, int group_m) {
  __shared__ __attribute__((aligned(1024))) uint8_t slot0[V4_SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t slot1[V4_SLOT];
  const int tiles_n = N / V4_BN, tiles_m = M / V4_BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  int tile_m, tile_n;
  if (group_m > 1) {
    const int per_group = group_m * tiles_n;
    const int g = bid / per_group, first = g * group_m, rows = min(tiles_m - first, group_m), in = bid % per_group;
    tile_m = first + in % rows;
    tile_n = in / rows;
  } else {
    tile_m = bid / tiles_n;
    tile_n = bid % tiles_n;
  }
  const int tm = tile_m * V4_BM, tn = tile_n * V4_BN;
  ACC_CHECK_OR_RETURN(tm + V4_BM <= M && tn + V4_BN <= N && K % 256 == 0 && bid < nwg, kChkGemmTile);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r16 = lane & 15, q = lane >> 4;
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;
  constexpr int SC = UNSCALED ? 0 : 0x7f7f7f7f;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wv = __builtin_amdgcn_readfirstlane(wave);
  unsigned voff[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int row = (wv * 8 + t) * 8 + (lane >> 3);
    voff[t] = (unsigned)(row * K + v4_swz(row, lane & 7) * 16);
  }
  const auto a_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * K), (short)0, V4_BM * K, 0x00020000);
  const auto b_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * K), (short)0, V4_BN * K, 0x00020000);
  const int nk = K / V4_BK;
  auto stage = [&](int kt, uint8_t* base) {
    const int so = kt < nk ? kt * V4_BK : 0x40000000;  // past the end: zero-fill, one count for every wait
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rs, base + (wv * 8 + t) * 1024, 16, voff[t], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rs, base + V4_BOFF + (wv * 8 + t) * 1024, 16, voff[t], so, 0, 0);
    }
  };
  const int f = (r16 >> 1) & 7;
  const int lo = (q ^ f) * 16, hi = ((q + 4) ^ f) * 16;
  const int arow = (wm + r16) * V4_BK, brow = V4_BOFF + (wn + r16) * V4_BK;
  auto frag = [&](const uint8_t* p) -> v8i {
    const uint4 a = *reinterpret_cast<const uint4*>(p + lo);
    const uint4 b = *reinterpret_cast<const uint4*>(p + hi);
    v8i v;
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    return v;
  };

  stage(0, slot0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  auto step = [&](int t, const uint8_t* cur, uint8_t* nxt) {
    stage(t + 1, nxt);
    v8i bf[8], ar[2];
#pragma unroll
    for (int j = 0; j < 8; ++j) bf[j] = frag(cur + brow + j * 16 * V4_BK);
    ar[0] = frag(cur + arow);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i < 7) ar[(i + 1) & 1] = frag(cur + arow + (i + 1) * 16 * V4_BK);
#pragma unroll
      for (int j = 0; j < 8; ++j)  // swapped operands: acc holds C^T blocks (lane <-> m, registers <-> 4 n)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], ar[i & 1], acc[i][j], FB, FA, 0, SC, 0, SC);
    }
    // issue order: the B / first A fragment reads first, then one DMA of t+1 per MFMA of rows 0-1
    __builtin_amdgcn_sched_group_barrier(0x100, 18, 0);  // DS read
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);  // VMEM read (buffer_load ... lds)
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);   // MFMA
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // t+1 landed (this wave), slot reads retired
    __builtin_amdgcn_s_barrier();                               // ... every wave's
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int t = 0; t < nk; t += 2) {  // nk even (host check: K % 256 == 0)
    step(t, slot0, slot1);
    step(t + 1, slot1, slot0);
  }

  const float s = sa[0] * sb[0] * smul;
  auto epilogue = [&](auto has_bias, auto acc_in) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = tm + wm + i * 16 + r16;
        const int n = tn + wn + j * 16 + 4 * q;
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = acc[i][j][u] * s;
        if constexpr (decltype(has_bias)::value) {
          const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] += bf2f(b4.v[u]);
        }
        if constexpr (OUT_F32) {
          float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (long)m * N + n);
          if constexpr (decltype(acc_in)::value) {
            const float4 o = *cp4;
            v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
          }
          *cp4 = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(C) + (long)m * N + n);
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
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (bias != nullptr) {
    if (accum) epilogue(T_{}, T_{}); else epilogue(T_{}, F_{});
  } else {
    if (accum) epilogue(F_{}, T_{}); else epilogue(F_{}, F_{});
  }
}

// ------------------------------------------------------------------------------------------------ GEMM v7
// v5's tiling (256x256, 4 waves of 128x128, 16x16x128 MFMA, BK 128, two 64 KiB LDS slots) with the global -> LDS copy
// staged through registers instead of LDS-DMA. A 16x16x128 MFMA leaves a 32-cycle gap, of which the MFMA itself holds 8;
// a `buffer_load ... lds` costs ~60 cycles to issue among MFMAs (MI355X_MICROARCH cycle constants), so v4 / v5 paid
// ~30 cycles per DMA piece, 16 pieces per K-step; a buffer_load_dwordx4 (~8) or a ds_write_b128 (~13) fits in a gap.
// Measured the register-only MFMA loop: 16x16x128 4.7 PF/s vs 32x32x64 4.3 PF/s (tools/microbench/mfma_peak.hip).
// One K-step per loop trip (t, slot s = t % 2; `cur` / `nxt` are __restrict__ so the waitcnt pass does not make the
// reads of `cur` wait for the writes into `nxt`), the instruction order pinned by sched_barrier after every MFMA:
//   B fragments of t + A fragment of row 0 (18 ds_read_b128) from slot s
//   row i = 0..7: 8 MFMAs, in their gaps: the A fragment of row i+1 (2 ds_read_b128), the staged 1 KiB chunks i of
//     tile t+1 (A and B; loaded one step earlier) written into slot s^1 (2 ds_write_b128; slot s^1 was released by
//     the barrier that ended t-1), and chunk i of tile t+2 loaded into the freed staging registers (2 buffer loads,
//     out-of-range soffset past the last tile: zeros, never stored anywhere read)
//   lgkmcnt(0) + barrier: tile t+1 is in slot s^1 for every wave, every wave is done with slot s
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int FA, int FB, bool OUT_F32, bool UNSCALED>
__global__ __launch_bounds__(256, 1) void fp8_gemm_v7_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                             const float* __restrict__ sa, const float* __restrict__ sb,
                                                             float smul, const bf16_t* __restrict__ bias, void* __restrict__ C,
                                                             int M, int N, int K, int accum, int group_m) {
  __shared__ __attribute__((aligned(1024))) uint8_t slot0[V4_SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t slot1[V4_SLOT];
  const int tiles_n = N / V4_BN, tiles_m = M / V4_BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  int tile_m, tile_n;
  if (group_m > 1) {
    const int per_group = group_m * tiles_n;
    const int g = bid / per_group, first = g * group_m, rows = min(tiles_m - first, group_m), in = bid % per_group;
    tile_m = first + in % rows;
    tile_n = in / rows;
  } else {
    tile_m = bid / tiles_n;
    tile_n = bid % tiles_n;
  }
  const int tm = tile_m * V4_BM, tn = tile_n * V4_BN;
  ACC_CHECK_OR_RETURN(tm + V4_BM <= M && tn + V4_BN <= N && K % V4_BK == 0 && bid < nwg, kChkGemmTile);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r16 = lane & 15, q = lane >> 4;
  const int wm = (wave >> 1) * 128, wn = (wave & 1) * 128;
  constexpr int SC = UNSCALED ? 0 : 0x7f7f7f7f;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // copy: each operand image = 32 blocks of 8 rows x 128 B (1 KiB); wave w moves blocks 8w .. 8w + 7 of both. Lane l of
  // a block reads row 8b + l / 8, logical chunk (l % 8) ^ ((row >> 1) & 7), and writes it at l * 16 in the block
  // (the same swizzled image as v4 / v5)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  unsigned voff[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int row = (wv * 8 + c) * 8 + (lane >> 3);
    voff[c] = (unsigned)(row * K + v4_swz(row, lane & 7) * 16);
  }
  const int woff = wv * 8 * 1024 + lane * 16;
  const auto a_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * K), (short)0, V4_BM * K, 0x00020000);
  const auto b_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * K), (short)0, V4_BN * K, 0x00020000);
  const int nk = K / V4_BK;
  auto soff = [&](int kt) { return kt < nk ? kt * V4_BK : 0x40000000; };
  u32x4 stA[8], stB[8];

  const int f = (r16 >> 1) & 7;
  const int lo = (q ^ f) * 16, hi = ((q + 4) ^ f) * 16;
  const int arow = (wm + r16) * V4_BK, brow = V4_BOFF + (wn + r16) * V4_BK;

  // prologue: tile 0 -> slot 0 through the registers, tile 1 -> registers
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    stA[c] = __builtin_amdgcn_raw_buffer_load_b128(a_rs, voff[c], soff(0), 0);
    stB[c] = __builtin_amdgcn_raw_buffer_load_b128(b_rs, voff[c], soff(0), 0);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    *reinterpret_cast<u32x4*>(slot0 + woff + c * 1024) = stA[c];
    *reinterpret_cast<u32x4*>(slot0 + V4_BOFF + woff + c * 1024) = stB[c];
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    stA[c] = __builtin_amdgcn_raw_buffer_load_b128(a_rs, voff[c], soff(1), 0);
    stB[c] = __builtin_amdgcn_raw_buffer_load_b128(b_rs, voff[c], soff(1), 0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  auto step = [&](int t, const uint8_t* __restrict__ cur, uint8_t* __restrict__ nxt) {
    v8i bf[8];
    uint4 alo[2], ahi[2];
    alo[0] = *reinterpret_cast<const uint4*>(cur + arow + lo);
    ahi[0] = *reinterpret_cast<const uint4*>(cur + arow + hi);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4 x = *reinterpret_cast<const uint4*>(cur + brow + j * 16 * V4_BK + lo);
      const uint4 y = *reinterpret_cast<const uint4*>(cur + brow + j * 16 * V4_BK + hi);
      bf[j][0] = x.x; bf[j][1] = x.y; bf[j][2] = x.z; bf[j][3] = x.w;
      bf[j][4] = y.x; bf[j][5] = y.y; bf[j][6] = y.z; bf[j][7] = y.w;
    }
    __builtin_amdgcn_sched_barrier(0);
    const int so2 = soff(t + 2);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ca = i & 1, nb = (i + 1) & 1;
      v8i af;
      af[0] = alo[ca].x; af[1] = alo[ca].y; af[2] = alo[ca].z; af[3] = alo[ca].w;
      af[4] = ahi[ca].x; af[5] = ahi[ca].y; af[6] = ahi[ca].z; af[7] = ahi[ca].w;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // swapped operands: acc holds C^T blocks (lane <-> m, registers <-> 4 n)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af, acc[i][j], FB, FA, 0, SC, 0, SC);
        if (j == 0 && i < 7) alo[nb] = *reinterpret_cast<const uint4*>(cur + arow + (i + 1) * 16 * V4_BK + lo);
        if (j == 1 && i < 7) ahi[nb] = *reinterpret_cast<const uint4*>(cur + arow + (i + 1) * 16 * V4_BK + hi);
        if (j == 2) *reinterpret_cast<u32x4*>(nxt + woff + i * 1024) = stA[i];
        if (j == 3) *reinterpret_cast<u32x4*>(nxt + V4_BOFF + woff + i * 1024) = stB[i];
        if (j == 4) stA[i] = __builtin_amdgcn_raw_buffer_load_b128(a_rs, voff[i], so2, 0);
        if (j == 5) stB[i] = __builtin_amdgcn_raw_buffer_load_b128(b_rs, voff[i], so2, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's writes of t+1 and reads of t retired
    __builtin_amdgcn_s_barrier();                      // ... every wave's
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int t = 0; t < nk; ++t) {
    const bool odd = t & 1;
    step(t, odd ? slot1 : slot0, odd ? slot0 : slot1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-filled loads past the end retire before the exit

  const float s = sa[0] * sb[0] * smul;
  auto epilogue = [&](auto has_bias, auto acc_in) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = tm + wm + i * 16 + r16;
        const int n = tn + wn + j * 16 + 4 * q;
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = acc[i][j][u] * s;
        if constexpr (decltype(has_bias)::value) {
          const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] += bf2f(b4.v[u]);
        }
        if constexpr (OUT_F32) {
          float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (long)m * N + n);
          if constexpr (decltype(acc_in)::value) {
            const float4 o = *cp4;
            v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
          }
          *cp4 = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(C) + (long)m * N + n);
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
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (bias != nullptr) {
    if (accum) epilogue(T_{}, T_{}); else epilogue(T_{}, F_{});
  } else {
    if (accum) epilogue(F_{}, T_{}); else epilogue(F_{}, F_{});
  }
}

// ------------------------------------------------------------------------------------------------ GEMM v8
// v7's tile, slots and register-staged copy with 8 waves in two groups of 4 (one wave of each group per SIMD) that
// run a barrier-staggered ping-pong (the 8-phase structure of cdna_hip_programming.md §5): group g = wave / 4 owns
// output rows 128 g .. +127, wave w % 4 of it columns 64 (w % 4) .. +63 (8 x 4 blocks of 16x16 = 128 accumulator
// registers). Each K-step is two phases per wave, each a MEMORY half (fragment reads, the staged chunks of tile t+1
// written into the other slot, loads of tile t+2 into the freed registers, lgkmcnt(0)) and a COMPUTE half (16 MFMAs
// under s_setprio 1), separated by s_barrier. Group 1 passes one extra barrier first, so between two barriers one group
// computes while the other does its memory half: each group's LDS latency and waits hide under the other's MFMAs.
// Ordering (regions between consecutive barriers; group 1 lags group 0 by one region): the slot a memory half writes
// (tile t+1) was last read for tile t-1 at least one barrier earlier by both groups, and the slot it reads (tile t)
// was completed, lgkmcnt(0) included, by both groups' memory halves of step t-1 before the barrier that precedes it.
template <int FA, int FB, bool OUT_F32, bool UNSCALED>
__global__ __launch_bounds__(512, 1) void fp8_gemm_v8_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                             const float* __restrict__ sa, const float* __restrict__ sb,
                                                             float smul, const bf16_t* __restrict__ bias, void* __restrict__ C,
                                                             int M, int N, int K, int accum, int group_m) {
  __shared__ __attribute__((aligned(1024))) uint8_t slot0[V4_SLOT];
  __shared__ __attribute__((aligned(1024))) uint8_t slot1[V4_SLOT];
  const int tiles_n = N / V4_BN, tiles_m = M / V4_BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  int tile_m, tile_n;
  if (group_m > 1) {
    const int per_group = group_m * tiles_n;
    const int g = bid / per_group, first = g * group_m, rows = min(tiles_m - first, group_m), in = bid % per_group;
    tile_m = first + in % rows;
    tile_n = in / rows;
  } else {
    tile_m = bid / tiles_n;
    tile_n = bid % tiles_n;
  }
  const int tm = tile_m * V4_BM, tn = tile_n * V4_BN;
  ACC_CHECK_OR_RETURN(tm + V4_BM <= M && tn + V4_BN <= N && K % V4_BK == 0 && bid < nwg, kChkGemmTile);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r16 = lane & 15, q = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int grp = wv >> 2;  // wave-uniform and provably so: the stagger barrier below is a scalar branch
  const int wm = grp * 128, wn = (wv & 3) * 64;
  constexpr int SC = UNSCALED ? 0 : 0x7f7f7f7f;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // copy: 32 A and 32 B blocks of 8 rows x 128 B per K-tile; wave w moves A blocks 4w .. 4w + 3 and B blocks 4w ..
  // 4w + 3 (the v4 image: lane l of a block reads logical chunk (l % 8) ^ ((row >> 1) & 7) of row 8b + l / 8 and
  // writes it at l * 16)
  unsigned voff[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int row = (wv * 4 + c) * 8 + (lane >> 3);
    voff[c] = (unsigned)(row * K + v4_swz(row, lane & 7) * 16);
  }
  const int woff = wv * 4 * 1024 + lane * 16;
  const auto a_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long)tm * K), (short)0, V4_BM * K, 0x00020000);
  const auto b_rs = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (long)tn * K), (short)0, V4_BN * K, 0x00020000);
  const int nk = K / V4_BK;
  auto soff = [&](int kt) { return kt < nk ? kt * V4_BK : 0x40000000; };
  u32x4 stA[4], stB[4];

  const int f = (r16 >> 1) & 7;
  const int lo = (q ^ f) * 16, hi = ((q + 4) ^ f) * 16;
  const int arow = (wm + r16) * V4_BK, brow = V4_BOFF + (wn + r16) * V4_BK;
  auto frag = [&](const uint8_t* p) -> v8i {
    const uint4 x = *reinterpret_cast<const uint4*>(p + lo);
    const uint4 y = *reinterpret_cast<const uint4*>(p + hi);
    v8i v;
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    return v;
  };

  // prologue: tile 0 -> slot 0 through the registers, tile 1 -> registers
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    stA[c] = __builtin_amdgcn_raw_buffer_load_b128(a_rs, voff[c], soff(0), 0);
    stB[c] = __builtin_amdgcn_raw_buffer_load_b128(b_rs, voff[c], soff(0), 0);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    *reinterpret_cast<u32x4*>(slot0 + woff + c * 1024) = stA[c];
    *reinterpret_cast<u32x4*>(slot0 + V4_BOFF + woff + c * 1024) = stB[c];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    stA[c] = __builtin_amdgcn_raw_buffer_load_b128(a_rs, voff[c], soff(1), 0);
    stB[c] = __builtin_amdgcn_raw_buffer_load_b128(b_rs, voff[c], soff(1), 0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger
  __builtin_amdgcn_sched_barrier(0);

  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto step = [&](int t, const uint8_t* __restrict__ cur, uint8_t* __restrict__ nxt) {
    const int so2 = soff(t + 2);
    v8i bf[4], af[4];
    // memory half 0: B fragments + A rows 0-3 of tile t; A chunks of tile t+1 -> nxt; A chunks of t+2 -> registers
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = frag(cur + brow + j * 16 * V4_BK);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(cur + arow + i * 16 * V4_BK);
#pragma unroll
    for (int c = 0; c < 4; ++c) *reinterpret_cast<u32x4*>(nxt + woff + c * 1024) = stA[c];
#pragma unroll
    for (int c = 0; c < 4; ++c) stA[c] = __builtin_amdgcn_raw_buffer_load_b128(a_rs, voff[c], so2, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)  // swapped operands: acc holds C^T blocks (lane <-> m, registers <-> 4 n)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af[i], acc[i][j], FB, FA, 0, SC, 0, SC);
    __builtin_amdgcn_s_setprio(0);
    sync();
    // memory half 1: A rows 4-7; B chunks of t+1 -> nxt; B chunks of t+2 -> registers
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(cur + arow + (i + 4) * 16 * V4_BK);
#pragma unroll
    for (int c = 0; c < 4; ++c) *reinterpret_cast<u32x4*>(nxt + V4_BOFF + woff + c * 1024) = stB[c];
#pragma unroll
    for (int c = 0; c < 4; ++c) stB[c] = __builtin_amdgcn_raw_buffer_load_b128(b_rs, voff[c], so2, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i + 4][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af[i], acc[i + 4][j], FB, FA, 0, SC, 0, SC);
    __builtin_amdgcn_s_setprio(0);
    sync();
  };
  for (int t = 0; t < nk; ++t) {
    const bool odd = t & 1;
    step(t, odd ? slot1 : slot0, odd ? slot0 : slot1);
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // equal barrier counts for both groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-filled loads past the end retire before the exit

  const float s = sa[0] * sb[0] * smul;
  auto epilogue = [&](auto has_bias, auto acc_in) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = tm + wm + i * 16 + r16;
        const int n = tn + wn + j * 16 + 4 * q;
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = acc[i][j][u] * s;
        if constexpr (decltype(has_bias)::value) {
          const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] += bf2f(b4.v[u]);
        }
        if constexpr (OUT_F32) {
          float4* cp4 = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (long)m * N + n);
          if constexpr (decltype(acc_in)::value) {
            const float4 o = *cp4;
            v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
          }
          *cp4 = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          bf16x4* cp4 = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(C) + (long)m * N + n);
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
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (bias != nullptr) {
    if (accum) epilogue(T_{}, T_{}); else epilogue(T_{}, F_{});
  } else {
    if (accum) epilogue(F_{}, T_{}); else epilogue(F_{}, F_{});
  }
}

}  // namespace

ACC_DEBUG_TAKE_FN(acc_dbg_take_fp8)

torch::Tensor fp8_amax(torch::Tensor x, c10::optional<torch::Tensor> out) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "fp8_amax: x must be contiguous bf16");
  torch::Tensor o = out.has_value() ? *out : torch::empty({1}, x.options().dtype(torch::kFloat32));
  auto stream = at::hip::getCurrentHIPStream();
  hipMemsetAsync(o.data_ptr(), 0, sizeof(float), stream);
  const long n = x.numel();
  if (n == 0) return o;
  // at most one 1024-thread workgroup per CU: every workgroup ends in one same-address atomic max, and 2048 of them
  // (the old 256-thread grid) queued ~40 us of serialised atomics behind a ~12 us stream of a 64 MB activation
  long g = (n / 8 + 1023) / 1024;
  g = std::max<long>(1, std::min<long>(g, 256));
  hipLaunchKernelGGL(amax_kernel, dim3(g), dim3(1024), 0, stream, reinterpret_cast<const bf16_t*>(x.data_ptr()), n,
                     reinterpret_cast<unsigned int*>(o.data_ptr()));
  return o;
}


// Per-segment amax of a flat bf16 shard: out[k] = max |x[lo[k]:hi[k]]| (0 for empty segments). lo/hi: int64 device;
// max_len: the longest segment (sizes the grid; every segment must be no longer).
void fp8_segment_amax(torch::Tensor x, torch::Tensor lo, torch::Tensor hi, torch::Tensor out, int64_t max_len) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "fp8_segment_amax: contiguous bf16 x");
  TORCH_CHECK(lo.scalar_type() == at::kLong && hi.scalar_type() == at::kLong && lo.numel() == hi.numel() &&
              out.scalar_type() == at::kFloat && out.numel() == lo.numel(), "fp8_segment_amax: bad segment tensors");
  auto stream = at::hip::getCurrentHIPStream();
  hipMemsetAsync(out.data_ptr(), 0, out.numel() * sizeof(float), stream);
  const long nseg = lo.numel();
  if (nseg == 0 || x.numel() == 0) return;
  TORCH_CHECK(max_len >= 0 && max_len <= x.numel(), "fp8_segment_amax: max_len");
  const long chunks = std::max<long>(1, (max_len + kSegChunk - 1) / kSegChunk);  // chunks of the longest segment
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "fp8_segment_amax: x must be 16-B aligned");
  hipLaunchKernelGGL(seg_amax_kernel, dim3(chunks, nseg), dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(x.data_ptr()),
                     lo.data_ptr<long>(), hi.data_ptr<long>(), reinterpret_cast<unsigned int*>(out.data_ptr()));
}

// y[lo[k]:hi[k]] = e4m3(x * qmax / amax[k]) segment by segment (y: fp8 e4m3 flat buffer of x's size).
void fp8_segment_cast(torch::Tensor x, torch::Tensor lo, torch::Tensor hi, torch::Tensor amax, double qmax, torch::Tensor y,
                      int64_t max_len) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "fp8_segment_cast: contiguous bf16 x");
  TORCH_CHECK(y.scalar_type() == at::kFloat8_e4m3fn && y.is_contiguous() && y.numel() == x.numel(), "fp8_segment_cast: y");
  TORCH_CHECK(amax.scalar_type() == at::kFloat && amax.numel() == lo.numel(), "fp8_segment_cast: amax");
  const long nseg = lo.numel();
  if (nseg == 0 || x.numel() == 0) return;
  TORCH_CHECK(max_len >= 0 && max_len <= x.numel(), "fp8_segment_cast: max_len");
  const long chunks = std::max<long>(1, (max_len + kSegChunk - 1) / kSegChunk);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0,
              "fp8_segment_cast: x / y alignment");
  hipLaunchKernelGGL(seg_cast_kernel, dim3(chunks, nseg), dim3(256), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16_t*>(x.data_ptr()), lo.data_ptr<long>(), hi.data_ptr<long>(),
                     amax.data_ptr<float>(), (float)qmax, reinterpret_cast<uint8_t*>(y.data_ptr()));
}

// x^T of a 2-D one-byte tensor (fp8 / uint8), or of every matrix of a 3-D [E, R, C] one.
torch::Tensor u8_transpose(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && (x.dim() == 2 || x.dim() == 3) && x.is_contiguous() && x.element_size() == 1,
              "u8_transpose: 2-D / 3-D contiguous byte tensor");
  const int E = x.dim() == 3 ? x.size(0) : 1, R = x.size(-2), C = x.size(-1);
  auto y = x.dim() == 3 ? torch::empty({E, C, R}, x.options()) : torch::empty({C, R}, x.options());
  if (x.numel() == 0) return y;
  dim3 grid((C + kCT - 1) / kCT, (R + kCT - 1) / kCT, E);
  hipLaunchKernelGGL(u8_transpose_kernel, grid, dim3(256), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const uint8_t*>(x.data_ptr()), reinterpret_cast<uint8_t*>(y.data_ptr()), R, C);
  return y;
}

// MXFP8 quantisation (see mx_quant_kernel): returns {q, s} or, with `colwise`, {q, s, qt, st}. q / qt: fp8
// (e4m3fn, or e5m2), s / st: uint8 e8m0 block scales in the grouped layout. C % 256 == 0 (and R % 256 == 0 with
// colwise) so that every row holds whole scale groups.
std::vector<torch::Tensor> mx_quant(torch::Tensor x, bool e5m2, bool colwise) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 2, "mx_quant: 2-D contiguous bf16");
  const int R = x.size(0), C = x.size(1);
  TORCH_CHECK(R % kMxT == 0 && C % 256 == 0 && (!colwise || R % 256 == 0),
              "mx_quant: rows must be a multiple of 64 (256 with colwise) and columns of 256");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "mx_quant: x must be 16-B aligned");
  auto dt = e5m2 ? at::kFloat8_e5m2 : at::kFloat8_e4m3fn;
  auto q = torch::empty({R, C}, x.options().dtype(dt));
  auto s = torch::empty({R, C / 32}, x.options().dtype(torch::kUInt8));
  torch::Tensor qt, st;
  if (colwise) {
    qt = torch::empty({C, R}, x.options().dtype(dt));
    st = torch::empty({C, R / 32}, x.options().dtype(torch::kUInt8));
  }
  if (R > 0 && C > 0) {
    dim3 grid(C / kMxT, R / kMxT);
    auto stream = at::hip::getCurrentHIPStream();
    const bf16_t* xp = reinterpret_cast<const bf16_t*>(x.data_ptr());
    uint8_t* qp = reinterpret_cast<uint8_t*>(q.data_ptr());
    uint8_t* sp = s.data_ptr<uint8_t>();
    uint8_t* qtp = colwise ? reinterpret_cast<uint8_t*>(qt.data_ptr()) : nullptr;
    uint8_t* stp = colwise ? st.data_ptr<uint8_t>() : nullptr;
#define MXQ(E, CW) hipLaunchKernelGGL((mx_quant_kernel<E, CW>), grid, dim3(256), 0, stream, xp, R, C, qp, sp, qtp, stp)
    if (e5m2) { if (colwise) MXQ(true, true); else MXQ(true, false); }
    else { if (colwise) MXQ(false, true); else MXQ(false, false); }
#undef MXQ
  }
  if (colwise) return {q, s, qt, st};
  return {q, s};
}

// scale = from_amax ? qmax / max(t, 1e-12) : t * qmax, read on the device (t: fp32 [1]).
std::vector<torch::Tensor> fp8_cast(torch::Tensor x, torch::Tensor t, double qmax, bool from_amax, bool e5m2, bool transpose) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 2, "fp8_cast: x must be 2-D contiguous bf16");
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.numel() >= 1, "fp8_cast: scale/amax must be a fp32 device tensor");
  const int M = x.size(0), N = x.size(1);
  auto dt = e5m2 ? at::kFloat8_e5m2 : at::kFloat8_e4m3fn;
  auto y = torch::empty({M, N}, x.options().dtype(dt));
  torch::Tensor yt;
  if (transpose) yt = torch::empty({N, M}, x.options().dtype(dt));
  if (M == 0 || N == 0) return transpose ? std::vector<torch::Tensor>{y, yt} : std::vector<torch::Tensor>{y};
  dim3 grid((N + kCT - 1) / kCT, (M + kCT - 1) / kCT);
  auto stream = at::hip::getCurrentHIPStream();
  uint8_t* yp = reinterpret_cast<uint8_t*>(y.data_ptr());
  uint8_t* ytp = transpose ? reinterpret_cast<uint8_t*>(yt.data_ptr()) : nullptr;
  const bf16_t* xp = reinterpret_cast<const bf16_t*>(x.data_ptr());
  const float* tp = t.data_ptr<float>();
  const float q = (float)qmax;
  const int fa = from_amax ? 1 : 0;
  if (e5m2) {
    if (transpose) hipLaunchKernelGGL((cast_kernel<true, true>), grid, dim3(256), 0, stream, xp, tp, q, fa, yp, ytp, M, N);
    else hipLaunchKernelGGL((cast_kernel<true, false>), grid, dim3(256), 0, stream, xp, tp, q, fa, yp, ytp, M, N);
  } else {
    if (transpose) hipLaunchKernelGGL((cast_kernel<false, true>), grid, dim3(256), 0, stream, xp, tp, q, fa, yp, ytp, M, N);
    else hipLaunchKernelGGL((cast_kernel<false, false>), grid, dim3(256), 0, stream, xp, tp, q, fa, yp, ytp, M, N);
  }
  if (transpose) return {y, yt};
  return {y};
}

// fp8_cast into caller-owned outputs: y [M, N] and (optionally) yt [N, M], both 1-byte fp8 of the matching kind. Used
// for the world-size-1 FSDP fp8 weights: one pass writes the persistent e4m3 weight and its K-major copy for dgrad.
void fp8_cast_into(torch::Tensor x, torch::Tensor t, double qmax, bool from_amax, bool e5m2, torch::Tensor y,
                   c10::optional<torch::Tensor> yt) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 2, "fp8_cast_into: x must be 2-D contiguous bf16");
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.numel() >= 1, "fp8_cast_into: scale/amax must be a fp32 device tensor");
  const int M = x.size(0), N = x.size(1);
  TORCH_CHECK(y.is_cuda() && y.element_size() == 1 && y.is_contiguous() && y.numel() == (long)M * N, "fp8_cast_into: bad y");
  const bool tr = yt.has_value();
  if (tr) TORCH_CHECK(yt->is_cuda() && yt->element_size() == 1 && yt->is_contiguous() && yt->numel() == (long)M * N, "fp8_cast_into: bad yt");
  if (M == 0 || N == 0) return;
  dim3 grid((N + kCT - 1) / kCT, (M + kCT - 1) / kCT);
  auto stream = at::hip::getCurrentHIPStream();
  uint8_t* yp = reinterpret_cast<uint8_t*>(y.data_ptr());
  uint8_t* ytp = tr ? reinterpret_cast<uint8_t*>(yt->data_ptr()) : nullptr;
  const bf16_t* xp = reinterpret_cast<const bf16_t*>(x.data_ptr());
  const float* tp = t.data_ptr<float>();
  const float q = (float)qmax;
  const int fa = from_amax ? 1 : 0;
  if (e5m2) {
    if (tr) hipLaunchKernelGGL((cast_kernel<true, true>), grid, dim3(256), 0, stream, xp, tp, q, fa, yp, ytp, M, N);
    else hipLaunchKernelGGL((cast_kernel<true, false>), grid, dim3(256), 0, stream, xp, tp, q, fa, yp, ytp, M, N);
  } else {
    if (tr) hipLaunchKernelGGL((cast_kernel<false, true>), grid, dim3(256), 0, stream, xp, tp, q, fa, yp, ytp, M, N);
    else hipLaunchKernelGGL((cast_kernel<false, false>), grid, dim3(256), 0, stream, xp, tp, q, fa, yp, ytp, M, N);
  }
}

// Per-matrix e4m3 cast of a [E, M, N] bf16 stack with one amax per matrix (scale 448 / amax[e], the conversion of
// seg_cast_kernel) into y [E, M, N] and its per-matrix transpose yt [E, N, M], one launch: the MoE expert weights'
// e4m3 copies and their K-major dgrad operands in one pass (no separate byte transpose re-reading y).
void fp8_cast_batched_into(torch::Tensor x, torch::Tensor amax, double qmax, torch::Tensor y, torch::Tensor yt) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 3,
              "fp8_cast_batched_into: x must be a 3-D contiguous bf16 stack");
  const int E = x.size(0), M = x.size(1), N = x.size(2);
  TORCH_CHECK(amax.is_cuda() && amax.scalar_type() == at::kFloat && amax.is_contiguous() && amax.numel() == E,
              "fp8_cast_batched_into: amax must be fp32 [E]");
  TORCH_CHECK(y.is_cuda() && y.element_size() == 1 && y.is_contiguous() && y.numel() == (long)E * M * N &&
                  yt.is_cuda() && yt.element_size() == 1 && yt.is_contiguous() && yt.numel() == (long)E * M * N,
              "fp8_cast_batched_into: bad y / yt");
  if (E == 0 || M == 0 || N == 0) return;
  TORCH_CHECK(E <= 65535, "fp8_cast_batched_into: too many matrices");
  dim3 grid((N + kCT - 1) / kCT, (M + kCT - 1) / kCT, E);
  hipLaunchKernelGGL((cast_kernel<false, true>), grid, dim3(256), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16_t*>(x.data_ptr()), amax.data_ptr<float>(), (float)qmax, 1,
                     reinterpret_cast<uint8_t*>(y.data_ptr()), reinterpret_cast<uint8_t*>(yt.data_ptr()), M, N);
}

// Kernel choice of fp8_gemm: 0 = default, 1 = v1 (128x128), 2 = v2 4 waves, 3 = v2 8 waves, 4 = v3 (4-deep ring),
// 5 = v3 8 waves, 6 = v4 (16x16x128 MFMA, BK 128, two slots), 7 = v4 with the unscaled MFMA opcode, 8 / 9 = v3 4 / 8
// waves with the unscaled MFMA opcode, 10 / 11 = v5 (v4 tiling, one barrier per K-step) scaled / unscaled, 12 / 13 =
// v6 (v3 with the LDS-DMA issue spread over the whole K-tile) scaled / unscaled, 14 / 15 = v7 (v5 tiling, copy staged
// through registers instead of LDS-DMA) scaled / unscaled, 16 / 17 = v8 (v7 with 8 waves in a barrier-staggered
// ping-pong) scaled / unscaled.
// Shapes a variant cannot tile fall back to the next one that can (v3 -> v2 -> v1).
constexpr int kFp8GemmDefault = 18;  // the asm-scheduled kernel (fp8_gemm_asm.hip; profiles/r5_gemm_fp8_asm.md); v8 for other shapes
// variant 18: the hand-scheduled asm main loop (fp8_gemm_asm.hip)
bool fp8_gemm_asm_launch(const uint8_t* a, const uint8_t* b, const float* sa, const float* sb, float smul,
                         const bf16_t* bias, void* c, int M, int N, int K, bool a_e5m2, bool b_e5m2, bool out_f32,
                         bool accum, int group_m, hipStream_t stream);
static int g_fp8_gemm_variant = 0;
static int g_fp8_gemm_group_m = 4;  // v3 tile-row grouping (1 = plain row-major tile order)
static int g_fp8_asm_group_m = 0;   // variant 18's grouping; 0 = by shape (fp8_gemm_asm_launch)
void fp8_gemm_select(int64_t variant, int64_t group_m) {
  TORCH_CHECK(variant >= 0 && variant <= 18, "fp8_gemm_select: variant 0..18");
  TORCH_CHECK(group_m >= 0 && group_m <= 64, "fp8_gemm_select: group_m 0..64");
  g_fp8_gemm_variant = (int)variant;
  if (group_m > 0) g_fp8_gemm_group_m = (int)group_m;
  g_fp8_asm_group_m = (int)group_m;
}

// C = (a . b^T) * sa[0] * sb[0] * smul (+ bias): sa / sb are inverse scales, or amax buffers with smul = 1/(qa*qb).
// `out` (optional): write into this contiguous [M, N] tensor (fp32 when out_fp32, else bf16) instead of a new one, adding
// to its contents when `accumulate` (the FSDP flat-grad / fp32 grad-shard destination of a weight gradient).
torch::Tensor fp8_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor a_scale_inv, torch::Tensor b_scale_inv, double smul,
                       bool a_e5m2, bool b_e5m2, c10::optional<torch::Tensor> bias, bool out_fp32,
                       c10::optional<torch::Tensor> out_opt, bool accumulate) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous(),
              "fp8_gemm: operands must be 2-D contiguous HIP tensors");
  TORCH_CHECK(a.element_size() == 1 && b.element_size() == 1, "fp8_gemm: operands must be fp8");
  const int M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "fp8_gemm: K mismatch");
  TORCH_CHECK(M % BM == 0 && N % BN == 0 && K % BK == 0, "fp8_gemm: M, N must be multiples of 128 and K of 64");
  torch::Tensor out;
  if (out_opt.has_value()) {
    out = *out_opt;
    TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.size(0) == M && out.size(1) == N &&
                    out.scalar_type() == (out_fp32 ? torch::kFloat32 : torch::kBFloat16),
                "fp8_gemm: out must be a contiguous [M, N] tensor of the output dtype");
  } else {
    TORCH_CHECK(!accumulate, "fp8_gemm: accumulate needs an out tensor");
    out = torch::empty({M, N}, a.options().dtype(out_fp32 ? torch::kFloat32 : torch::kBFloat16));
  }
  const int accum = accumulate ? 1 : 0;
  const bf16_t* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->numel() == N, "fp8_gemm: bias must be bf16 [N]");
    bp = reinterpret_cast<const bf16_t*>(bias->data_ptr());
  }
  auto stream = at::hip::getCurrentHIPStream();
  const uint8_t* ap = reinterpret_cast<const uint8_t*>(a.data_ptr());
  const uint8_t* bptr = reinterpret_cast<const uint8_t*>(b.data_ptr());
  const float* sap = a_scale_inv.data_ptr<float>();
  const float* sbp = b_scale_inv.data_ptr<float>();
  void* cp = out.data_ptr();
  static const bool force_v1 = std::getenv("ACCELERATE_FP8_GEMM_V1") != nullptr;
  static const bool env_w8 = [] {
    const char* e = std::getenv("ACCELERATE_FP8_GEMM_WAVES");
    return e != nullptr && std::atoi(e) == 8;
  }();
  int variant = g_fp8_gemm_variant;
  if (variant == 0) variant = force_v1 ? 1 : (env_w8 ? 3 : kFp8GemmDefault);
  if (variant == 18) {
    if (fp8_gemm_asm_launch(ap, bptr, sap, sbp, (float)smul, bp, cp, M, N, K, a_e5m2, b_e5m2, out_fp32, accumulate,
                            g_fp8_asm_group_m, stream))
      return out;
    variant = 17;
  }
  if ((variant == 10 || variant == 11) && M % V4_BM == 0 && N % V4_BN == 0 && K % 256 == 0 &&
      (long)V4_BM * K < (1L << 30) && (reinterpret_cast<uintptr_t>(bp) & 7) == 0) {
    const int nwg5 = (M / V4_BM) * (N / V4_BN);
    const bool un = variant == 11;
#define GEMM5_LAUNCH(FA, FB, OF)                                                                                        \
  do {                                                                                                                  \
    if (un)                                                                                                             \
      hipLaunchKernelGGL((fp8_gemm_v5_kernel<FA, FB, OF, true>), dim3(nwg5), dim3(256), 0, stream, ap, bptr, sap, sbp,   \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
    else                                                                                                                \
      hipLaunchKernelGGL((fp8_gemm_v5_kernel<FA, FB, OF, false>), dim3(nwg5), dim3(256), 0, stream, ap, bptr, sap, sbp,  \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
  } while (0)
    if (!a_e5m2 && !b_e5m2) { if (out_fp32) GEMM5_LAUNCH(0, 0, true); else GEMM5_LAUNCH(0, 0, false); }
    else if (!a_e5m2 && b_e5m2) { if (out_fp32) GEMM5_LAUNCH(0, 1, true); else GEMM5_LAUNCH(0, 1, false); }
    else if (a_e5m2 && !b_e5m2) { if (out_fp32) GEMM5_LAUNCH(1, 0, true); else GEMM5_LAUNCH(1, 0, false); }
    else { if (out_fp32) GEMM5_LAUNCH(1, 1, true); else GEMM5_LAUNCH(1, 1, false); }
#undef GEMM5_LAUNCH
    return out;
  }
  if (variant == 10 || variant == 11) variant = 4;
  if ((variant == 12 || variant == 13) && M % V3_BM == 0 && N % V3_BN == 0 && K % 256 == 0 &&
      (long)V3_BM * K < (1L << 30) && (reinterpret_cast<uintptr_t>(bp) & 7) == 0) {
    const int nwg6 = (M / V3_BM) * (N / V3_BN);
    const bool un = variant == 13;
#define GEMM6_LAUNCH(FA, FB, OF)                                                                                        \
  do {                                                                                                                  \
    if (un)                                                                                                             \
      hipLaunchKernelGGL((fp8_gemm_v6_kernel<FA, FB, OF, true>), dim3(nwg6), dim3(256), 0, stream, ap, bptr, sap, sbp,   \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
    else                                                                                                                \
      hipLaunchKernelGGL((fp8_gemm_v6_kernel<FA, FB, OF, false>), dim3(nwg6), dim3(256), 0, stream, ap, bptr, sap, sbp,  \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
  } while (0)
    if (!a_e5m2 && !b_e5m2) { if (out_fp32) GEMM6_LAUNCH(0, 0, true); else GEMM6_LAUNCH(0, 0, false); }
    else if (!a_e5m2 && b_e5m2) { if (out_fp32) GEMM6_LAUNCH(0, 1, true); else GEMM6_LAUNCH(0, 1, false); }
    else if (a_e5m2 && !b_e5m2) { if (out_fp32) GEMM6_LAUNCH(1, 0, true); else GEMM6_LAUNCH(1, 0, false); }
    else { if (out_fp32) GEMM6_LAUNCH(1, 1, true); else GEMM6_LAUNCH(1, 1, false); }
#undef GEMM6_LAUNCH
    return out;
  }
  if (variant == 12 || variant == 13) variant = 4;
  if ((variant == 14 || variant == 15) && M % V4_BM == 0 && N % V4_BN == 0 && K % V4_BK == 0 &&
      (long)V4_BM * K < (1L << 30) && (reinterpret_cast<uintptr_t>(bp) & 7) == 0) {
    const int nwg7 = (M / V4_BM) * (N / V4_BN);
    const bool un = variant == 15;
#define GEMM7_LAUNCH(FA, FB, OF)                                                                                        \
  do {                                                                                                                  \
    if (un)                                                                                                             \
      hipLaunchKernelGGL((fp8_gemm_v7_kernel<FA, FB, OF, true>), dim3(nwg7), dim3(256), 0, stream, ap, bptr, sap, sbp,   \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
    else                                                                                                                \
      hipLaunchKernelGGL((fp8_gemm_v7_kernel<FA, FB, OF, false>), dim3(nwg7), dim3(256), 0, stream, ap, bptr, sap, sbp,  \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
  } while (0)
    if (!a_e5m2 && !b_e5m2) { if (out_fp32) GEMM7_LAUNCH(0, 0, true); else GEMM7_LAUNCH(0, 0, false); }
    else if (!a_e5m2 && b_e5m2) { if (out_fp32) GEMM7_LAUNCH(0, 1, true); else GEMM7_LAUNCH(0, 1, false); }
    else if (a_e5m2 && !b_e5m2) { if (out_fp32) GEMM7_LAUNCH(1, 0, true); else GEMM7_LAUNCH(1, 0, false); }
    else { if (out_fp32) GEMM7_LAUNCH(1, 1, true); else GEMM7_LAUNCH(1, 1, false); }
#undef GEMM7_LAUNCH
    return out;
  }
  if (variant == 14 || variant == 15) variant = 4;
  if ((variant == 16 || variant == 17) && M % V4_BM == 0 && N % V4_BN == 0 && K % V4_BK == 0 &&
      (long)V4_BM * K < (1L << 30) && (reinterpret_cast<uintptr_t>(bp) & 7) == 0) {
    const int nwg8 = (M / V4_BM) * (N / V4_BN);
    const bool un = variant == 17;
#define GEMM8_LAUNCH(FA, FB, OF)                                                                                        \
  do {                                                                                                                  \
    if (un)                                                                                                             \
      hipLaunchKernelGGL((fp8_gemm_v8_kernel<FA, FB, OF, true>), dim3(nwg8), dim3(512), 0, stream, ap, bptr, sap, sbp,   \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
    else                                                                                                                \
      hipLaunchKernelGGL((fp8_gemm_v8_kernel<FA, FB, OF, false>), dim3(nwg8), dim3(512), 0, stream, ap, bptr, sap, sbp,  \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
  } while (0)
    if (!a_e5m2 && !b_e5m2) { if (out_fp32) GEMM8_LAUNCH(0, 0, true); else GEMM8_LAUNCH(0, 0, false); }
    else if (!a_e5m2 && b_e5m2) { if (out_fp32) GEMM8_LAUNCH(0, 1, true); else GEMM8_LAUNCH(0, 1, false); }
    else if (a_e5m2 && !b_e5m2) { if (out_fp32) GEMM8_LAUNCH(1, 0, true); else GEMM8_LAUNCH(1, 0, false); }
    else { if (out_fp32) GEMM8_LAUNCH(1, 1, true); else GEMM8_LAUNCH(1, 1, false); }
#undef GEMM8_LAUNCH
    return out;
  }
  if (variant == 16 || variant == 17) variant = 4;
  if ((variant == 6 || variant == 7) && M % V4_BM == 0 && N % V4_BN == 0 && K % 256 == 0 && (long)V4_BM * K < (1L << 30) &&
      (reinterpret_cast<uintptr_t>(bp) & 7) == 0) {
    const int nwg4 = (M / V4_BM) * (N / V4_BN);
    const bool un = variant == 7;
#define GEMM4_LAUNCH(FA, FB, OF)                                                                                        \
  do {                                                                                                                  \
    if (un)                                                                                                             \
      hipLaunchKernelGGL((fp8_gemm_v4_kernel<FA, FB, OF, true>), dim3(nwg4), dim3(256), 0, stream, ap, bptr, sap, sbp,   \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
    else                                                                                                                \
      hipLaunchKernelGGL((fp8_gemm_v4_kernel<FA, FB, OF, false>), dim3(nwg4), dim3(256), 0, stream, ap, bptr, sap, sbp,  \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
  } while (0)
    if (!a_e5m2 && !b_e5m2) { if (out_fp32) GEMM4_LAUNCH(0, 0, true); else GEMM4_LAUNCH(0, 0, false); }
    else if (!a_e5m2 && b_e5m2) { if (out_fp32) GEMM4_LAUNCH(0, 1, true); else GEMM4_LAUNCH(0, 1, false); }
    else if (a_e5m2 && !b_e5m2) { if (out_fp32) GEMM4_LAUNCH(1, 0, true); else GEMM4_LAUNCH(1, 0, false); }
    else { if (out_fp32) GEMM4_LAUNCH(1, 1, true); else GEMM4_LAUNCH(1, 1, false); }
#undef GEMM4_LAUNCH
    return out;
  }
  if (variant == 6 || variant == 7) variant = 4;  // shapes v4 cannot tile
  const bool v3_unscaled = variant == 8 || variant == 9;
  if (v3_unscaled) variant -= 4;
  const bool v3 = variant == 4 || variant == 5;
  if (v3 && !(M % V3_BM == 0 && N % V3_BN == 0 && K % (4 * V3_BK) == 0)) variant = 2;
  if (v3 && (reinterpret_cast<uintptr_t>(bp) & 7) != 0) variant = 2;  // v3 reads the bias 4 at a time
  // v3's buffer descriptors hold one 256-row panel: its byte size must stay below the zero-fill soffset (2^30)
  if (v3 && (long)V3_BM * K >= (1L << 30)) variant = 2;
  if (variant == 4 || variant == 5) {
    const int nwg3 = (M / V3_BM) * (N / V3_BN);
    const bool w8_3 = variant == 5;
#define GEMM3_LAUNCH(FA, FB, OF)                                                                                        \
  do {                                                                                                                  \
    if (w8_3 && v3_unscaled)                                                                                            \
      hipLaunchKernelGGL((fp8_gemm_v3_w8_kernel<FA, FB, OF, true>), dim3(nwg3), dim3(512), 0, stream, ap, bptr, sap, sbp, \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
    else if (w8_3)                                                                                                      \
      hipLaunchKernelGGL((fp8_gemm_v3_w8_kernel<FA, FB, OF>), dim3(nwg3), dim3(512), 0, stream, ap, bptr, sap, sbp, (float)smul, bp, \
                         cp, M, N, K, accum, g_fp8_gemm_group_m);                                                        \
    else if (v3_unscaled)                                                                                               \
      hipLaunchKernelGGL((fp8_gemm_v3_kernel<FA, FB, OF, true>), dim3(nwg3), dim3(256), 0, stream, ap, bptr, sap, sbp,    \
                         (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m);                                       \
    else                                                                                                                \
      hipLaunchKernelGGL((fp8_gemm_v3_kernel<FA, FB, OF>), dim3(nwg3), dim3(256), 0, stream, ap, bptr, sap, sbp, (float)smul, bp, \
                         cp, M, N, K, accum, g_fp8_gemm_group_m);                                                        \
  } while (0)
    if (!a_e5m2 && !b_e5m2) { if (out_fp32) GEMM3_LAUNCH(0, 0, true); else GEMM3_LAUNCH(0, 0, false); }
    else if (!a_e5m2 && b_e5m2) { if (out_fp32) GEMM3_LAUNCH(0, 1, true); else GEMM3_LAUNCH(0, 1, false); }
    else if (a_e5m2 && !b_e5m2) { if (out_fp32) GEMM3_LAUNCH(1, 0, true); else GEMM3_LAUNCH(1, 0, false); }
    else { if (out_fp32) GEMM3_LAUNCH(1, 1, true); else GEMM3_LAUNCH(1, 1, false); }
#undef GEMM3_LAUNCH
    return out;
  }
  if (variant != 1 && M % V2_BM == 0 && N % V2_BN == 0 && K % V2_BK == 0) {
    const int nwg2 = (M / V2_BM) * (N / V2_BN);
    const bool w8 = variant == 3;
#define GEMM2_LAUNCH(FA, FB, OF)                                                                                      \
  do {                                                                                                                \
    if (w8)                                                                                                           \
      hipLaunchKernelGGL((fp8_gemm_v2_w8_kernel<FA, FB, OF>), dim3(nwg2), dim3(512), 0, stream, ap, bptr, sap, sbp, (float)smul, bp, \
                         cp, M, N, K, accum);                                                                                \
    else                                                                                                              \
      hipLaunchKernelGGL((fp8_gemm_v2_w4_kernel<FA, FB, OF>), dim3(nwg2), dim3(256), 0, stream, ap, bptr, sap, sbp, (float)smul, bp, \
                         cp, M, N, K, accum);                                                                                \
  } while (0)
    if (!a_e5m2 && !b_e5m2) { if (out_fp32) GEMM2_LAUNCH(0, 0, true); else GEMM2_LAUNCH(0, 0, false); }
    else if (!a_e5m2 && b_e5m2) { if (out_fp32) GEMM2_LAUNCH(0, 1, true); else GEMM2_LAUNCH(0, 1, false); }
    else if (a_e5m2 && !b_e5m2) { if (out_fp32) GEMM2_LAUNCH(1, 0, true); else GEMM2_LAUNCH(1, 0, false); }
    else { if (out_fp32) GEMM2_LAUNCH(1, 1, true); else GEMM2_LAUNCH(1, 1, false); }
#undef GEMM2_LAUNCH
    return out;
  }
  const int nwg = (M / BM) * (N / BN);
#define GEMM_LAUNCH(FA, FB, OF) \
  hipLaunchKernelGGL((fp8_gemm_kernel<FA, FB, OF>), dim3(nwg), dim3(256), 0, stream, ap, bptr, sap, sbp, (float)smul, bp, cp, M, N, K, accum)
  if (!a_e5m2 && !b_e5m2) { if (out_fp32) GEMM_LAUNCH(0, 0, true); else GEMM_LAUNCH(0, 0, false); }
  else if (!a_e5m2 && b_e5m2) { if (out_fp32) GEMM_LAUNCH(0, 1, true); else GEMM_LAUNCH(0, 1, false); }
  else if (a_e5m2 && !b_e5m2) { if (out_fp32) GEMM_LAUNCH(1, 0, true); else GEMM_LAUNCH(1, 0, false); }
  else { if (out_fp32) GEMM_LAUNCH(1, 1, true); else GEMM_LAUNCH(1, 1, false); }
#undef GEMM_LAUNCH
  return out;
}

// C = (a . b^T) * smul (+ bias) with MX block scales: a [M, K] / b [N, K] fp8, sa [M, K/32] / sb [N, K/32] uint8 e8m0
// in mx_quant's grouped layout. Needs the v3 tiling: M, N multiples of 256, K of 256. out / accumulate as in fp8_gemm.
torch::Tensor mx_gemm(torch::Tensor a, torch::Tensor b, torch::Tensor sa, torch::Tensor sb, double smul,
                      c10::optional<torch::Tensor> bias, bool out_fp32, c10::optional<torch::Tensor> out_opt, bool accumulate) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() &&
                  a.element_size() == 1 && b.element_size() == 1, "mx_gemm: operands must be 2-D contiguous fp8");
  const int M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "mx_gemm: K mismatch");
  TORCH_CHECK(M % V3_BM == 0 && N % V3_BN == 0 && K % (4 * V3_BK) == 0, "mx_gemm: M, N, K must be multiples of 256");
  TORCH_CHECK((long)V3_BM * K < (1L << 30), "mx_gemm: K too large");
  TORCH_CHECK(sa.scalar_type() == at::kByte && sb.scalar_type() == at::kByte && sa.is_contiguous() && sb.is_contiguous() &&
                  sa.numel() == (long)M * (K / 32) && sb.numel() == (long)N * (K / 32), "mx_gemm: scales must be uint8 [rows, K/32]");
  const bool e5a = a.scalar_type() == at::kFloat8_e5m2, e5b = b.scalar_type() == at::kFloat8_e5m2;
  torch::Tensor out;
  if (out_opt.has_value()) {
    out = *out_opt;
    TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.size(0) == M && out.size(1) == N &&
                    out.scalar_type() == (out_fp32 ? torch::kFloat32 : torch::kBFloat16),
                "mx_gemm: out must be a contiguous [M, N] tensor of the output dtype");
  } else {
    TORCH_CHECK(!accumulate, "mx_gemm: accumulate needs an out tensor");
    out = torch::empty({M, N}, a.options().dtype(out_fp32 ? torch::kFloat32 : torch::kBFloat16));
  }
  const bf16_t* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->numel() == N && bias->is_contiguous(), "mx_gemm: bias must be bf16 [N]");
    bp = reinterpret_cast<const bf16_t*>(bias->data_ptr());
    TORCH_CHECK((reinterpret_cast<uintptr_t>(bp) & 7) == 0, "mx_gemm: bias must be 8-B aligned");
  }
  const int accum = accumulate ? 1 : 0;
  auto stream = at::hip::getCurrentHIPStream();
  const uint8_t* ap = reinterpret_cast<const uint8_t*>(a.data_ptr());
  const uint8_t* bq = reinterpret_cast<const uint8_t*>(b.data_ptr());
  const uint8_t* sap = sa.data_ptr<uint8_t>();
  const uint8_t* sbp = sb.data_ptr<uint8_t>();
  void* cp = out.data_ptr();
  const int nwg = (M / V3_BM) * (N / V3_BN);
#define MXG(FA, FB, OF) \
  hipLaunchKernelGGL((mx_gemm_kernel<FA, FB, OF>), dim3(nwg), dim3(256), 0, stream, ap, bq, sap, sbp, (float)smul, bp, cp, M, N, K, accum, g_fp8_gemm_group_m)
  if (!e5a && !e5b) { if (out_fp32) MXG(0, 0, true); else MXG(0, 0, false); }
  else if (!e5a && e5b) { if (out_fp32) MXG(0, 1, true); else MXG(0, 1, false); }
  else if (e5a && !e5b) { if (out_fp32) MXG(1, 0, true); else MXG(1, 0, false); }
  else { if (out_fp32) MXG(1, 1, true); else MXG(1, 1, false); }
#undef MXG
  return out;
}
