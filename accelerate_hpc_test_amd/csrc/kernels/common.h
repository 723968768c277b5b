// Shared device helpers for the CDNA4 (gfx950 / MI355X) kernels of accelerate_hpc_test_amd.
//
// Conventions used by every kernel in this directory:
//  * wave64: all cross-lane reductions are over 64 lanes (`__shfl_xor` up to offset 32).
//  * bf16 is handled as raw 16-bit storage (`bf16_t`), converted with the gfx950 hardware
//    conversion (`__bf16` casts lower to v_cvt_pk_bf16_f32, NaN preserving).
//  * memory-bound kernels move 16 bytes per lane per access (8 x bf16 or 4 x fp32).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace acc {

using bf16_t = uint16_t;

struct alignas(16) bf16x8 { bf16_t v[8]; };
struct alignas(8) bf16x4 { bf16_t v[4]; };

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(static_cast<uint32_t>(x) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T> __device__ __forceinline__ float to_f(T x);
template <> __device__ __forceinline__ float to_f<float>(float x) { return x; }
template <> __device__ __forceinline__ float to_f<bf16_t>(bf16_t x) { return bf2f(x); }

template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float x) { return f2bf(x); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (16 waves). `scratch` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = (threadIdx.x < nw) ? scratch[threadIdx.x] : 0.f;
  if (wid == 0) r = wave_sum(r);
  if (threadIdx.x == 0) scratch[0] = r;
  __syncthreads();
  r = scratch[0];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = (threadIdx.x < nw) ? scratch[threadIdx.x] : -INFINITY;
  if (wid == 0) r = wave_max(r);
  if (threadIdx.x == 0) scratch[0] = r;
  __syncthreads();
  r = scratch[0];
  return r;
}

// Bijective XCD-aware remap of a 1-D workgroup id (MI355X: 8 XCDs, blocks dealt round-robin):
// consecutive *logical* tiles land on the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  if (nwg <= nx) return bid;
  const int q = nwg / nx, r = nwg % nx;
  const int xcd = bid % nx, k = bid / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// ---- device-side checks of the debug build ------------------------------------------------------
// Compiled in only for the `_C_debug` extension (-DACC_DEBUG_BOUNDS; `ACCELERATE_DEBUG_KERNELS=1` loads it instead of
// `_C`). A failed check records (check id, source line) in this translation unit's device error word and the guarded
// access is skipped: ACC_CHECK_OR_RETURN leaves the kernel (only for block-uniform conditions, before any barrier),
// ACC_CHECK just records (the caller then takes its safe path). Nothing traps: a trapping wave faults the GPU.
// Each kernel file defines `ACC_DEBUG_TAKE_FN(name)`, a host function returning (id << 32 | line) of the first failed
// check since the last call (0 = none) and clearing it; `_C.debug_status()` polls every file.
enum AccCheck : int {
  kChkAttnTile = 1, kChkGemmTile = 2, kChkGroupSeg = 3, kChkNormRow = 4, kChkXentLabel = 5, kChkMtChunk = 6,
  kChkAllreduceSize = 7, kChkRopePos = 8, kChkRoutePos = 9, kChkCastTable = 10, kChkSelfTest = 99,
};
#ifdef ACC_DEBUG_BOUNDS
static __device__ int acc_dbg_word[2];
__device__ __forceinline__ void acc_dbg_fail(int code, int line) {
  if (atomicCAS(&acc_dbg_word[0], 0, code) == 0) atomicExch(&acc_dbg_word[1], line);
}
#define ACC_CHECK(cond, code) \
  do {                         \
    if (!(cond)) ::acc::acc_dbg_fail((code), __LINE__); \
  } while (0)
#define ACC_CHECK_OR_RETURN(cond, code) \
  do {                                   \
    if (!(cond)) {                       \
      ::acc::acc_dbg_fail((code), __LINE__); \
      return;                            \
    }                                    \
  } while (0)
#define ACC_DEBUG_TAKE_FN(name)                                                                  \
  int64_t name() {                                                                               \
    int w[2] = {0, 0};                                                                           \
    (void)hipDeviceSynchronize();                                                                \
    (void)hipMemcpyFromSymbol(w, HIP_SYMBOL(::acc::acc_dbg_word), sizeof(w), 0, hipMemcpyDeviceToHost); \
    if (w[0] != 0) {                                                                             \
      const int z[2] = {0, 0};                                                                   \
      (void)hipMemcpyToSymbol(HIP_SYMBOL(::acc::acc_dbg_word), z, sizeof(z), 0, hipMemcpyHostToDevice); \
    }                                                                                            \
    return ((int64_t)w[0] << 32) | (uint32_t)w[1];                                               \
  }
#define ACC_DEBUG_BUILD 1
#else
#define ACC_CHECK(cond, code) ((void)0)
#define ACC_CHECK_OR_RETURN(cond, code) ((void)0)
#define ACC_DEBUG_TAKE_FN(name) \
  int64_t name() { return 0; }
#define ACC_DEBUG_BUILD 0
#endif

}  // namespace acc
