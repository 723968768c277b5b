// Sustained rate of the gfx950 fp8 MFMA shapes with operands in registers (no memory traffic): one 256-thread
// workgroup per CU (one wave per SIMD), NACC independent accumulators per wave, ITERS trips of a fully unrolled
// chain. Answers whether v_mfma_f32_32x32x64_f8f6f4 and v_mfma_f32_16x16x128_f8f6f4 (scaled / unscaled) reach the same
// fraction of the 5 PF/s dense fp8 peak at one wave per SIMD, on random operands.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/mfma_peak.hip -o /tmp/mfma_peak && /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int SCALE>
__global__ __launch_bounds__(256, 1) void k32(const int* __restrict__ in, float* __restrict__ out, int iters) {
  v8i a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[i][e] = in[(threadIdx.x * 64 + i * 8 + e) & 4095];
      b[i][e] = in[(threadIdx.x * 64 + 32 + i * 8 + e) & 4095];
    }
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b[j], a[i], acc[i][j], 0, 0, 0, SCALE, 0, SCALE);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) s += acc[i][j][e];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int SCALE>
__global__ __launch_bounds__(256, 1) void k16(const int* __restrict__ in, float* __restrict__ out, int iters) {
  v8i a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[i][e] = in[(threadIdx.x * 128 + i * 8 + e) & 4095];
      b[i][e] = in[(threadIdx.x * 128 + 64 + i * 8 + e) & 4095];
    }
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b[j], a[i], acc[i][j], 0, 0, 0, SCALE, 0, SCALE);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += acc[i][j][e];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K>
float timeit(K kern, const int* in, float* out, int iters, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, iters);
  hipEventRecord(e0);
  const int reps = 10;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const int grid = 256, iters = 4000;
  int* in;
  float* out;
  hipMalloc(&in, 4096 * sizeof(int));
  hipMalloc(&out, grid * 256 * sizeof(float));
  int host[4096];
  srand(1);
  for (int i = 0; i < 4096; ++i) host[i] = rand() & 0x7f7f7f7f;  // random finite e4m3 bytes (no NaN pattern)
  hipMemcpy(in, host, sizeof(host), hipMemcpyHostToDevice);
  // per wave per trip: k32 = 16 MFMAs of 32x32x64 (2*32*32*64 FLOP each), k16 = 64 of 16x16x128 (2*16*16*128 each),
  // i.e. k16 does twice the work of k32 per trip
  const double flop32 = (double)grid * 4 * iters * 16 * 2.0 * 32 * 32 * 64;
  const double flop16 = (double)grid * 4 * iters * 64 * 2.0 * 16 * 16 * 128;
  const float t32s = timeit(k32<0x7f7f7f7f>, in, out, iters, grid);
  const float t32u = timeit(k32<0>, in, out, iters, grid);
  const float t16s = timeit(k16<0x7f7f7f7f>, in, out, iters, grid);
  const float t16u = timeit(k16<0>, in, out, iters, grid);
  printf("{\"mfma_32x32x64_scaled_tflops\": %.1f, \"mfma_32x32x64_unscaled_tflops\": %.1f, "
         "\"mfma_16x16x128_scaled_tflops\": %.1f, \"mfma_16x16x128_unscaled_tflops\": %.1f}\n",
         flop32 / t32s / 1e9, flop32 / t32u / 1e9, flop16 / t16s / 1e9, flop16 / t16u / 1e9);
  return 0;
}
