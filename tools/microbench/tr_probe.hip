// What gfx950's transposing LDS reads deliver, lane by lane: fills a 4 KiB LDS window with a byte pattern that encodes
// each byte's address (two runs: low and high address byte), lets every lane read with `ds_read_b64_tr_b16` /
// `ds_read_b64_tr_b8` at an address of the probe's choosing, and prints, for each lane and each delivered byte, the LDS
// address it came from. Used to pin the tr_b8 operand map before building an fp8 MN-major GEMM on it (the tr_b16 map is
// documented in cdna_hip_programming.md T10 and serves as the check of the probe itself).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/tr_probe.hip -o /tmp/tr_probe && /tmp/tr_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

// lane l reads at byte address addr[l]; out[l * 8 + b] = pattern byte b delivered to lane l
template <int KIND>
__global__ __launch_bounds__(64) void probe(const unsigned* __restrict__ addr, int hi, unsigned char* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = hi ? (unsigned char)(i >> 8) : (unsigned char)(i & 255);
  __syncthreads();
  const unsigned a = static_cast<unsigned>(reinterpret_cast<uintptr_t>(lds)) + addr[threadIdx.x];
  unsigned long long r;
  if (KIND == 16)
    asm volatile("ds_read_b64_tr_b16 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a));
  else
    asm volatile("ds_read_b64_tr_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a));
  for (int b = 0; b < 8; ++b) out[threadIdx.x * 8 + b] = (unsigned char)(r >> (8 * b));
}

int main() {
  unsigned h_addr[64];
  // natural probe addresses: lane l -> row (l & 15) of a [16 rows][256 B] image, column block (l >> 4) * 8 B
  // (arbitrary but distinct 8-B-aligned addresses; the output shows where every delivered byte came from)
  for (int l = 0; l < 64; ++l) h_addr[l] = (unsigned)((l & 15) * 256 + (l >> 4) * 8);
  unsigned* d_addr;
  unsigned char* d_out;
  hipMalloc(&d_addr, sizeof(h_addr));
  hipMalloc(&d_out, 512);
  hipMemcpy(d_addr, h_addr, sizeof(h_addr), hipMemcpyHostToDevice);
  unsigned char lo[512], hi[512];
  for (int kind : {16, 8}) {
    for (int h = 0; h < 2; ++h) {
      if (kind == 16) hipLaunchKernelGGL(probe<16>, dim3(1), dim3(64), 0, 0, d_addr, h, d_out);
      else hipLaunchKernelGGL(probe<8>, dim3(1), dim3(64), 0, 0, d_addr, h, d_out);
      hipMemcpy(h ? hi : lo, d_out, 512, hipMemcpyDeviceToHost);
    }
    printf("kind tr_b%d: lane: [byte0 addr, ...]  (lane address given as row*256+colbyte)\n", kind);
    for (int l = 0; l < 64; ++l) {
      printf("lane %2d (addr %4u):", l, h_addr[l]);
      for (int b = 0; b < 8; ++b) printf(" %4d", (int)lo[l * 8 + b] | ((int)hi[l * 8 + b] << 8));
      printf("\n");
    }
  }
  hipFree(d_addr);
  hipFree(d_out);
  return 0;
}
