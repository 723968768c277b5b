// Host-side runtime kernels with no torch / HIP dependency, shared by the extension (cpu_adam.cpp, h2d_engine.cpp)
// and by the sanitizer harness tests/native/host_sanitize.cpp (built with -fsanitize=address,undefined on the CPU,
// tests/test_host_sanitizers.py).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <string>

namespace acc_host {

struct Hyper {
  float lr, beta1, beta2, eps, wd, bc1, bc2_sqrt;
  bool adamw;
};

inline uint16_t to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

// static: one copy (with its own clone resolver) per translation unit that includes this header
__attribute__((target_clones("avx512f", "avx2", "default")))
static void adam_range(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                uint16_t* __restrict__ shadow, int64_t n, Hyper h) {
  const float step_size = h.lr / h.bc1, bc2s = h.bc2_sqrt, decay = 1.f - h.lr * h.wd;
  const float b1 = h.beta1, b2 = h.beta2, c1 = 1.f - h.beta1, c2 = 1.f - h.beta2;
  constexpr int64_t kBlock = 1 << 14;
  const int64_t nblk = (n + kBlock - 1) / kBlock;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nblk; ++b) {
    const int64_t lo = b * kBlock, hi = std::min(n, lo + kBlock);
#pragma omp simd
    for (int64_t i = lo; i < hi; ++i) {
      float pf = p[i], gf = g[i];
      if (!h.adamw) gf += h.wd * pf;
      const float mf = b1 * m[i] + c1 * gf;
      const float vf = b2 * v[i] + c2 * gf * gf;
      if (h.adamw) pf *= decay;
      pf -= step_size * mf / (std::sqrt(vf) / bc2s + h.eps);
      m[i] = mf;
      v[i] = vf;
      p[i] = pf;
    }
    if (shadow != nullptr) {
#pragma omp simd
      for (int64_t i = lo; i < hi; ++i) shadow[i] = to_bf16_rne(p[i]);
    }
  }
}


// Rolling FNV-1a hash over the sequence of collectives a rank issued (op, group size, dtype, numel). In debug
// mode ranks compare it every N steps, catching a desynchronised collective order before RCCL deadlocks.
class CollectiveSeq {
 public:
  void record(const std::string& op, int64_t group, int64_t dtype, int64_t numel) {
    auto mix = [this](uint64_t v) {
      for (int i = 0; i < 8; ++i) {
        h_ ^= (v >> (8 * i)) & 0xff;
        h_ *= 1099511628211ull;
      }
    };
    for (char c : op) mix((uint64_t)(unsigned char)c);
    mix((uint64_t)group);
    mix((uint64_t)dtype);
    mix((uint64_t)numel);
    ++count_;
  }
  uint64_t digest() const { return h_; }
  int64_t count() const { return count_; }
  void reset() { h_ = 1469598103934665603ull; count_ = 0; }

 private:
  uint64_t h_ = 1469598103934665603ull;
  int64_t count_ = 0;
};

}  // namespace acc_host
