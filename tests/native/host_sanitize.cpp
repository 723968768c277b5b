// Host-side sanitizer harness for the native runtime's CPU code (csrc/runtime/host_kernels.h): the OpenMP host AdamW
// of FSDP CPU offload and the collective-sequence digest. Built by tests/test_host_sanitizers.py with
// -fsanitize=address,undefined (GPU AddressSanitizer is not available on this pool; the GPU kernels are covered by
// their numerics tests). Exit status 0 = every check passed and the sanitizers reported nothing.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "host_kernels.h"

using namespace acc_host;

static int failures = 0;
#define CHECK(cond, ...)              \
  do {                                \
    if (!(cond)) {                    \
      std::fprintf(stderr, __VA_ARGS__); \
      std::fprintf(stderr, "\n");     \
      ++failures;                     \
    }                                 \
  } while (0)

static void check_adam(int64_t n, bool adamw, bool with_shadow, std::mt19937& rng) {
  std::normal_distribution<float> nd(0.f, 1.f);
  // exact-size heap buffers: an out-of-range access in any tail / block boundary is an ASan report
  std::vector<float> p(n), g(n), m(n), v(n), p0, m0, v0;
  for (int64_t i = 0; i < n; ++i) {
    p[i] = nd(rng);
    g[i] = 1e-2f * nd(rng);
    m[i] = 1e-3f * nd(rng);
    v[i] = 1e-5f * std::fabs(nd(rng));
  }
  p0 = p, m0 = m, v0 = v;
  std::vector<uint16_t> sh(with_shadow ? n : 0);
  const Hyper h{1e-3f, 0.9f, 0.999f, 1e-8f, 0.01f, 0.19f, 0.0447f, adamw};
  adam_range(p.data(), g.data(), m.data(), v.data(), with_shadow ? sh.data() : nullptr, n, h);
  for (int64_t i = 0; i < n; ++i) {  // double-precision reference of the same update
    double pf = p0[i], gf = g[i];
    if (!adamw) gf += (double)h.wd * pf;
    const double mf = (double)h.beta1 * m0[i] + (1.0 - h.beta1) * gf;
    const double vf = (double)h.beta2 * v0[i] + (1.0 - h.beta2) * gf * gf;
    if (adamw) pf *= 1.0 - (double)h.lr * h.wd;
    pf -= (double)h.lr / h.bc1 * mf / (std::sqrt(vf) / h.bc2_sqrt + h.eps);
    CHECK(std::fabs(p[i] - pf) <= 1e-5 * (1.0 + std::fabs(pf)), "adam p[%ld] %g vs %g (n=%ld)", (long)i, p[i], pf, (long)n);
    CHECK(std::fabs(m[i] - mf) <= 1e-6 * (1.0 + std::fabs(mf)), "adam m[%ld]", (long)i);
    CHECK(std::fabs(v[i] - vf) <= 1e-6 * (1.0 + std::fabs(vf)), "adam v[%ld]", (long)i);
    if (with_shadow) CHECK(sh[i] == to_bf16_rne(p[i]), "shadow[%ld]", (long)i);
  }
}

static float from_bf16(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

int main() {
  std::mt19937 rng(1234);
  const int64_t sizes[] = {0, 1, 7, 16383, 16384, 16385, 3 * 16384 + 5, 100003};
  for (int64_t n : sizes)
    for (int aw = 0; aw < 2; ++aw)
      for (int sh = 0; sh < 2; ++sh) check_adam(n, aw != 0, sh != 0, rng);
  // bf16 round-to-nearest-even: ties, NaN, infinities, the largest finite values
  CHECK(to_bf16_rne(1.0f) == 0x3f80, "bf16(1)");
  CHECK(from_bf16(to_bf16_rne(1.00390625f)) == 1.0f, "tie to even (down)");
  CHECK(from_bf16(to_bf16_rne(1.01171875f)) == 1.015625f, "tie to even (up)");
  CHECK((to_bf16_rne(std::nanf("")) & 0x7fc0) == 0x7fc0, "NaN stays NaN");
  CHECK(to_bf16_rne(INFINITY) == 0x7f80 && to_bf16_rne(-INFINITY) == 0xff80, "inf");
  CHECK(to_bf16_rne(3.4e38f) == 0x7f80, "overflow rounds to inf");
  // collective digest: order-sensitive, reset restores the initial state
  CollectiveSeq a, b;
  a.record("all_reduce", 8, 6, 1024);
  a.record("all_gather", 8, 15, 4096);
  b.record("all_gather", 8, 15, 4096);
  b.record("all_reduce", 8, 6, 1024);
  CHECK(a.digest() != b.digest() && a.count() == 2 && b.count() == 2, "digest must depend on order");
  b.reset();
  b.record("all_reduce", 8, 6, 1024);
  b.record("all_gather", 8, 15, 4096);
  CHECK(a.digest() == b.digest(), "digest must be reproducible after reset");
  std::printf("host_sanitize: %d failure(s)\n", failures);
  return failures == 0 ? 0 : 1;
}
