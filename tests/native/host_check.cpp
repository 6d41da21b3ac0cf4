// Host-side sanitizer check: the launch-planning code of the extension (index
// fast-division, tile / split-K / workspace selection, attention support predicates) compiled
// with AddressSanitizer + UndefinedBehaviorSanitizer on the HOST side only (-Xarch_host
// -fsanitize=...; GPU sanitizers are not used) and driven over the model zoo's layer shapes. No
// kernel is launched: this runs on a machine without a GPU (tests/test_native_host.py).
#include <cstdio>
#include <cstdlib>
#include <random>

#include "dls.h"

static int failures = 0;
#define CHECK(c, ...)                      \
  do {                                     \
    if (!(c)) {                            \
      ++failures;                          \
      if (failures < 20) {                 \
        fprintf(stderr, "FAIL %s: ", #c);  \
        fprintf(stderr, __VA_ARGS__);      \
        fprintf(stderr, "\n");             \
      }                                    \
    }                                      \
  } while (0)

// device fdiv() in 32-bit arithmetic: (umulhi(n, mul) + n) >> shift
static uint32_t fdiv_host(uint32_t n, const FastDiv& f) {
  const uint32_t hi = (uint32_t)(((uint64_t)n * f.mul) >> 32);
  return (uint32_t)(hi + n) >> f.shift;
}

int main() {
  std::mt19937_64 rng(1234);
  // 1) fast division: every divisor the kernels use (H·W products, W, KW·C, C) up to 2^20,
  //    numerators below 2^31 (the documented range) incl. the edges
  long checked = 0;
  for (uint32_t d = 1; d <= (1u << 20); d = d < 4096 ? d + 1 : d + 1 + (uint32_t)(rng() % 997)) {
    const FastDiv f = make_fastdiv(d);
    const uint32_t edges[] = {0u, 1u, d - 1, d, d + 1, 2 * d - 1, (1u << 31) - 1, (1u << 31) - d};
    for (uint32_t n : edges) {
      if (n >= (1u << 31)) continue;
      CHECK(fdiv_host(n, f) == n / d, "n=%u d=%u", n, d);
      ++checked;
    }
    for (int t = 0; t < 64; ++t) {
      const uint32_t n = (uint32_t)(rng() % (1ull << 31));
      CHECK(fdiv_host(n, f) == n / d, "n=%u d=%u", n, d);
      ++checked;
    }
  }
  // 2) launch planning over ResNet / DenseNet / Transformer / MLP layer shapes
  const int Ks[] = {1, 3, 13, 50, 100, 128};
  const int chans[] = {3, 8, 12, 16, 64, 100, 128, 256, 512, 2048};
  const int hw[] = {1, 4, 8, 16, 32, 56, 224};
  for (int K : Ks)
    for (int co : chans)
      for (int ci : chans)
        for (int h : hw) {
          const int M = 64 * h * h, R = 9 * ci;
          for (int bkm = 0; bkm < 2; ++bkm) {
            const int v = conv_nt_default_variant(M, co, R, bkm);
            CHECK(v >= 0 && v < conv_nt_num_variants(), "nt variant %d", v);
          }
          for (int f32 = 0; f32 < 2; ++f32) {
            const int sk = conv_tn_splitk(K, co, R, M, ci, -1, f32);
            CHECK(sk >= 1 && sk <= M, "splitk %d (K=%d co=%d R=%d M=%d f32=%d)", sk, K, co, R, M, f32);
          }
          for (int v = 0; v < conv_tn_f32_num_variants(); ++v) {
            const int sk = conv_tn_f32_splitk(K, co, R, M, co, ci, v);
            CHECK(sk >= 1 && sk <= M, "f32 splitk %d", sk);
          }
          const long ws = bn_workspace_floats(K, M, co);
          CHECK(ws >= 3L * K * co, "bn workspace %ld", ws);
          (void)conv_gl_wanted(K, M, co, ci, 9, -1);
          (void)conv_gl_supported(ci, co, 9);
        }
  // 3) attention support predicates
  for (int L = 1; L <= 1024; L += 37)
    for (int dh : {8, 16, 20, 32, 50, 64, 100, 128}) {
      const bool packed = attn_packed_supported(L, dh), mfma = attn_mfma_supported(L, dh);
      (void)attn_supported(L, dh);
      CHECK(!packed || mfma || attn_supported(L, dh), "packed without a kernel L=%d dh=%d", L, dh);
    }
  printf("host_check: %ld fast-division cases, %d failures\n", checked, failures);
  return failures ? 1 : 0;
}
