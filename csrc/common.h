// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of the cohort FL simulator.
// Wave64 everywhere; bf16 stored as raw uint16 and converted with RNE.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CHECK_HIP(x)                                                                  \
  do {                                                                                \
    hipError_t err__ = (x);                                                           \
    if (err__ != hipSuccess) {                                                        \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(err__), __FILE__, \
              __LINE__);                                                              \
    }                                                                                 \
  } while (0)

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (bf16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// 8 bf16 packed in a uint4 (16 B)
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f);
// 8 bf16 + 8 bf16 (fp32 add, one rounding): epilogue accumulate of a second gradient branch
__device__ __forceinline__ uint4 add_bf16x8(const uint4& a, const uint4& b) {
  float fa[8], fb[8];
  unpack8(a, fa);
  unpack8(b, fb);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[i] += fb[i];
  return pack8(fa);
}
// keep the 8 bf16 of v where the matching gate value is > 0 (bit-exact select, no arithmetic)
__device__ __forceinline__ uint4 gate_bf16x8(const uint4& v, const uint4& g) {
  uint32_t out[4];
  const uint32_t* vv = reinterpret_cast<const uint32_t*>(&v);
  const uint32_t* gg = reinterpret_cast<const uint32_t*>(&g);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool lo = __uint_as_float(gg[i] << 16) > 0.f, hi = __uint_as_float(gg[i] & 0xffff0000u) > 0.f;
    out[i] = (lo ? (vv[i] & 0xffffu) : 0u) | (hi ? (vv[i] & 0xffff0000u) : 0u);
  }
  return make_uint4(out[0], out[1], out[2], out[3]);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---- element-type-generic access: every activation kernel is instantiated for bf16 storage
// (fast mode) and fp32 storage (reference precision, the reference trains in fp32:
// conf/global.yaml `use_amp: false`). Arithmetic is always fp32.
__device__ __forceinline__ float ldf(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ void stf(bf16_t* p, float v) { *p = f2bf(v); }
__device__ __forceinline__ void stf(float* p, float v) { *p = v; }
// the value a store of v to T would read back (bf16 rounding only for bf16 storage)
template <typename T>
__device__ __forceinline__ float rt(float v) {
  if constexpr (sizeof(T) == 2) return bf2f(f2bf(v)); else return v;
}

template <int V>
__device__ __forceinline__ void load_vec(const bf16_t* p, float* f) {
  if constexpr (V == 8) {
    unpack8(*reinterpret_cast<const uint4*>(p), f);
  } else if constexpr (V == 4) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    f[0] = __uint_as_float(u.x << 16);
    f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16);
    f[3] = __uint_as_float(u.y & 0xffff0000u);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) f[i] = bf2f(p[i]);
  }
}
template <int V>
__device__ __forceinline__ void load_vec(const float* p, float* f) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V; i += 4) {
      const float4 u = *reinterpret_cast<const float4*>(p + i);
      f[i] = u.x;
      f[i + 1] = u.y;
      f[i + 2] = u.z;
      f[i + 3] = u.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) f[i] = p[i];
  }
}
template <int V>
__device__ __forceinline__ void store_vec(bf16_t* p, const float* f) {
  if constexpr (V == 8) {
    *reinterpret_cast<uint4*>(p) = pack8(f);
  } else if constexpr (V == 4) {
    uint2 u;
    u.x = (uint32_t)f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16);
    u.y = (uint32_t)f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16);
    *reinterpret_cast<uint2*>(p) = u;
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) p[i] = f2bf(f[i]);
  }
}
template <int V>
__device__ __forceinline__ void store_vec(float* p, const float* f) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V; i += 4) *reinterpret_cast<float4*>(p + i) = make_float4(f[i], f[i + 1], f[i + 2], f[i + 3]);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) p[i] = f[i];
  }
}

// ---- split-bf16 ("bf16x3") operands of the fp32-accurate GEMMs: x = hi + lo with
// hi = bf16(x), lo = bf16(x − hi) (both RNE) ⇒ |x − hi − lo| ≤ 2⁻¹⁷|x|. A·B is then
// Ah·Bh + Al·Bh + Ah·Bl on the bf16 MFMA (fp32 accumulate); the dropped Al·Bl term is
// ≤ 2⁻¹⁸|A||B|. Three bf16 MFMAs cost 3/16 of one f32 MFMA's time for the same tile.
__device__ __forceinline__ void split2(float x, bf16_t& hi, bf16_t& lo) {
  const __bf16 h = (__bf16)x;  // RNE; hipcc emits v_cvt_pk_bf16_f32 for pairs
  const __bf16 l = (__bf16)(x - (float)h);
  hi = __builtin_bit_cast(bf16_t, h);
  lo = __builtin_bit_cast(bf16_t, l);
}
// Two floats → packed (hi1:hi0) and (lo1:lo0) bf16 pairs in 2.5 VALU ops per element: one
// v_cvt_pk_bf16_f32 for both hi (RNE), hi back to fp32 by a shift (element 0) and a mask
// (element 1), one v_pk_add_f32 for both residuals, one v_cvt_pk_bf16_f32 for both lo.
// (split2 per element compiles to cvt + shift + sub and a second packing cvt: 4 ops.)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split_pair(float x0, float x1, uint32_t& hi, uint32_t& lo) {
  const f32x2_t v = {x0, x1};
  const bf16x2_t h = __builtin_convertvector(v, bf16x2_t);
  const uint32_t hb = __builtin_bit_cast(uint32_t, h);
  const f32x2_t hf = {__uint_as_float(hb << 16), __uint_as_float(hb & 0xffff0000u)};
  const f32x2_t r = v - hf;
  hi = hb;
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2_t));
}

// V consecutive floats → V hi + V lo bf16 (V = 4: 8-B halves, V = 8: 16-B halves)
template <int V>
__device__ __forceinline__ void split_vec(const float* f, bf16_t* hi, bf16_t* lo) {
#pragma unroll
  for (int i = 0; i < V; ++i) split2(f[i], hi[i], lo[i]);
}

// 32-bit hash of (index, seed): the per-element uniforms of masks and stochastic rounding
// (identical to ops/fl.py `_mix`, so CPU and GPU draw the same numbers)
__device__ __forceinline__ uint32_t mix32(uint32_t x, uint32_t seed) {
  x ^= seed * 0x9E3779B9u;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// dropout keep-decision of element (m, n) of an [M][N] output of client row k (GEMM epilogues,
// dropout_apply): mix32(m·N + n, seed_k) >= p·2^32
__device__ __forceinline__ bool drop_keep(uint32_t seed, long m, int N, int n, float p) {
  const uint32_t thr = (uint32_t)fminf(p * 4294967296.f, 4294967040.f);
  return mix32((uint32_t)(m * (long)N + n), seed) >= thr;
}

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

// XCD-aware bijective remap of a 1-D block id (guide §5 "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD (shared L2) instead of round-robin.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg < nxcd) return orig;
  const int q = nwg / nxcd, r = nwg % nxcd;
  const int xcd = orig % nxcd, pos = orig / nxcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
