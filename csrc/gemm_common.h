// Helpers shared by the implicit-GEMM kernels (conv_nt.hip, conv_tn.hip).
#pragma once
#include "common.h"

template <int V>
struct VecT;
template <>
struct VecT<8> {
  typedef uint4 T;
};
template <>
struct VecT<4> {
  typedef uint2 T;
};
template <>
struct VecT<1> {
  typedef uint16_t T;
};

template <int V>
__device__ __forceinline__ typename VecT<V>::T vzero() {
  typename VecT<V>::T z;
  if constexpr (V == 8)
    z = make_uint4(0, 0, 0, 0);
  else if constexpr (V == 4)
    z = make_uint2(0, 0);
  else
    z = 0;
  return z;
}

// 32x32x16 MFMA operand fragment from a k-major LDS image via two ds_read_b64_tr_b16:
// lane 16g+4q+p supplies row q / cols 4p..4p+3 of a 4x16 block, lane i of the group gets
// column i of the 4 rows (CDNA4 hardware transpose read).
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* lo_addr, const bf16_t* hi_addr) {
  bf16x4 lo = __builtin_bit_cast(
      bf16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4_t __attribute__((address_space(3)))*)lo_addr));
  bf16x4 hi = __builtin_bit_cast(
      bf16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((short4_t __attribute__((address_space(3)))*)hi_addr));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// ---- buffer-resource operand loads (fp32 GEMM loaders)
// A per-client operand window as a buffer resource: a lane whose byte offset is past
// `bytes` (OOB_OFF) reads zeros, so padding / tails / idle loader threads need no branch and no
// zero-fill moves. Descriptor inputs are made provably wave-uniform (readfirstlane) so the
// compiler keeps the descriptor in SGPRs (no waterfall loop).
constexpr uint32_t OOB_OFF = 0x80000000u;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
// V consecutive floats at byte offset `off` (V = 8: two 16-B loads, 4: one, 1: one dword)
template <int V>
__device__ __forceinline__ void buf_load(float* f, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (V % 4 == 0) {
#pragma unroll
    for (int i = 0; i < V; i += 4) {
      const u32x4_t u = __builtin_amdgcn_raw_buffer_load_b128(r, off + 4 * i, 0, 0);
      f[i] = __uint_as_float(u.x);
      f[i + 1] = __uint_as_float(u.y);
      f[i + 2] = __uint_as_float(u.z);
      f[i + 3] = __uint_as_float(u.w);
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) f[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * i, 0, 0));
  }
}
