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
