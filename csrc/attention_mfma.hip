// Multi-head attention fwd / bwd on the MFMA (gfx950), head dim 32 or 64, any sequence length.
//
//   q, k, v, o, do, dq, dk, dv : [KBH][L][DH] (bf16, or fp32 = reference precision)
//   lse, delta                 : [KBH][L] fp32;   key_valid [KB] (valid keys per sequence)
//
// Flash-style (no L×L matrix in HBM): one workgroup = 4 waves = 128 query rows (fwd, dq) or
// 128 key rows (dkv) of one (sequence, head); the other operand streams through LDS in 32-row
// blocks. Every product is a v_mfma_f32_32x32x16_bf16; in fp32 mode operands are split
// hi + lo bf16 and each product is three MFMAs (ah·bh + al·bh + ah·bl, fp32 accumulate — as
// conv_f32.hip), so the result carries ~2⁻¹⁶ relative error per product instead of bf16's 2⁻⁸.
//
// Orientation trick: the score tile is computed TRANSPOSED where that puts the softmax index in
// the lane's column — the 32×32 C layout gives lane ℓ column ℓ&31 and 16 rows — so the per-query
// (fwd / dq) max, sum and rescale of the output accumulator are in-lane plus one xor-32
// shuffle, and the output itself is accumulated transposed (Oᵀ = Vᵀ·Pᵀ) so its columns are the
// same queries. P / dS round-trip through a per-wave LDS tile to become MFMA operands.
//   fwd : Sᵀ = K·Qᵀ → online softmax per query → Oᵀ += Vᵀ·Pᵀ                       (writes lse)
//   dq  : δ = rowsum(dO∘O); Sᵀ, Pᵀ = exp(Sᵀ − lse); dPᵀ = V·dOᵀ; dSᵀ = Pᵀ(dPᵀ − δ)·s;
//         dQᵀ += Kᵀ·dSᵀ                                                         (writes δ)
//   dkv : S = Q·Kᵀ, P, dP = dO·Vᵀ, dS (per 32-query block);  dVᵀ += dOᵀ·P;  dKᵀ += Qᵀ·dS
#include "common.h"
#include "dls.h"
#include "gemm_common.h"

namespace {

constexpr int WG = 256;  // 4 waves
constexpr int RB = 32;   // rows per streamed block / per wave

template <typename T>
struct Frag {
  bf16x8 h, l;  // l: the lo plane of the fp32 split (unused for bf16)
};

template <typename T>
__device__ __forceinline__ void mma(f32x16& acc, const Frag<T>& a, const Frag<T>& b) {
  if constexpr (sizeof(T) == 4) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, acc, 0, 0, 0);
  }
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, acc, 0, 0, 0);
}

// 8 consecutive elements of a global row → an operand fragment (zeros when !ok)
template <typename T>
__device__ __forceinline__ Frag<T> frag_global(const T* p, bool ok) {
  Frag<T> f;
  if constexpr (sizeof(T) == 2) {
    uint4 u = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
    f.h = __builtin_bit_cast(bf16x8, u);
  } else {
    float x[8];
    if (ok) {
      load_vec<8>(p, x);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = 0.f;
    }
    union {
      bf16x8 v;
      bf16_t e[8];
    } hh, ll;
#pragma unroll
    for (int i = 0; i < 8; ++i) split2(x[i], hh.e[i], ll.e[i]);
    f.h = hh.v;
    f.l = ll.v;
  }
  return f;
}

// LDS images: NP planes (hi[, lo]) of [rows][ld] bf16, plane stride PS elements
template <typename T>
struct Img {
  bf16_t* p;
  int ld, ps;
};

// row-major image M[r][k]: lane ℓ gets M[r0 + ℓ&31][k0 + 8(ℓ>>5) .. +8]  (A rows / B columns)
template <typename T>
__device__ __forceinline__ Frag<T> frag_rm(const Img<T>& m, int r0, int k0) {
  const int lane = threadIdx.x & 63;
  const int off = (r0 + (lane & 31)) * m.ld + k0 + 8 * (lane >> 5);
  Frag<T> f;
  f.h = *reinterpret_cast<const bf16x8*>(m.p + off);
  if constexpr (sizeof(T) == 4) f.l = *reinterpret_cast<const bf16x8*>(m.p + m.ps + off);
  return f;
}

// k-major image M[k][r]: the same fragment of the transposed operand via ds_read_b64_tr_b16
template <typename T>
__device__ __forceinline__ Frag<T> frag_km(const Img<T>& m, int k0, int r0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = lane >> 5;
  const int o0 = (k0 + 8 * h + q) * m.ld + r0 + 16 * (g & 1) + 4 * pp, o1 = o0 + 4 * m.ld;
  Frag<T> f;
  f.h = tr_frag(m.p + o0, m.p + o1);
  if constexpr (sizeof(T) == 4) f.l = tr_frag(m.p + m.ps + o0, m.p + m.ps + o1);
  return f;
}

// Where one head's [L][DH] matrix lives: rows at stride ld, head base = (head / H)·s_kb +
// (head % H)·s_h. Contiguous [KBH][L][DH]: (H·L·DH, L·DH, DH). Packed projection output
// [KB][L][n·D] read in place (q/k/v are column blocks of the QKV GEMM's rows, o is the out
// projection's input rows): (L·ld, DH, ld) — no permute / contiguous copies around attention.
struct HeadLayout {
  long s_kb, s_h;
  int ld;
};
__device__ __forceinline__ long hbase(const HeadLayout& hl, long head, int H) {
  return (head / H) * hl.s_kb + (head % H) * hl.s_h;
}

// stage rows [r0, r0+RB) of a head matrix (row stride ld) into an image (zero rows past L)
template <typename T, int DH>
__device__ __forceinline__ void stage(const T* __restrict__ src, int ld, int r0, int L, const Img<T>& m) {
  for (int c = threadIdx.x; c < RB * DH / 8; c += WG) {
    const int r = c / (DH / 8), d = (c % (DH / 8)) * 8;
    const bool ok = r0 + r < L;
    float x[8];
    if (ok) {
      load_vec<8>(src + (long)(r0 + r) * ld + d, x);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = 0.f;
    }
    union {
      uint4 v;
      bf16_t e[8];
    } hh, ll;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (sizeof(T) == 4)
        split2(x[i], hh.e[i], ll.e[i]);
      else
        hh.e[i] = f2bf(x[i]);  // exact: x came from bf16
    }
    *reinterpret_cast<uint4*>(m.p + r * m.ld + d) = hh.v;
    if constexpr (sizeof(T) == 4) *reinterpret_cast<uint4*>(m.p + m.ps + r * m.ld + d) = ll.v;
  }
}

// C-layout tile (lane column c = ℓ&31, rows (e&3)+8(e>>2)+4(ℓ>>5)) → image M[c][row] (a
// transposed store: 4 × 8-B writes per plane)
template <typename T>
__device__ __forceinline__ void put_colrows(const Img<T>& m, const f32x16& v) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    union {
      uint2 u;
      bf16_t e[4];
    } hh, ll;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (sizeof(T) == 4)
        split2(v[4 * j + i], hh.e[i], ll.e[i]);
      else
        hh.e[i] = __builtin_bit_cast(bf16_t, (__bf16)v[4 * j + i]);
    }
    const int off = c * m.ld + 8 * j + 4 * h;
    *reinterpret_cast<uint2*>(m.p + off) = hh.u;
    if constexpr (sizeof(T) == 4) *reinterpret_cast<uint2*>(m.p + m.ps + off) = ll.u;
  }
}

// global store of a transposed accumulator tile (lane column = matrix row `row`, tile rows =
// 16 of the DH columns starting at d0): out[row][d0 + rows(e)]
template <typename T>
__device__ __forceinline__ void store_rowcols(T* out_row, int d0, const f32x16& v, float mul) {
  const int h = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float x[4] = {v[4 * j] * mul, v[4 * j + 1] * mul, v[4 * j + 2] * mul, v[4 * j + 3] * mul};
    store_vec<4>(out_row + d0 + 8 * j + 4 * h, x);
  }
}

__device__ __forceinline__ int crow(int e) { return (e & 3) + 8 * (e >> 2) + 4 * ((threadIdx.x & 63) >> 5); }

constexpr int pad_ld(int n) { return n + 8; }  // 16-B padded rows: conflict-free ds_read_b128

// ------------------------------------------------------------------------------ forward
template <typename T, int DH>
__global__ void __launch_bounds__(WG) attn_fwd_mfma_kernel(const T* __restrict__ q, const T* __restrict__ k,
                                                           const T* __restrict__ v, const int* __restrict__ key_valid,
                                                           T* __restrict__ o, float* __restrict__ lse, int L, int H,
                                                           float scale, HeadLayout lq, HeadLayout lo) {
  constexpr int NP = sizeof(T) == 4 ? 2 : 1;
  constexpr int LDK = pad_ld(DH), LDP = pad_ld(RB);
  __shared__ __attribute__((aligned(16))) bf16_t Ks[NP * RB * LDK], Vs[NP * RB * LDK];
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][NP * RB * LDP];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 31;
  const long head = blockIdx.x;
  const long base = hbase(lq, head, H), obase = hbase(lo, head, H);
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  const int qrow = blockIdx.y * (4 * RB) + wid * RB + c;
  const bool qok = qrow < L;
  const Img<T> KI{Ks, LDK, RB * LDK}, VI{Vs, LDK, RB * LDK}, PI{Ps[wid], LDP, RB * LDP};

  Frag<T> qf[DH / 16];
#pragma unroll
  for (int ks = 0; ks < DH / 16; ++ks) qf[ks] = frag_global<T>(q + base + (long)qrow * lq.ld + ks * 16 + 8 * (lane >> 5), qok);
  f32x16 ot[DH / 32];
#pragma unroll
  for (int t = 0; t < DH / 32; ++t) ot[t] = f32x16{};
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < nk; k0 += RB) {
    stage<T, DH>(k + base, lq.ld, k0, nk, KI);
    stage<T, DH>(v + base, lq.ld, k0, nk, VI);
    __syncthreads();
    f32x16 st = f32x16{};  // Sᵀ[key][query]
#pragma unroll
    for (int ks = 0; ks < DH / 16; ++ks) mma<T>(st, frag_rm<T>(KI, 0, ks * 16), qf[ks]);
    float mloc = -INFINITY;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float s = (k0 + crow(e) < nk) ? st[e] * scale : -INFINITY;
      st[e] = s;
      mloc = fmaxf(mloc, s);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float mn = fmaxf(m, mloc);
    const float corr = (m == -INFINITY) ? 0.f : __expf(m - mn);
    float ls = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float p = (st[e] == -INFINITY) ? 0.f : __expf(st[e] - mn);
      st[e] = p;
      ls += p;
    }
    ls += __shfl_xor(ls, 32, 64);
    l = l * corr + ls;
    m = mn;
#pragma unroll
    for (int t = 0; t < DH / 32; ++t) ot[t] *= corr;
    put_colrows<T>(PI, st);  // P[query][key]
    __syncthreads();
#pragma unroll
    for (int t = 0; t < DH / 32; ++t)
#pragma unroll
      for (int ks = 0; ks < RB / 16; ++ks) mma<T>(ot[t], frag_km<T>(VI, ks * 16, t * 32), frag_rm<T>(PI, 0, ks * 16));
    __syncthreads();  // K / V / P tiles are rewritten next block
  }
  if (qok) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int t = 0; t < DH / 32; ++t) store_rowcols<T>(o + obase + (long)qrow * lo.ld, t * 32, ot[t], inv);
    if ((lane >> 5) == 0) lse[head * L + qrow] = l > 0.f ? m + __logf(l) : 0.f;
  }
}

// ------------------------------------------------------------------------------ dQ
template <typename T, int DH>
__global__ void __launch_bounds__(WG) attn_bwd_dq_mfma_kernel(const T* __restrict__ dout, const T* __restrict__ q,
                                                              const T* __restrict__ k, const T* __restrict__ v,
                                                              const T* __restrict__ o, const float* __restrict__ lse,
                                                              const int* __restrict__ key_valid, T* __restrict__ dq,
                                                              float* __restrict__ delta, int L, int H, float scale,
                                                              HeadLayout lq, HeadLayout lo) {
  constexpr int NP = sizeof(T) == 4 ? 2 : 1;
  constexpr int LDK = pad_ld(DH), LDP = pad_ld(RB);
  __shared__ __attribute__((aligned(16))) bf16_t Ks[NP * RB * LDK], Vs[NP * RB * LDK];
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][NP * RB * LDP];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long head = blockIdx.x;
  const long base = hbase(lq, head, H), obase = hbase(lo, head, H);
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  const int qrow = blockIdx.y * (4 * RB) + wid * RB + c;
  const bool qok = qrow < L;
  const Img<T> KI{Ks, LDK, RB * LDK}, VI{Vs, LDK, RB * LDK}, PI{Ps[wid], LDP, RB * LDP};

  Frag<T> qf[DH / 16], df[DH / 16];
#pragma unroll
  for (int ks = 0; ks < DH / 16; ++ks) {
    qf[ks] = frag_global<T>(q + base + (long)qrow * lq.ld + ks * 16 + 8 * h, qok);
    df[ks] = frag_global<T>(dout + obase + (long)qrow * lo.ld + ks * 16 + 8 * h, qok);
  }
  // δ = dO·O of this lane's query (each half-wave sums half of the head dim)
  float dl = 0.f;
  if (qok) {
    const T* dr = dout + obase + (long)qrow * lo.ld + h * (DH / 2);
    const T* orow = o + obase + (long)qrow * lo.ld + h * (DH / 2);
#pragma unroll
    for (int d = 0; d < DH / 2; d += 8) {
      float a[8], b[8];
      load_vec<8>(dr + d, a);
      load_vec<8>(orow + d, b);
#pragma unroll
      for (int i = 0; i < 8; ++i) dl = fmaf(a[i], b[i], dl);
    }
  }
  dl += __shfl_xor(dl, 32, 64);
  if (qok && h == 0) delta[head * L + qrow] = dl;
  const float lse_q = qok ? lse[head * L + qrow] : 0.f;
  f32x16 dqt[DH / 32];
#pragma unroll
  for (int t = 0; t < DH / 32; ++t) dqt[t] = f32x16{};
  for (int k0 = 0; k0 < nk; k0 += RB) {
    stage<T, DH>(k + base, lq.ld, k0, nk, KI);
    stage<T, DH>(v + base, lq.ld, k0, nk, VI);
    __syncthreads();
    f32x16 st = f32x16{}, dpt = f32x16{};
#pragma unroll
    for (int ks = 0; ks < DH / 16; ++ks) {
      mma<T>(st, frag_rm<T>(KI, 0, ks * 16), qf[ks]);   // Sᵀ = K·Qᵀ
      mma<T>(dpt, frag_rm<T>(VI, 0, ks * 16), df[ks]);  // dPᵀ = V·dOᵀ
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const bool ok = qok && (k0 + crow(e) < nk);
      const float p = ok ? __expf(st[e] * scale - lse_q) : 0.f;
      st[e] = p * (dpt[e] - dl) * scale;  // dSᵀ
    }
    put_colrows<T>(PI, st);  // dS[query][key]
    __syncthreads();
#pragma unroll
    for (int t = 0; t < DH / 32; ++t)
#pragma unroll
      for (int ks = 0; ks < RB / 16; ++ks) mma<T>(dqt[t], frag_km<T>(KI, ks * 16, t * 32), frag_rm<T>(PI, 0, ks * 16));
    __syncthreads();
  }
  if (qok) {
#pragma unroll
    for (int t = 0; t < DH / 32; ++t) store_rowcols<T>(dq + base + (long)qrow * lq.ld, t * 32, dqt[t], 1.f);
  }
}

// ------------------------------------------------------------------------------ dK, dV
template <typename T, int DH>
__global__ void __launch_bounds__(WG) attn_bwd_dkv_mfma_kernel(const T* __restrict__ dout, const T* __restrict__ q,
                                                               const T* __restrict__ k, const T* __restrict__ v,
                                                               const float* __restrict__ lse,
                                                               const float* __restrict__ delta,
                                                               const int* __restrict__ key_valid, T* __restrict__ dk,
                                                               T* __restrict__ dv, int L, int H, float scale,
                                                               HeadLayout lq, HeadLayout lo) {
  constexpr int NP = sizeof(T) == 4 ? 2 : 1;
  constexpr int LDK = pad_ld(DH), LDP = pad_ld(RB);
  __shared__ __attribute__((aligned(16))) bf16_t Qs[NP * RB * LDK], Os[NP * RB * LDK];
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][NP * RB * LDP], Ss[4][NP * RB * LDP];
  __shared__ __attribute__((aligned(16))) float Lq[RB], Dq[RB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long head = blockIdx.x;
  const long base = hbase(lq, head, H), obase = hbase(lo, head, H);
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  const int key = blockIdx.y * (4 * RB) + wid * RB + c;
  const bool kok = key < nk;
  const Img<T> QI{Qs, LDK, RB * LDK}, OI{Os, LDK, RB * LDK};
  const Img<T> PI{Ps[wid], LDP, RB * LDP}, SI{Ss[wid], LDP, RB * LDP};

  Frag<T> kf[DH / 16], vf[DH / 16];
#pragma unroll
  for (int ks = 0; ks < DH / 16; ++ks) {
    kf[ks] = frag_global<T>(k + base + (long)key * lq.ld + ks * 16 + 8 * h, kok);
    vf[ks] = frag_global<T>(v + base + (long)key * lq.ld + ks * 16 + 8 * h, kok);
  }
  f32x16 dkt[DH / 32], dvt[DH / 32];
#pragma unroll
  for (int t = 0; t < DH / 32; ++t) dkt[t] = dvt[t] = f32x16{};
  // a workgroup whose keys are all padding still writes their zero gradients (no early exit:
  // every wave must reach every barrier)
  const bool any = blockIdx.y * (4 * RB) < nk;
  for (int q0 = 0; any && q0 < L; q0 += RB) {
    stage<T, DH>(q + base, lq.ld, q0, L, QI);
    stage<T, DH>(dout + obase, lo.ld, q0, L, OI);
    if (threadIdx.x < RB) {
      const bool ok = q0 + threadIdx.x < L;
      Lq[threadIdx.x] = ok ? lse[head * L + q0 + threadIdx.x] : 0.f;
      Dq[threadIdx.x] = ok ? delta[head * L + q0 + threadIdx.x] : 0.f;
    }
    __syncthreads();
    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int ks = 0; ks < DH / 16; ++ks) {
      mma<T>(s, frag_rm<T>(QI, 0, ks * 16), kf[ks]);   // S = Q·Kᵀ   [query][key]
      mma<T>(dp, frag_rm<T>(OI, 0, ks * 16), vf[ks]);  // dP = dO·Vᵀ [query][key]
    }
    f32x16 ds;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int qr = crow(e);
      const bool ok = kok && (q0 + qr < L);
      const float p = ok ? __expf(s[e] * scale - Lq[qr]) : 0.f;
      s[e] = p;
      ds[e] = p * (dp[e] - Dq[qr]) * scale;
    }
    put_colrows<T>(PI, s);   // P[key][query]
    put_colrows<T>(SI, ds);  // dS[key][query]
    __syncthreads();
#pragma unroll
    for (int t = 0; t < DH / 32; ++t)
#pragma unroll
      for (int ks = 0; ks < RB / 16; ++ks) {
        mma<T>(dvt[t], frag_km<T>(OI, ks * 16, t * 32), frag_rm<T>(PI, 0, ks * 16));  // dVᵀ += dOᵀ·P
        mma<T>(dkt[t], frag_km<T>(QI, ks * 16, t * 32), frag_rm<T>(SI, 0, ks * 16));  // dKᵀ += Qᵀ·dS
      }
    __syncthreads();
  }
  if (key < L) {
#pragma unroll
    for (int t = 0; t < DH / 32; ++t) {
      store_rowcols<T>(dk + base + (long)key * lq.ld, t * 32, dkt[t], 1.f);
      store_rowcols<T>(dv + base + (long)key * lq.ld, t * 32, dvt[t], 1.f);
    }
  }
}

#define MFMA_DH(DHV, CALL) \
  switch (DHV) {           \
    case 32: {             \
      constexpr int D = 32; \
      CALL;                \
    } break;               \
    case 64: {             \
      constexpr int D = 64; \
      CALL;                \
    } break;               \
    default: return false; \
  }

#define DISPATCH_T(F32, ...) \
  if (F32) {                 \
    typedef float TT;        \
    __VA_ARGS__;             \
  } else {                   \
    typedef bf16_t TT;       \
    __VA_ARGS__;             \
  }
#define CP(p) static_cast<const TT*>(p)
#define MP(p) static_cast<TT*>(p)

}  // namespace

bool attn_mfma_supported(int L, int DH) { return (DH == 32 || DH == 64) && L >= 1; }

// ldqkv / ldo = 0: contiguous [KBH][L][DH]; otherwise packed [KB][L][ld] rows (module docs)
static HeadLayout head_layout(int ld, int H, int L, int DH) {
  if (ld == 0) return HeadLayout{(long)H * L * DH, (long)L * DH, DH};
  return HeadLayout{(long)L * ld, (long)DH, ld};
}

bool attn_fwd_mfma(const void* q, const void* k, const void* v, const int* key_valid, void* o, float* lse, long KBH,
                   int H, int L, int DH, int f32, hipStream_t s, int ldqkv, int ldo) {
  if (!attn_mfma_supported(L, DH)) return false;
  const dim3 grid((unsigned)KBH, cdiv(L, 4 * RB));
  const float scale = 1.0f / sqrtf((float)DH);
  const HeadLayout lq = head_layout(ldqkv, H, L, DH), lo = head_layout(ldo, H, L, DH);
  DISPATCH_T(f32, MFMA_DH(DH, hipLaunchKernelGGL((attn_fwd_mfma_kernel<TT, D>), grid, dim3(WG), 0, s, CP(q), CP(k),
                                                 CP(v), key_valid, MP(o), lse, L, H, scale, lq, lo)));
  return true;
}

bool attn_bwd_mfma(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                   const int* key_valid, void* dq, void* dk, void* dv, float* delta, long KBH, int H, int L, int DH,
                   int f32, hipStream_t s, int ldqkv, int ldo) {
  if (!attn_mfma_supported(L, DH)) return false;
  const dim3 grid((unsigned)KBH, cdiv(L, 4 * RB));
  const float scale = 1.0f / sqrtf((float)DH);
  const HeadLayout lq = head_layout(ldqkv, H, L, DH), lo = head_layout(ldo, H, L, DH);
  DISPATCH_T(f32, MFMA_DH(DH, hipLaunchKernelGGL((attn_bwd_dq_mfma_kernel<TT, D>), grid, dim3(WG), 0, s, CP(dout),
                                                 CP(q), CP(k), CP(v), CP(o), lse, key_valid, MP(dq), delta, L, H,
                                                 scale, lq, lo)));
  DISPATCH_T(f32, MFMA_DH(DH, hipLaunchKernelGGL((attn_bwd_dkv_mfma_kernel<TT, D>), grid, dim3(WG), 0, s, CP(dout),
                                                 CP(q), CP(k), CP(v), lse, delta, key_valid, MP(dk), MP(dv), L, H,
                                                 scale, lq, lo)));
  return true;
}
