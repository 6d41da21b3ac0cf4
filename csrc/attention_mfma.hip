// Multi-head attention fwd / bwd on the MFMA (gfx950), any head dim ≤ 64 with dh % 4 == 0 (run at
// the padded width 32 or 64: zero columns past dh, so e.g. the reference imdb model's dh = 20
// runs here instead of the VALU kernels), any sequence length, optional dropout on the attention
// probabilities (nn.MultiheadAttention's `dropout`, inside nn.TransformerEncoderLayer).
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
// Dropout (p > 0): P̃ = P∘M/(1−p) with M the keep mask hash(head, query, key) of the client's
// seed — the same mask in all three kernels and in ops/ref.py. The forward normalises with the
// undropped P (l, lse) and accumulates O = P̃V; the backward uses dP = (dO·Vᵀ)∘M/(1−p) in
// dS = P∘(dP − δ) with δ = rowsum(dO∘O), and dV = P̃ᵀdO.
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

// up to 8 consecutive elements of a global row (n valid, n % 4 == 0; the rest read as zeros)
template <typename T>
__device__ __forceinline__ void load8n(const T* p, int n, float* x) {
  if (n >= 8) {
    // (two 4-element loads: a dh = 20 head's bf16 rows are only 8-B aligned)
    load_vec<4>(p, x);
    load_vec<4>(p + 4, x + 4);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = 0.f;
    if (n >= 4) load_vec<4>(p, x);
  }
}

// 8 consecutive elements of a global row → an operand fragment (n valid: zeros beyond)
template <typename T>
__device__ __forceinline__ Frag<T> frag_global(const T* p, int n) {
  Frag<T> f;
  if constexpr (sizeof(T) == 2) {
    uint4 u = make_uint4(0, 0, 0, 0);
    if (n >= 8) {
      const uint2 a = *reinterpret_cast<const uint2*>(p), b = *reinterpret_cast<const uint2*>(p + 4);
      u = make_uint4(a.x, a.y, b.x, b.y);
    } else if (n >= 4) {
      const uint2 h = *reinterpret_cast<const uint2*>(p);
      u.x = h.x;
      u.y = h.y;
    }
    f.h = __builtin_bit_cast(bf16x8, u);
  } else {
    float x[8];
    load8n(p, n, x);
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

// Staging rows [r0, r0+RB) of a head matrix (row stride ld, DH real columns) into an image of DP
// padded columns (zero rows past L, zero columns past DH): `stage` in one go, or split in two
// (DP ≤ 64: one 8-column chunk per thread at most): stage_load fills the thread's chunk,
// stage_store splits it into the image. (Issuing the next block's stage_load under the current
// block's MFMAs cost the backward kernels the registers of their second / third workgroup per CU,
// which hides that latency better: profiles/r6_c13_attn_occupancy.log)
template <typename T, int DH, int DP>
__device__ __forceinline__ void stage(const T* __restrict__ src, int ld, int r0, int L, const Img<T>& m) {
  for (int c = threadIdx.x; c < RB * DP / 8; c += WG) {
    const int r = c / (DP / 8), d = (c % (DP / 8)) * 8;
    const int n = r0 + r < L ? min(8, max(0, DH - d)) : 0;
    float x[8];
    load8n(src + (long)(r0 + r) * ld + d, n, x);
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
template <typename T, int DH, int DP>
__device__ __forceinline__ void stage_load(const T* __restrict__ src, int ld, int r0, int L, float (&x)[8]) {
  static_assert(RB * DP / 8 <= WG, "one chunk per thread");
  const int c = threadIdx.x;
  if (c < RB * DP / 8) {
    const int r = c / (DP / 8), d = (c % (DP / 8)) * 8;
    const int n = r0 + r < L ? min(8, max(0, DH - d)) : 0;
    load8n(src + (long)(r0 + r) * ld + d, n, x);
  }
}
template <typename T, int DP>
__device__ __forceinline__ void stage_store(const float (&x)[8], const Img<T>& m) {
  const int c = threadIdx.x;
  if (c < RB * DP / 8) {
    const int r = c / (DP / 8), d = (c % (DP / 8)) * 8;
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
// (writing the outputs' split planes here for the projections' plane GEMMs measured +0.4-0.5 s
// per FedOBD Transformer round each for o and dqkv — their stores cost more than the plane GEMMs
// gain at d 512, profiles/r5_c6_ab_tfm_planes.txt — and was removed)
template <typename T, int DH>
__device__ __forceinline__ void store_rowcols(T* out_row, int d0, const f32x16& v, float mul) {
  const int h = (threadIdx.x & 63) >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float x[4] = {v[4 * j] * mul, v[4 * j + 1] * mul, v[4 * j + 2] * mul, v[4 * j + 3] * mul};
    const int d = d0 + 8 * j + 4 * h;
    if (d < DH) {
      store_vec<4>(out_row + d, x);  // (DH % 4 == 0)
    }
  }
}

// attention-probability dropout of one score (client seed, head within the client, query, key)
struct AttnDropArgs {
  const uint32_t* seeds;  // [clients]; nullptr = no dropout
  int hpc;                // heads per client (B·H)
  float p;
};
__device__ __forceinline__ float attn_keep(const AttnDropArgs& d, long head, int L, int qi, int kj) {
  const uint32_t seed = d.seeds[head / d.hpc];
  const uint32_t idx = (uint32_t)(((long)(head % d.hpc) * L + qi) * L + kj);
  const uint32_t thr = (uint32_t)fminf(d.p * 4294967296.f, 4294967040.f);
  return mix32(idx, seed) >= thr ? 1.f / (1.f - d.p) : 0.f;
}

__device__ __forceinline__ int crow(int e) { return (e & 3) + 8 * (e >> 2) + 4 * ((threadIdx.x & 63) >> 5); }

constexpr int pad_ld(int n) { return n + 8; }  // 16-B padded rows: conflict-free ds_read_b128

// ------------------------------------------------------------------------------ forward
// four workgroups per CU (127 VGPRs at dh 64, none spilled; the fp32 dh-48 build would spill at
// four and keeps three)
template <typename T, int DH, int DP>
__global__ void __launch_bounds__(WG, (sizeof(T) == 4 && DH == 48) ? 3 : 4) attn_fwd_mfma_kernel(const T* __restrict__ q, const T* __restrict__ k,
                                                           const T* __restrict__ v, const int* __restrict__ key_valid,
                                                           T* __restrict__ o, float* __restrict__ lse, int L, int H,
                                                           float scale, HeadLayout lq, HeadLayout lo,
                                                           AttnDropArgs dr) {
  constexpr int NP = sizeof(T) == 4 ? 2 : 1;
  constexpr int LDK = pad_ld(DP), LDP = pad_ld(RB);
  __shared__ __attribute__((aligned(16))) bf16_t Ks[NP * RB * LDK], Vs[NP * RB * LDK];
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][NP * RB * LDP];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 31;
  const long head = blockIdx.x;
  const long base = hbase(lq, head, H), obase = hbase(lo, head, H);
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  const int qrow = blockIdx.y * (4 * RB) + wid * RB + c;
  const bool qok = qrow < L;
  const bool drop = dr.seeds != nullptr && dr.p > 0.f;
  const Img<T> KI{Ks, LDK, RB * LDK}, VI{Vs, LDK, RB * LDK}, PI{Ps[wid], LDP, RB * LDP};

  Frag<T> qf[DP / 16];
#pragma unroll
  for (int ks = 0; ks < DP / 16; ++ks) {
    const int d = ks * 16 + 8 * (lane >> 5);
    qf[ks] = frag_global<T>(q + base + (long)qrow * lq.ld + d, qok ? min(8, max(0, DH - d)) : 0);
  }
  f32x16 ot[DP / 32];
#pragma unroll
  for (int t = 0; t < DP / 32; ++t) ot[t] = f32x16{};
  float m = -INFINITY, l = 0.f;
  // (no register prefetch of the next block here: it costs this kernel a wave per SIMD, 3 → 2)
  for (int k0 = 0; k0 < nk; k0 += RB) {
    stage<T, DH, DP>(k + base, lq.ld, k0, nk, KI);
    stage<T, DH, DP>(v + base, lq.ld, k0, nk, VI);
    __syncthreads();
    f32x16 st = f32x16{};  // Sᵀ[key][query]
#pragma unroll
    for (int ks = 0; ks < DP / 16; ++ks) mma<T>(st, frag_rm<T>(KI, 0, ks * 16), qf[ks]);
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
      ls += p;  // (the normaliser sums the undropped probabilities)
      st[e] = (drop && p != 0.f) ? p * attn_keep(dr, head, L, qrow, k0 + crow(e)) : p;
    }
    ls += __shfl_xor(ls, 32, 64);
    l = l * corr + ls;
    m = mn;
#pragma unroll
    for (int t = 0; t < DP / 32; ++t) ot[t] *= corr;
    put_colrows<T>(PI, st);  // P̃[query][key]
    __syncthreads();
#pragma unroll
    for (int t = 0; t < DP / 32; ++t)
#pragma unroll
      for (int ks = 0; ks < RB / 16; ++ks) mma<T>(ot[t], frag_km<T>(VI, ks * 16, t * 32), frag_rm<T>(PI, 0, ks * 16));
    __syncthreads();  // K / V / P tiles are rewritten next block
  }
  if (qok) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int t = 0; t < DP / 32; ++t)
      store_rowcols<T, DH>(o + obase + (long)qrow * lo.ld, t * 32, ot[t], inv);
    if ((lane >> 5) == 0) lse[head * L + qrow] = l > 0.f ? m + __logf(l) : 0.f;
  }
}

// ------------------------------------------------------------------------------ dQ
// three workgroups per CU, the key block loaded at its step (as the dK/dV kernel: 1.93 → 1.85 ms)
template <typename T, int DH, int DP>
__global__ void __launch_bounds__(WG, 3) attn_bwd_dq_mfma_kernel(const T* __restrict__ dout, const T* __restrict__ q,
                                                              const T* __restrict__ k, const T* __restrict__ v,
                                                              const T* __restrict__ o, const float* __restrict__ lse,
                                                              const int* __restrict__ key_valid, T* __restrict__ dq,
                                                              float* __restrict__ delta, int L, int H, float scale,
                                                              HeadLayout lq, HeadLayout lo, AttnDropArgs dr) {
  constexpr int NP = sizeof(T) == 4 ? 2 : 1;
  constexpr int LDK = pad_ld(DP), LDP = pad_ld(RB);
  __shared__ __attribute__((aligned(16))) bf16_t Ks[NP * RB * LDK], Vs[NP * RB * LDK];
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][NP * RB * LDP];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long head = blockIdx.x;
  const long base = hbase(lq, head, H), obase = hbase(lo, head, H);
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  const int qrow = blockIdx.y * (4 * RB) + wid * RB + c;
  const bool qok = qrow < L;
  const bool drop = dr.seeds != nullptr && dr.p > 0.f;
  const Img<T> KI{Ks, LDK, RB * LDK}, VI{Vs, LDK, RB * LDK}, PI{Ps[wid], LDP, RB * LDP};

  Frag<T> qf[DP / 16], df[DP / 16];
#pragma unroll
  for (int ks = 0; ks < DP / 16; ++ks) {
    const int d = ks * 16 + 8 * h, n = qok ? min(8, max(0, DH - d)) : 0;
    qf[ks] = frag_global<T>(q + base + (long)qrow * lq.ld + d, n);
    df[ks] = frag_global<T>(dout + obase + (long)qrow * lo.ld + d, n);
  }
  // δ = dO·O of this lane's query (the two half-waves take alternate 4-column chunks)
  float dl = 0.f;
  if (qok) {
    const T* dr_ = dout + obase + (long)qrow * lo.ld;
    const T* orow = o + obase + (long)qrow * lo.ld;
#pragma unroll
    for (int d = 4 * h; d < DH; d += 8) {
      float a[4], b[4];
      load_vec<4>(dr_ + d, a);
      load_vec<4>(orow + d, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) dl = fmaf(a[i], b[i], dl);
    }
  }
  dl += __shfl_xor(dl, 32, 64);
  if (qok && h == 0) delta[head * L + qrow] = dl;
  const float lse_q = qok ? lse[head * L + qrow] : 0.f;
  f32x16 dqt[DP / 32];
#pragma unroll
  for (int t = 0; t < DP / 32; ++t) dqt[t] = f32x16{};
  float kx[8], vx[8];
  for (int k0 = 0; k0 < nk; k0 += RB) {
    stage_load<T, DH, DP>(k + base, lq.ld, k0, nk, kx);
    stage_load<T, DH, DP>(v + base, lq.ld, k0, nk, vx);
    stage_store<T, DP>(kx, KI);
    stage_store<T, DP>(vx, VI);
    __syncthreads();
    f32x16 st = f32x16{}, dpt = f32x16{};
#pragma unroll
    for (int ks = 0; ks < DP / 16; ++ks) {
      mma<T>(st, frag_rm<T>(KI, 0, ks * 16), qf[ks]);   // Sᵀ = K·Qᵀ
      mma<T>(dpt, frag_rm<T>(VI, 0, ks * 16), df[ks]);  // dP̃ᵀ = V·dOᵀ
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const bool ok = qok && (k0 + crow(e) < nk);
      const float p = ok ? __expf(st[e] * scale - lse_q) : 0.f;
      const float dp = (drop && p != 0.f) ? dpt[e] * attn_keep(dr, head, L, qrow, k0 + crow(e)) : dpt[e];
      st[e] = p * (dp - dl) * scale;  // dSᵀ
    }
    put_colrows<T>(PI, st);  // dS[query][key]
    __syncthreads();
#pragma unroll
    for (int t = 0; t < DP / 32; ++t)
#pragma unroll
      for (int ks = 0; ks < RB / 16; ++ks) mma<T>(dqt[t], frag_km<T>(KI, ks * 16, t * 32), frag_rm<T>(PI, 0, ks * 16));
    __syncthreads();
  }
  if (qok) {
#pragma unroll
    for (int t = 0; t < DP / 32; ++t)
      store_rowcols<T, DH>(dq + base + (long)qrow * lq.ld, t * 32, dqt[t], 1.f);
  }
}

// ------------------------------------------------------------------------------ dK, dV
// The lane's K / V fragments stay in registers for the whole kernel (at fp32 dh 64: 64 VGPRs, one
// wave per SIMD). Re-reading them per query block instead (two waves per SIMD) measured 2.73 →
// 2.23 ms per launch alone but 22.40 → 22.62 s per FedOBD stage-1 round beside the other
// sub-cohort's GEMMs (profiles/r5_c10_ab_attn_dkv_reload.txt): removed.
// two workgroups per CU (≤ 256 registers per lane, a few spilled): with one, every barrier of the
// 3-barrier query-block step stalled its CU. The query block is loaded at its step, not a step
// ahead — the other workgroup covers the load, and the look-ahead registers would spill more
// (2.56 → 1.92 ms per backward at 25 clients × 64 × 8 heads × 128², profiles/r6_c13_attn_occupancy.log)
template <typename T, int DH, int DP>
__global__ void __launch_bounds__(WG, 2) attn_bwd_dkv_mfma_kernel(const T* __restrict__ dout, const T* __restrict__ q,
                                                               const T* __restrict__ k, const T* __restrict__ v,
                                                               const float* __restrict__ lse,
                                                               const float* __restrict__ delta,
                                                               const int* __restrict__ key_valid, T* __restrict__ dk,
                                                               T* __restrict__ dv, int L, int H, float scale,
                                                               HeadLayout lq, HeadLayout lo, AttnDropArgs dr) {
  constexpr int NP = sizeof(T) == 4 ? 2 : 1;
  constexpr int LDK = pad_ld(DP), LDP = pad_ld(RB);
  __shared__ __attribute__((aligned(16))) bf16_t Qs[NP * RB * LDK], Os[NP * RB * LDK];
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][NP * RB * LDP], Ss[4][NP * RB * LDP];
  __shared__ __attribute__((aligned(16))) float Lq[RB], Dq[RB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long head = blockIdx.x;
  const long base = hbase(lq, head, H), obase = hbase(lo, head, H);
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  const int key = blockIdx.y * (4 * RB) + wid * RB + c;
  const bool kok = key < nk;
  const bool drop = dr.seeds != nullptr && dr.p > 0.f;
  const Img<T> QI{Qs, LDK, RB * LDK}, OI{Os, LDK, RB * LDK};
  const Img<T> PI{Ps[wid], LDP, RB * LDP}, SI{Ss[wid], LDP, RB * LDP};

  Frag<T> kf[DP / 16], vf[DP / 16];
#pragma unroll
  for (int ks = 0; ks < DP / 16; ++ks) {
    const int d = ks * 16 + 8 * h, n = kok ? min(8, max(0, DH - d)) : 0;
    kf[ks] = frag_global<T>(k + base + (long)key * lq.ld + d, n);
    vf[ks] = frag_global<T>(v + base + (long)key * lq.ld + d, n);
  }
  f32x16 dkt[DP / 32], dvt[DP / 32];
#pragma unroll
  for (int t = 0; t < DP / 32; ++t) dkt[t] = dvt[t] = f32x16{};
  // a workgroup whose keys are all padding still writes their zero gradients (no early exit:
  // every wave must reach every barrier)
  const bool any = blockIdx.y * (4 * RB) < nk;
  float qx[8], ox[8], lq_r = 0.f, dq_r = 0.f;
  auto load_qblock = [&](int q0) {
    stage_load<T, DH, DP>(q + base, lq.ld, q0, L, qx);
    stage_load<T, DH, DP>(dout + obase, lo.ld, q0, L, ox);
    if (threadIdx.x < RB) {
      const bool ok = q0 + threadIdx.x < L;
      lq_r = ok ? lse[head * L + q0 + threadIdx.x] : 0.f;
      dq_r = ok ? delta[head * L + q0 + threadIdx.x] : 0.f;
    }
  };
  for (int q0 = 0; any && q0 < L; q0 += RB) {
    load_qblock(q0);
    stage_store<T, DP>(qx, QI);
    stage_store<T, DP>(ox, OI);
    if (threadIdx.x < RB) {
      Lq[threadIdx.x] = lq_r;
      Dq[threadIdx.x] = dq_r;
    }
    __syncthreads();
    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int ks = 0; ks < DP / 16; ++ks) {
      mma<T>(s, frag_rm<T>(QI, 0, ks * 16), kf[ks]);   // S = Q·Kᵀ   [query][key]
      mma<T>(dp, frag_rm<T>(OI, 0, ks * 16), vf[ks]);  // dP̃ = dO·Vᵀ [query][key]
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int qr = crow(e);
      const bool ok = kok && (q0 + qr < L);
      const float p = ok ? __expf(s[e] * scale - Lq[qr]) : 0.f;
      const float mk = (drop && p != 0.f) ? attn_keep(dr, head, L, q0 + qr, key) : 1.f;
      s[e] = p * mk;                              // P̃ (dV)
      dp[e] = p * (dp[e] * mk - Dq[qr]) * scale;  // dS = P∘(dP − δ), in place
    }
    put_colrows<T>(PI, s);   // P̃[key][query]
    put_colrows<T>(SI, dp);  // dS[key][query]
    __syncthreads();
#pragma unroll
    for (int t = 0; t < DP / 32; ++t)
#pragma unroll
      for (int ks = 0; ks < RB / 16; ++ks) {
        mma<T>(dvt[t], frag_km<T>(OI, ks * 16, t * 32), frag_rm<T>(PI, 0, ks * 16));  // dVᵀ += dOᵀ·P̃
        mma<T>(dkt[t], frag_km<T>(QI, ks * 16, t * 32), frag_rm<T>(SI, 0, ks * 16));  // dKᵀ += Qᵀ·dS
      }
    __syncthreads();
  }
  if (key < L) {
#pragma unroll
    for (int t = 0; t < DP / 32; ++t) {
      store_rowcols<T, DH>(dk + base + (long)key * lq.ld, t * 32, dkt[t], 1.f);
      store_rowcols<T, DH>(dv + base + (long)key * lq.ld, t * 32, dvt[t], 1.f);
    }
  }
}

// (logical head dim, padded MFMA width) pairs compiled
#define MFMA_DH(DHV, CALL)                      \
  switch (DHV) {                                \
    case 8: {                                   \
      constexpr int D = 8, DPAD = 32;           \
      CALL;                                     \
    } break;                                    \
    case 16: {                                  \
      constexpr int D = 16, DPAD = 32;          \
      CALL;                                     \
    } break;                                    \
    case 20: {                                  \
      constexpr int D = 20, DPAD = 32;          \
      CALL;                                     \
    } break;                                    \
    case 32: {                                  \
      constexpr int D = 32, DPAD = 32;          \
      CALL;                                     \
    } break;                                    \
    case 48: {                                  \
      constexpr int D = 48, DPAD = 64;          \
      CALL;                                     \
    } break;                                    \
    case 64: {                                  \
      constexpr int D = 64, DPAD = 64;          \
      CALL;                                     \
    } break;                                    \
    default: return false;                      \
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

bool attn_mfma_supported(int L, int DH) {
  return (DH == 8 || DH == 16 || DH == 20 || DH == 32 || DH == 48 || DH == 64) && L >= 1;
}

// ldqkv / ldo = 0: contiguous [KBH][L][DH]; otherwise packed [KB][L][ld] rows (module docs)
static HeadLayout head_layout(int ld, int H, int L, int DH) {
  if (ld == 0) return HeadLayout{(long)H * L * DH, (long)L * DH, DH};
  return HeadLayout{(long)L * ld, (long)DH, ld};
}

bool attn_fwd_mfma(const void* q, const void* k, const void* v, const int* key_valid, void* o, float* lse, long KBH,
                   int H, int L, int DH, int f32, hipStream_t s, int ldqkv, int ldo, const uint32_t* drop_seeds,
                   int heads_per_client, float drop_p) {
  if (!attn_mfma_supported(L, DH)) return false;
  const dim3 grid((unsigned)KBH, cdiv(L, 4 * RB));
  const float scale = 1.0f / sqrtf((float)DH);
  const HeadLayout lq = head_layout(ldqkv, H, L, DH), lo = head_layout(ldo, H, L, DH);
  const int hpc = heads_per_client > 0 ? heads_per_client : 1;
  const AttnDropArgs dr{drop_p > 0.f ? drop_seeds : nullptr, hpc, drop_p};
  DISPATCH_T(f32, MFMA_DH(DH, hipLaunchKernelGGL((attn_fwd_mfma_kernel<TT, D, DPAD>), grid, dim3(WG), 0, s, CP(q),
                                                 CP(k), CP(v), key_valid, MP(o), lse, L, H, scale, lq, lo, dr)));
  return true;
}

bool attn_bwd_mfma(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                   const int* key_valid, void* dq, void* dk, void* dv, float* delta, long KBH, int H, int L, int DH,
                   int f32, hipStream_t s, int ldqkv, int ldo, const uint32_t* drop_seeds, int heads_per_client,
                   float drop_p) {
  if (!attn_mfma_supported(L, DH)) return false;
  const dim3 grid((unsigned)KBH, cdiv(L, 4 * RB));
  const float scale = 1.0f / sqrtf((float)DH);
  const HeadLayout lq = head_layout(ldqkv, H, L, DH), lo = head_layout(ldo, H, L, DH);
  const int hpc = heads_per_client > 0 ? heads_per_client : 1;
  const AttnDropArgs dr{drop_p > 0.f ? drop_seeds : nullptr, hpc, drop_p};
  DISPATCH_T(f32, MFMA_DH(DH, hipLaunchKernelGGL((attn_bwd_dq_mfma_kernel<TT, D, DPAD>), grid, dim3(WG), 0, s,
                                                 CP(dout), CP(q), CP(k), CP(v), CP(o), lse, key_valid, MP(dq), delta,
                                                 L, H, scale, lq, lo, dr)));
  DISPATCH_T(f32, MFMA_DH(DH, hipLaunchKernelGGL((attn_bwd_dkv_mfma_kernel<TT, D, DPAD>), grid, dim3(WG), 0, s,
                                                 CP(dout), CP(q), CP(k), CP(v), lse, delta, key_valid, MP(dk), MP(dv),
                                                 L, H, scale, lq, lo, dr)));
  return true;
}
