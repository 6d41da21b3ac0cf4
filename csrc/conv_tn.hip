// Client-batched weight gradient, "TN" form, for gfx950 (MI355X, CDNA4).
//
//   dW[co][r] = Σ_m dY[m][co] · im2col(X)[m][r]      (conv: r = (kh, kw, ci); linear: KH=KW=1)
//
// The pixel reduction (m) is the slow axis of both operands, so both tiles are staged k-major
// in LDS (row stride ≡ 64 mod 256 B ⇒ conflict-free) and MFMA fragments come from
// ds_read_b64_tr_b16 hardware-transposed reads. Split-K over pixels with fp32 atomics into
// the (pre-zeroed) flat gradient buffer when the (client, co, r) tile count alone cannot fill
// 256 CUs; pixel index decomposition by multiply-high (FastDiv). DEPTH=2 (two K tiles in
// registers) is kept selectable but measured slower: it costs the second wave per SIMD.
#include "dls.h"
#include "gemm_common.h"

namespace {

constexpr int BKT = 64;  // pixel (reduction) tile

template <int BMc, int BNr, int VA, int VB, int DEPTH>
__global__ void __launch_bounds__(256) conv_tn_kernel(ConvTNParams p) {
  constexpr int T = 256;
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BMc / (WM * 32), TN = BNr / (WN * 32);
  constexpr int LDA = BMc + 32;
  constexpr int LDB = BNr + 32;
  constexpr int CCA = BMc / VA, RPA = T / CCA, PA = BKT / RPA;
  constexpr int CCB = BNr / VB, RPB = T / CCB, PB = BKT / RPB;
  static_assert(PA >= 1 && PB >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) bf16_t As[2][BKT][LDA];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BKT][LDB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tilesM = (p.Co + BMc - 1) / BMc, tilesN = (p.R + BNr - 1) / BNr;
  const int per_client = tilesM * tilesN * p.splitk;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  int t = bid % per_client;
  const int split = t % p.splitk;
  t /= p.splitk;
  const int co0 = (t / tilesN) * BMc, r0 = (t % tilesN) * BNr;
  const int mbeg = split * p.m_per_split;
  const int mend = min(p.M, mbeg + p.m_per_split);

  const bf16_t* __restrict__ dy = p.dy + (long)client * p.dy_cs;
  const bf16_t* __restrict__ x = p.x + (long)client * p.x_cs;

  // B-side (im2col) column decomposition is fixed per thread
  const int cb = tid % CCB;
  const int rcol = r0 + cb * VB;
  const bool rok = rcol < p.R;
  int kh = 0, kw = 0, c = 0;
  if (rok) {
    kh = rcol / (p.KW * p.C);
    const int rr = rcol - kh * p.KW * p.C;
    kw = rr / p.C;
    c = rr - kw * p.C;
  }
  const int ca = tid % CCA;
  const int cocol = co0 + ca * VA;
  const bool cok = cocol < p.Co;

  typedef typename VecT<VA>::T TA;
  typedef typename VecT<VB>::T TB;
  TA ra0[PA], ra1[PA];
  TB rb0[PB], rb1[PB];
  int k_next = mbeg;
  auto load_into = [&](TA* ra, TB* rb) {
    const int k0 = k_next;
    k_next += BKT;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int m = k0 + tid / CCA + j * RPA;
      ra[j] = vzero<VA>();
      if (cok && m < mend) ra[j] = *reinterpret_cast<const TA*>(dy + (long)m * p.Co + cocol);
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int m = k0 + tid / CCB + j * RPB;
      rb[j] = vzero<VB>();
      if (!(rok && m < mend)) continue;
      const uint32_t b = fdiv(m, p.fd_ohw);
      const uint32_t rem = m - b * p.OH * p.OW;
      const uint32_t oh = fdiv(rem, p.fd_ow);
      const uint32_t ow = rem - oh * p.OW;
      const int ih = (int)oh * p.stride - p.pad + kh, iw = (int)ow * p.stride - p.pad + kw;
      if (ih < 0 || ih >= p.H || iw < 0 || iw >= p.W) continue;
      rb[j] = *reinterpret_cast<const TB*>(x + (((long)b * p.H + ih) * p.W + iw) * p.C + c);
    }
  };
  auto store_from = [&](const TA* ra, const TB* rb, int buf) {
#pragma unroll
    for (int j = 0; j < PA; ++j) *reinterpret_cast<TA*>(&As[buf][tid / CCA + j * RPA][ca * VA]) = ra[j];
#pragma unroll
    for (int j = 0; j < PB; ++j) *reinterpret_cast<TB*>(&Bs[buf][tid / CCB + j * RPB][cb * VB]) = rb[j];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const int wm0 = (wid / WN) * (TM * 32), wn0 = (wid % WN) * (TN * 32);
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = lane >> 5;
  auto compute = [&](int buf) {
#pragma unroll
    for (int ks = 0; ks < BKT / 16; ++ks) {
      bf16x8 af[TM], bfr[TN];
      const int krow = ks * 16 + 8 * h + q;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm0 + i * 32 + 16 * (g & 1) + 4 * pp;
        af[i] = tr_frag(&As[buf][krow][col], &As[buf][krow + 4][col]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn0 + j * 32 + 16 * (g & 1) + 4 * pp;
        bfr[j] = tr_frag(&Bs[buf][krow][col], &Bs[buf][krow + 4][col]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = (mend - mbeg + BKT - 1) / BKT;
  if (nk <= 0) return;
  if constexpr (DEPTH == 1) {
    load_into(ra0, rb0);
    store_from(ra0, rb0, 0);
    __syncthreads();
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load_into(ra0, rb0);
      compute(buf);
      if (kt + 1 < nk) store_from(ra0, rb0, buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  } else {
    load_into(ra0, rb0);
    if (nk > 1) load_into(ra1, rb1);
    store_from(ra0, rb0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      if (kt + 2 < nk) load_into(ra0, rb0);
      compute(0);
      if (kt + 1 < nk) store_from(ra1, rb1, 1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      if (kt + 3 < nk) load_into(ra1, rb1);
      compute(1);
      if (kt + 2 < nk) store_from(ra0, rb0, 0);
      __syncthreads();
    }
  }

  float* __restrict__ dw = p.dw + (long)client * p.dw_cs;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int r = r0 + wn0 + j * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wm0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (co < p.Co && r < p.R) {
          float* dst = dw + (long)co * p.R + r;
          if (p.splitk > 1)
            atomicAdd(dst, acc[i][j][e]);
          else
            *dst = acc[i][j][e];
        }
      }
    }
  }
}

template <int BMc, int BNr>
void launch_tn_v(const ConvTNParams& p, int va, int vb, int grid, hipStream_t s) {
#define TN_CASE(A, B)                                                                          \
  if (va == A && vb == B) {                                                                    \
    hipLaunchKernelGGL((conv_tn_kernel<BMc, BNr, A, B, 1>), dim3(grid), dim3(256), 0, s, p); \
    return;                                                                                    \
  }
  TN_CASE(8, 8) TN_CASE(4, 4) TN_CASE(1, 1) TN_CASE(8, 4) TN_CASE(4, 8) TN_CASE(8, 1) TN_CASE(1, 8) TN_CASE(4, 1)
  TN_CASE(1, 4)
#undef TN_CASE
  fprintf(stderr, "conv_tn: unsupported vector widths %d %d\n", va, vb);
}

int vec_width(int c) { return (c % 8 == 0) ? 8 : (c % 4 == 0) ? 4 : 1; }

void tn_split(int K, int Co, int R, int M, int& splitk, int& mps) {
  const int BMc = Co <= 64 ? 64 : 128, BNr = 128;
  const long tiles = (long)K * cdiv(Co, BMc) * cdiv(R, BNr);
  splitk = 1;
  const int target = 1024;  // >= 4 blocks per CU
  if (tiles < target) {
    splitk = (int)((target + tiles - 1) / tiles);
    splitk = min(splitk, max(1, M / (4 * BKT)));
  }
  mps = cdiv(M, splitk);
  mps = ((mps + BKT - 1) / BKT) * BKT;
  splitk = cdiv(M, mps);
}

}  // namespace

void conv_tn(ConvTNParams p, int K, hipStream_t s) {
  p.fd_ohw = make_fastdiv((uint32_t)(p.OH * p.OW));
  p.fd_ow = make_fastdiv((uint32_t)p.OW);
  const int va = vec_width(p.Co);
  const int vb = vec_width(p.C);
  const bool small_m = p.Co <= 64;
  tn_split(K, p.Co, p.R, p.M, p.splitk, p.m_per_split);
  const long tiles = (long)K * cdiv(p.Co, small_m ? 64 : 128) * cdiv(p.R, 128);
  const int grid = (int)(tiles * p.splitk);
  if (small_m)
    launch_tn_v<64, 128>(p, va, vb, grid, s);
  else
    launch_tn_v<128, 128>(p, va, vb, grid, s);
}

int conv_tn_splitk(int K, int Co, int R, int M) {
  int splitk, mps;
  tn_split(K, Co, R, M, splitk, mps);
  return splitk;
}
