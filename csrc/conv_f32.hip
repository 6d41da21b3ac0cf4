// fp32-accurate client-batched implicit-GEMM convolution / linear for gfx950 (MI355X, CDNA4).
//
// The reference trains in fp32 (conf/global.yaml `use_amp: false`). gfx950 has no xf32/TF32 and
// its f32-input MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate, so these kernels
// compute every product as split bf16 ("bf16x3"):
//
//   a = ah + al, b = bh + bl  (ah = bf16(a), al = bf16(a − ah), RNE)
//   a·b ≈ ah·bh + al·bh + ah·bl      (three v_mfma_f32_32x32x16_bf16, fp32 accumulate)
//
// |a − ah − al| ≤ 2⁻¹⁷|a| and the dropped al·bl ≤ 2⁻¹⁸|a||b|, so each product carries ≤ ~2⁻¹⁶
// relative error (fp32-level results: the GPU tests compare against fp64 at ≤ 1e-5 relative) at
// 3/16 of the f32-MFMA time. Operands are stored fp32 in HBM; the split happens ONCE per element
// per workgroup, when the register-staged tile is written to LDS as two bf16 planes (hi, lo) —
// the fragment reads and MFMA inner loop are the bf16 kernel's, with twice the fragments.
//
//   conv_nt_f32 : Y[m][n] = Σ_r A[m][r] B[n][r]  (forward, dgrad with B read from the forward
//                 weight in place — k-major LDS image + ds_read_b64_tr_b16, as conv_nt.hip)
//   conv_tn_f32 : dW[co][r] = Σ_m dY[m][co] X̃[m][r]  (weight gradient, split-K fp32 atomics)
#include "dls.h"
#include "gemm_common.h"
#include "epilogue_f32.h"

#include <numeric>

namespace {

template <int V>
struct FV {
  float v[V];
};

template <int V>
__device__ __forceinline__ void fzero(FV<V>& f) {
#pragma unroll
  for (int i = 0; i < V; ++i) f.v[i] = 0.f;
}

template <int V>
__device__ __forceinline__ void fload(FV<V>& f, const float* p) {
  load_vec<V>(p, f.v);
}

// V floats → V bf16 hi at `hi`, V bf16 lo at `lo` (one 2/8/16-B LDS store per plane)
template <int V>
__device__ __forceinline__ void st_split(bf16_t* hi, bf16_t* lo, const FV<V>& f) {
  typedef typename VecT<V>::T TV;
  union {
    TV v;
    bf16_t e[V];
    uint32_t p[V / 2 > 0 ? V / 2 : 1];
  } h, l;
  if constexpr (V % 2 == 0) {
#pragma unroll
    for (int i = 0; i < V / 2; ++i) split_pair(f.v[2 * i], f.v[2 * i + 1], h.p[i], l.p[i]);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) split2(f.v[i], h.e[i], l.e[i]);
  }
  *reinterpret_cast<TV*>(hi) = h.v;
  *reinterpret_cast<TV*>(lo) = l.v;
}

// element offset of k-column e inside row r of a BK-wide bf16 row-major image (16-B slot XOR)
template <int BK>
__device__ __forceinline__ int swz(int r, int e) {
  constexpr int S = BK / 8, RPR = 256 / (BK * 2);  // slots per row, rows per 256-B bank row
  static_assert(S >= 2 && RPR >= 1, "swizzle needs 16..128-element rows");
  return (((e >> 3) ^ ((r / RPR) % S)) << 3) | (e & 7);
}

// ------------------------------------------------------------------------- NT (fwd / dgrad)
template <int BM, int BN, int BK, int WM, int WN, int VA, int VB, bool BKM, int NBUF, int MINW = 1, bool BSPL = false>
__global__ void __launch_bounds__(WM* WN * 64, MINW) conv_nt_f32_kernel(ConvNTParams p) {
  // BSPL: B comes pre-split (p.wsplit hi / lo bf16 planes, written by the SGD step): its loads
  // are 16-B bf16 vectors stored to LDS as they are, no split VALU for B in the loop
  static_assert(!BSPL || VB == 8, "pre-split B needs 8-element vectors");
  constexpr int T = WM * WN * 64;
  constexpr int TM = BM / (WM * 32);
  constexpr int TN = BN / (WN * 32);
  // row-major [row][k] images (A, and B when !BKM) are unpadded BK-element rows whose 16-B slots
  // are XOR-swizzled by the row's position in the 256-B bank row: ds_read_b128 fragment reads and
  // the 8-lane ds_write_b128 / 16-lane ds_write_b64 split stores are all conflict-free (a +8 pad
  // made the stores straddle bank rows: 2-way, 20-35 % of LDS cycles in SQ_LDS_BANK_CONFLICT)
  constexpr int LDA = BK;
  constexpr int KCA = BK / VA, RPA = T / KCA, PA = BM / RPA;
  // B row-major [n][k] / k-major [k][n]; a narrow B (BN = 32) has fewer rows than loader threads:
  // one pass, threads past the last row idle (B_PART / K_PART)
  constexpr int KCB = BK / VB, RPB = T / KCB, PB = RPB > BN ? 1 : BN / RPB;
  constexpr int CCB = BN / VB, RPK = T / CCB, PK = RPK > BK ? 1 : BK / RPK;
  constexpr bool B_PART = RPB > BN, K_PART = RPK > BK;
  constexpr int LDBK = BN + 32;                                // row bytes ≡ 64 (mod 256)
  constexpr int NB = BKM ? PK : PB;
  static_assert(PA >= 1 && NB >= 1, "tile too small for thread count");
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  constexpr int B_ROWS = BKM ? BK : BN, B_COLS = BKM ? LDBK : LDA;
  constexpr int A_PLANE = NBUF * BM * LDA, B_PLANE = NBUF * B_ROWS * B_COLS;  // bf16 elements
  constexpr int LOOP_BYTES = 2 * (A_PLANE + B_PLANE) * 2;
  constexpr int SW = TN * 32 + 4;                   // epilogue slab row (fp32), 16-B aligned
  constexpr int EPI_BYTES = WM * WN * 32 * SW * 4;  // one 32-row slab per wave
  constexpr int SMEM = LOOP_BYTES > EPI_BYTES ? LOOP_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  bf16_t* const As = reinterpret_cast<bf16_t*>(smem);  // [plane hi/lo][NBUF][BM][LDA]
  bf16_t* const Bs = As + 2 * A_PLANE;                 // [plane][NBUF][B_ROWS][B_COLS]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tilesM = (p.M + BM - 1) / BM, tilesN = (p.N + BN - 1) / BN;
  const int per_client = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  const int t = bid % per_client;
  const int m0 = (t / tilesN) * BM, n0 = (t % tilesN) * BN;
  const float* __restrict__ x = reinterpret_cast<const float*>(p.x) + (long)client * p.x_cs;
  const float* __restrict__ w = reinterpret_cast<const float*>(p.w) + (long)(client / p.rep) * p.w_cs;

  // --- operand windows as buffer resources: an out-of-range lane offset reads zeros, so image
  // padding, M / N / R tails and idle loader threads cost a select instead of a branch
  const auto xr = make_rsrc(x, (uint32_t)((long)p.B * p.H * p.W * p.ldx * 4));
  const long w_ext = BKM ? (long)p.C * p.wKH * p.wKW * p.N : (long)p.N * p.R;  // elements
  const auto wr = make_rsrc(w, (uint32_t)(w_ext * 4));
  const auto wsr = make_rsrc(BSPL ? (const void*)(p.wsplit + (long)(client / p.rep) * p.ws_cs) : (const void*)w,
                             BSPL ? (uint32_t)((p.ws_plane + w_ext) * 2) : 0u);
  const uint32_t ws_lo = (uint32_t)(p.ws_plane * 2);  // byte distance hi → lo plane

  // --- A loader: PA rows per thread, one fixed K sub-chunk, incremental im2col state. A row's
  // element offset is a_off0[j] (its pixel window origin) + koff, the tap / channel part shared by
  // every row of the thread and advanced with adds only
  const int kca = tid % KCA;
  int a_ih0[PA], a_iw0[PA], a_off0[PA];
  bool a_ok[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int m = m0 + tid / KCA + j * RPA;
    a_ok[j] = m < p.M;
    const uint32_t mm = a_ok[j] ? m : 0;
    const uint32_t b = fdiv(mm, p.fd_ohw);
    const uint32_t rem = mm - b * p.OH * p.OW;
    const uint32_t oh = fdiv(rem, p.fd_ow);
    const uint32_t ow = rem - oh * p.OW;
    a_ih0[j] = (int)oh * p.stride - p.pad;
    a_iw0[j] = (int)ow * p.stride - p.pad_w;
    a_off0[j] = (((int)b * p.H + a_ih0[j]) * p.W + a_iw0[j]) * p.ldx;
  }
  int r_cur = kca * VA;
  int kh, kw, c;
  {
    kh = (int)fdiv(r_cur, p.fd_kwc);
    const int rr = r_cur - kh * p.KW * p.C;
    kw = (int)fdiv(rr, p.fd_c);
    c = rr - kw * p.C;
  }
  int koff = (kh * p.W + kw) * p.ldx + c;
  const int kcb = tid % (BKM ? CCB : KCB);
  const int nk = (p.R + BK - 1) / BK;
  int k_next = 0;
  // B row offsets (row-major B): -1 marks a row past N or an idle thread of a narrow tile
  int b_row[BKM ? 1 : PB];
  // k-major B (dgrad: the forward weight read in place, taps flipped / strided by parity class):
  // each of the thread's PK k-rows keeps its (channel, tap column) position and element offset,
  // advanced by BK per step with adds only
  int bk_co[BKM ? PK : 1], bk_kw[BKM ? PK : 1], bk_off[BKM ? PK : 1];
  const int nb0 = n0 + kcb * VB;
  const bool b_live = BKM ? (!(K_PART && tid / CCB >= BK) && nb0 < p.N) : true;
  if constexpr (!BKM) {
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int n = n0 + tid / KCB + j * RPB;
      b_row[j] = (n < p.N && !(B_PART && tid / KCB >= BN)) ? n * p.R : -1;
    }
  } else {
#pragma unroll
    for (int j = 0; j < PK; ++j) {
      const int k = tid / CCB + j * RPK;
      const int kh2 = (int)fdiv(k, p.fd_kwc);
      const int rr = k - kh2 * p.KW * p.C;
      const int kw2 = (int)fdiv(rr, p.fd_c);
      const int co = rr - kw2 * p.C;
      const int khh = p.kh_off - p.kh_step * kh2, kww = p.kw_off - p.kw_step * kw2;
      bk_co[j] = co;
      bk_kw[j] = kw2;
      bk_off[j] = ((co * p.wKH + khh) * p.wKW + kww) * p.N + nb0;
    }
  }
  const int w_co_step = p.wKH * p.wKW * p.N;  // element offset of one input channel

  FV<VA> ra[PA];
  FV<BSPL ? 1 : VB> rb[NB];
  u32x4_t rbh[BSPL ? NB : 1], rbl[BSPL ? NB : 1];
  auto load_b = [&](int j, uint32_t e_off, bool ok) {  // B element offset e_off (w's layout)
    if constexpr (BSPL) {
      rbh[j] = __builtin_amdgcn_raw_buffer_load_b128(wsr, ok ? e_off * 2u : OOB_OFF, 0, 0);
      rbl[j] = __builtin_amdgcn_raw_buffer_load_b128(wsr, ok ? e_off * 2u + ws_lo : OOB_OFF, 0, 0);
    } else {
      buf_load<VB>(rb[j].v, wr, ok ? e_off * 4u : OOB_OFF);
    }
  };

  auto load = [&]() {
    const int k0 = k_next;
    k_next += BK;
    const bool rok = r_cur < p.R;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int qh = a_ih0[j] + kh, qw = a_iw0[j] + kw;
      const bool ok = rok && a_ok[j] && (unsigned)qh < (unsigned)p.H && (unsigned)qw < (unsigned)p.W;
      buf_load<VA>(ra[j].v, xr, ok ? (uint32_t)(a_off0[j] + koff) * 4u : OOB_OFF);
    }
    if constexpr (!BKM) {
      const int rB = k0 + kcb * VB;
#pragma unroll
      for (int j = 0; j < PB; ++j) load_b(j, (uint32_t)(b_row[j] + rB), b_row[j] >= 0 && rB < p.R);
    } else {
#pragma unroll
      for (int j = 0; j < PK; ++j) {
        const int k = k0 + tid / CCB + j * RPK;
        load_b(j, (uint32_t)bk_off[j], b_live && k < p.R);
        // advance this k-row by BK: channel, then tap column (kw_step apart in the weight), then
        // tap row (kh_step apart)
        bk_co[j] += BK;
        bk_off[j] += BK * w_co_step;
        while (bk_co[j] >= p.C) {
          bk_co[j] -= p.C;
          bk_off[j] -= p.C * w_co_step + p.kw_step * p.N;
          if (++bk_kw[j] == p.KW) {
            bk_kw[j] = 0;
            bk_off[j] += (p.KW * p.kw_step - p.kh_step * p.wKW) * p.N;
          }
        }
      }
    }
    r_cur += BK;
    c += BK;
    koff += BK;
    while (c >= p.C) {
      c -= p.C;
      koff += p.ldx - p.C;
      if (++kw == p.KW) {
        kw = 0;
        ++kh;
        koff += (p.W - p.KW) * p.ldx;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int r = tid / KCA + j * RPA;
      const int off = (buf * BM + r) * LDA + swz<BK>(r, kca * VA);
      st_split(As + off, As + A_PLANE + off, ra[j]);
    }
    if constexpr (!BKM) {
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int r = tid / KCB + j * RPB;
        if (B_PART && r >= BN) continue;
        const int off = (buf * B_ROWS + r) * B_COLS + swz<BK>(r, kcb * VB);
        if constexpr (BSPL) {
          *reinterpret_cast<u32x4_t*>(Bs + off) = rbh[j];
          *reinterpret_cast<u32x4_t*>(Bs + B_PLANE + off) = rbl[j];
        } else {
          st_split(Bs + off, Bs + B_PLANE + off, rb[j]);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < PK; ++j) {
        if (K_PART && tid / CCB >= BK) continue;
        const int off = (buf * B_ROWS + tid / CCB + j * RPK) * B_COLS + kcb * VB;
        if constexpr (BSPL) {
          *reinterpret_cast<u32x4_t*>(Bs + off) = rbh[j];
          *reinterpret_cast<u32x4_t*>(Bs + B_PLANE + off) = rbl[j];
        } else {
          st_split(Bs + off, Bs + B_PLANE + off, rb[j]);
        }
      }
    }
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
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm0 + i * 32 + (lane & 31);
        const int off = (buf * BM + r) * LDA + swz<BK>(r, ks * 16 + 8 * h);
        ah[i] = *reinterpret_cast<const bf16x8*>(As + off);
        al[i] = *reinterpret_cast<const bf16x8*>(As + A_PLANE + off);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (!BKM) {
          const int r = wn0 + j * 32 + (lane & 31);
          const int off = (buf * B_ROWS + r) * B_COLS + swz<BK>(r, ks * 16 + 8 * h);
          bh[j] = *reinterpret_cast<const bf16x8*>(Bs + off);
          bl[j] = *reinterpret_cast<const bf16x8*>(Bs + B_PLANE + off);
        } else {
          const int col = wn0 + j * 32 + 16 * (g & 1) + 4 * pp;
          const int o0 = (buf * B_ROWS + ks * 16 + 8 * h + q) * B_COLS + col;
          const int o1 = o0 + 4 * B_COLS;
          bh[j] = tr_frag(Bs + o0, Bs + o1);
          bl[j] = tr_frag(Bs + B_PLANE + o0, Bs + B_PLANE + o1);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  };

  if constexpr (NBUF == 1) {
    load();
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load();
      compute(0);
      if (kt + 1 < nk) {
        __syncthreads();
        store(0);
        __syncthreads();
      }
    }
  } else {
    load();
    store(0);
    __syncthreads();
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load();
      compute(buf);
      if (kt + 1 < nk) store(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  nt_f32_epilogue<TM, TN, WM * WN, -1, false>(p, acc, smem, client, m0, n0, wm0, wn0, wid, lane);
}

// VSET 0: the 32-B (8, 8) gathers of wide layers; 1: + 16-B (4, ·) widths (d_model = 100,
// DenseNet's 12-channel growth); 2: every combination incl. scalar (stems, LeNet, tiny linears)
template <int BM, int BN, int BK, int WM, int WN, int NBUF, int VSET, int MINW = 1>
bool launch_nt_f32_cfg(const ConvNTParams& p, int K, int va, int vb, bool bkm, hipStream_t s) {
  const int grid = K * cdiv(p.M, BM) * cdiv(p.N, BN);
  if (p.wsplit && va == 8 && vb == 8) {  // pre-split weight planes (8-wide vectors only)
    if (bkm)
      hipLaunchKernelGGL((conv_nt_f32_kernel<BM, BN, BK, WM, WN, 8, 8, true, NBUF, MINW, true>), dim3(grid),
                         dim3(WM * WN * 64), 0, s, p);
    else
      hipLaunchKernelGGL((conv_nt_f32_kernel<BM, BN, BK, WM, WN, 8, 8, false, NBUF, MINW, true>), dim3(grid),
                         dim3(WM * WN * 64), 0, s, p);
    return true;
  }
#define NTF_CASE(A, B)                                                                                       \
  if (va == A && vb == B) {                                                                                  \
    if (bkm)                                                                                                 \
      hipLaunchKernelGGL((conv_nt_f32_kernel<BM, BN, BK, WM, WN, A, B, true, NBUF, MINW>), dim3(grid),             \
                         dim3(WM * WN * 64), 0, s, p);                                                       \
    else                                                                                                     \
      hipLaunchKernelGGL((conv_nt_f32_kernel<BM, BN, BK, WM, WN, A, B, false, NBUF, MINW>), dim3(grid),            \
                         dim3(WM * WN * 64), 0, s, p);                                                       \
    return true;                                                                                             \
  }
  NTF_CASE(8, 8)
  if constexpr (VSET >= 1) { NTF_CASE(4, 4) NTF_CASE(8, 4) NTF_CASE(4, 8) }
  if constexpr (VSET >= 2) { NTF_CASE(8, 1) NTF_CASE(4, 1) NTF_CASE(1, 8) NTF_CASE(1, 4) NTF_CASE(1, 1) }
#undef NTF_CASE
  return false;
}

// variant ids are stable (bench/kernel_bench.py --f32 sweeps them)
bool launch_nt_f32_variant(int v, const ConvNTParams& p, int K, int va, int vb, bool bkm, hipStream_t s) {
  switch (v) {
    case 0: return launch_nt_f32_cfg<128, 128, 32, 2, 2, 2, 1>(p, K, va, vb, bkm, s);  // 80 KB: 2 blocks/CU
    case 1: return launch_nt_f32_cfg<128, 128, 32, 2, 2, 1, 0>(p, K, va, vb, bkm, s);  // 40 KB
    case 2: return launch_nt_f32_cfg<256, 128, 32, 4, 2, 1, 0>(p, K, va, vb, bkm, s);  // 60 KB
    case 3: return launch_nt_f32_cfg<64, 64, 32, 2, 2, 2, 2>(p, K, va, vb, bkm, s);    // 40 KB, any width
    case 4: return launch_nt_f32_cfg<128, 64, 32, 4, 1, 2, 1>(p, K, va, vb, bkm, s);   // 60 KB, N <= 64
    case 5: return launch_nt_f32_cfg<128, 128, 64, 2, 2, 1, 0>(p, K, va, vb, bkm, s);  // 72 KB
    case 6: return launch_nt_f32_cfg<256, 64, 32, 4, 1, 1, 0>(p, K, va, vb, bkm, s);   // 50 KB, N <= 64
    case 7: return launch_nt_f32_cfg<64, 64, 32, 2, 2, 1, 1>(p, K, va, vb, bkm, s);    // 20 KB
    // variants 1 / 6 compiled for 3 waves per SIMD (<= 168 registers) instead of 2
    case 8: return launch_nt_f32_cfg<128, 128, 32, 2, 2, 1, 0, 3>(p, K, va, vb, bkm, s);
    case 9: return launch_nt_f32_cfg<256, 64, 32, 4, 1, 1, 0, 3>(p, K, va, vb, bkm, s);
    // N <= 32 (DenseNet's 12-channel growth convs): a 32-wide B tile wastes 62 % of each MFMA
    // instead of 81 % in the 64-wide ones, 36 KB
    case 10: return launch_nt_f32_cfg<256, 32, 32, 4, 1, 1, 1>(p, K, va, vb, bkm, s);
    default: return false;
  }
}

int vw(int c) { return (c % 8 == 0) ? 8 : (c % 4 == 0) ? 4 : 1; }

// (small-cohort 64x64 tile rules for the NT and wgrad kernels won in isolation — kernel_bench at
// K = 4 — but lost inside a round, where the other sub-cohort stream fills the GPU and per-CU
// efficiency matters more than grid fill: rank 0's share of an 8-rank round, 2 streams, 743 ms
// without, 757 / 765 ms with the NT / wgrad rule — removed)

// --------------------------------------------------------------------------- TN (wgrad)
template <int BMc, int BNr, int BKT, int WM, int WN, int VA, int VB, int NBUF>
__global__ void __launch_bounds__(WM* WN * 64) conv_tn_f32_kernel(ConvTNParams p) {
  constexpr int T = WM * WN * 64;
  constexpr int TM = BMc / (WM * 32), TN = BNr / (WN * 32);
  constexpr int LDA = BMc + 32;
  constexpr int LDB = BNr + 32;
  // a 32-row dY tile (BMc = 32: DenseNet's 12-channel growth convs) with 8-wide vectors has more
  // loader threads than k-rows: one pass, the extra threads idle (A_PART)
  constexpr int CCA = BMc / VA, RPA = T / CCA, PA = RPA > BKT ? 1 : BKT / RPA;
  constexpr bool A_PART = RPA > BKT;
  constexpr int CCB = BNr / VB, RPB = T / CCB, PB = BKT / RPB;
  static_assert(PA >= 1 && PB >= 1, "tile too small");
  constexpr int A_PLANE = NBUF * BKT * LDA, B_PLANE = NBUF * BKT * LDB;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (A_PLANE + B_PLANE)];
  bf16_t* const As = smem;               // [plane][NBUF][BKT][LDA]
  bf16_t* const Bs = smem + 2 * A_PLANE;  // [plane][NBUF][BKT][LDB]

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

  const float* __restrict__ dy = reinterpret_cast<const float*>(p.dy) + (long)client * p.dy_cs;
  const float* __restrict__ x = reinterpret_cast<const float*>(p.x) + (long)client * p.x_cs;

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

  FV<VA> ra[PA];
  FV<VB> rb[PB];
  // operand windows as buffer resources (out-of-range offset ⇒ zeros: no branches / zero fills)
  const auto dyr = make_rsrc(dy, (uint32_t)((long)p.M * p.ldy * 4));
  const auto xr = make_rsrc(x, (uint32_t)((long)p.B * p.H * p.W * p.ldx * 4));
  const bool a_live = cok && !(A_PART && tid / CCA >= BKT);
  int k_next = mbeg;
  // im2col rows of X̃ without divisions in the loop: each of the thread's PB GEMM rows m keeps
  // its input coordinates (ih, iw) and element offset, advanced by BKT rows per step through the
  // fixed decomposition BKT = q_b·OH·OW + q_oh·OW + r_ow (one carry per level: no muls)
  const int q_b = BKT / (p.OH * p.OW), rem_b = BKT - q_b * p.OH * p.OW;
  const int q_oh = rem_b / p.OW, r_ow = rem_b - q_oh * p.OW;
  const int s_ldx = p.stride * p.ldx, s_row = p.stride * p.W * p.ldx, img = p.H * p.W * p.ldx;
  const int d_iw = r_ow * p.stride, d_off = r_ow * s_ldx + q_oh * s_row + q_b * img;
  const int w_wrap = p.OW * p.stride, off_c1 = s_row - p.OW * s_ldx;    // ow wraps: next output row
  const int d_ih0 = q_oh * p.stride, d_ih1 = (q_oh + 1) * p.stride;
  const int h_wrap = p.OH * p.stride, off_c2 = img - p.OH * s_row;       // oh wraps: next image
  int bx_ow[PB], bx_oh[PB], bx_ih[PB], bx_iw[PB], bx_off[PB];
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const uint32_t m = mbeg + tid / CCB + j * RPB;
    const uint32_t b = fdiv(m, p.fd_ohw);
    const uint32_t rem = m - b * p.OH * p.OW;
    const uint32_t oh = fdiv(rem, p.fd_ow);
    const uint32_t ow = rem - oh * p.OW;
    bx_ow[j] = ow;
    bx_oh[j] = oh;
    bx_ih[j] = (int)oh * p.stride - p.pad + kh;
    bx_iw[j] = (int)ow * p.stride - p.pad + kw;
    bx_off[j] = (((int)b * p.H + bx_ih[j]) * p.W + bx_iw[j]) * p.ldx + c;
  }
  int a_off = (mbeg + tid / CCA) * p.ldy + cocol;  // + j·RPA·ldy for row j
  const int a_jstep = RPA * p.ldy, a_kstep = BKT * p.ldy;
  auto load = [&]() {
    const int k0 = k_next;
    k_next += BKT;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int m = k0 + tid / CCA + j * RPA;
      buf_load<VA>(ra[j].v, dyr, (a_live && m < mend) ? (uint32_t)(a_off + j * a_jstep) * 4u : OOB_OFF);
    }
    a_off += a_kstep;
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int m = k0 + tid / CCB + j * RPB;
      const bool ok = rok && m < mend && (unsigned)bx_ih[j] < (unsigned)p.H && (unsigned)bx_iw[j] < (unsigned)p.W;
      buf_load<VB>(rb[j].v, xr, ok ? (uint32_t)bx_off[j] * 4u : OOB_OFF);
      // advance row m by BKT (wave-uniform step constants; the carries are selects)
      bx_ow[j] += r_ow;
      bx_iw[j] += d_iw;
      bx_off[j] += d_off;
      const bool c1 = bx_ow[j] >= p.OW;
      bx_ow[j] -= c1 ? p.OW : 0;
      bx_oh[j] += c1 ? q_oh + 1 : q_oh;
      bx_iw[j] -= c1 ? w_wrap : 0;
      bx_ih[j] += c1 ? d_ih1 : d_ih0;
      bx_off[j] += c1 ? off_c1 : 0;
      const bool c2 = bx_oh[j] >= p.OH;
      bx_oh[j] -= c2 ? p.OH : 0;
      bx_ih[j] -= c2 ? h_wrap : 0;
      bx_off[j] += c2 ? off_c2 : 0;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      if (A_PART && tid / CCA >= BKT) continue;
      const int off = (buf * BKT + tid / CCA + j * RPA) * LDA + ca * VA;
      st_split(As + off, As + A_PLANE + off, ra[j]);
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int off = (buf * BKT + tid / CCB + j * RPB) * LDB + cb * VB;
      st_split(Bs + off, Bs + B_PLANE + off, rb[j]);
    }
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
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
      const int krow = buf * BKT + ks * 16 + 8 * h + q;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int o0 = krow * LDA + wm0 + i * 32 + 16 * (g & 1) + 4 * pp, o1 = o0 + 4 * LDA;
        ah[i] = tr_frag(As + o0, As + o1);
        al[i] = tr_frag(As + A_PLANE + o0, As + A_PLANE + o1);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int o0 = krow * LDB + wn0 + j * 32 + 16 * (g & 1) + 4 * pp, o1 = o0 + 4 * LDB;
        bh[j] = tr_frag(Bs + o0, Bs + o1);
        bl[j] = tr_frag(Bs + B_PLANE + o0, Bs + B_PLANE + o1);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  };

  const int nk = (mend - mbeg + BKT - 1) / BKT;
  if (nk <= 0) return;
  if constexpr (NBUF == 1) {
    load();
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load();
      compute(0);
      if (kt + 1 < nk) {
        __syncthreads();
        store(0);
        __syncthreads();
      }
    }
  } else {
    load();
    store(0);
    __syncthreads();
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load();
      compute(buf);
      if (kt + 1 < nk) store(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // split-K: this split's slab of the deterministic fold (ConvTNParams::part), or fp32 atomics
  // into the pre-zeroed rows when no slab buffer was given
  const bool slab = p.splitk > 1 && p.part != nullptr;
  const bool atom = p.splitk > 1 && !slab;
  float* __restrict__ dw = slab ? p.part + ((long)split * (gridDim.x / per_client) + client) * p.Co * p.R
                                : p.dw + (long)client * p.dw_cs;
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
          if (atom)
            atomicAdd(dst, acc[i][j][e]);
          else
            *dst = acc[i][j][e];
        }
      }
    }
  }
}

template <int BMc, int BNr, int BKT, int WM, int WN, int NBUF, bool ALLV>
bool launch_tn_f32_cfg(const ConvTNParams& p, int va, int vb, int grid, hipStream_t s) {
#define TNF_CASE(A, B)                                                                                          \
  if (va == A && vb == B) {                                                                                     \
    hipLaunchKernelGGL((conv_tn_f32_kernel<BMc, BNr, BKT, WM, WN, A, B, NBUF>), dim3(grid), dim3(WM * WN * 64), \
                       0, s, p);                                                                                \
    return true;                                                                                                \
  }
  TNF_CASE(8, 8)
  if constexpr (ALLV) {
    TNF_CASE(4, 4) TNF_CASE(8, 4) TNF_CASE(4, 8) TNF_CASE(1, 1) TNF_CASE(8, 1) TNF_CASE(1, 8) TNF_CASE(4, 1)
    TNF_CASE(1, 4)
  }
#undef TNF_CASE
  return false;
}

struct TnTile {
  int bm, bn;
};
constexpr TnTile kTnF32Tiles[] = {{128, 128}, {64, 128}, {128, 128}, {256, 128}, {128, 256}, {64, 64}, {32, 128},
                                   {64, 256}};
constexpr int kTnF32Variants = sizeof(kTnF32Tiles) / sizeof(kTnF32Tiles[0]);
constexpr int TN_BKT_MAX = 32;

bool launch_tn_f32_variant(int v, const ConvTNParams& p, int va, int vb, int grid, hipStream_t s) {
  switch (v) {
    case 0: return launch_tn_f32_cfg<128, 128, 32, 2, 2, 2, true>(p, va, vb, grid, s);  // 80 KB
    case 1: return launch_tn_f32_cfg<64, 128, 32, 2, 2, 2, true>(p, va, vb, grid, s);   // 60 KB
    case 2: return launch_tn_f32_cfg<128, 128, 32, 2, 2, 1, false>(p, va, vb, grid, s);  // 40 KB
    case 3: return launch_tn_f32_cfg<256, 128, 32, 4, 2, 1, false>(p, va, vb, grid, s);  // 60 KB
    case 4: return launch_tn_f32_cfg<128, 256, 32, 2, 4, 1, false>(p, va, vb, grid, s);  // 60 KB
    case 5: return launch_tn_f32_cfg<64, 64, 32, 2, 2, 2, true>(p, va, vb, grid, s);    // 40 KB
    case 6: return launch_tn_f32_cfg<32, 128, 32, 1, 4, 2, true>(p, va, vb, grid, s);   // 56 KB, Co <= 32
    // 64x256, 49 KB single-buffered: 4 column fragments per wave, twice the MFMAs per k-step of
    // the 64x128 tile. Measured slower on Co = 64 (l1 wgrad 172 vs 197 TFLOP/s at K = 100,
    // profiles/r2_kernel_bench_f32_tn64x256_sweep.jsonl): sweep-only
    case 7: return launch_tn_f32_cfg<64, 256, 32, 2, 2, 1, false>(p, va, vb, grid, s);
    default: return false;
  }
}

// measured (kernel_bench --f32 --sweep, K = 100): Co = 64 layers want the 64x128 double-buffered
// tile (l1 165 TFLOP/s), the rest the single-buffer 128x128 (l2 248, l3 277, l4a 260), the
// 256x128 tile only at Co >= 512 with enough tiles (l4 286 vs 273)
int tn_f32_default_variant(int K, int Co, int R) {
  auto tiles = [&](int bm, int bn) { return (long)K * cdiv(Co, bm) * cdiv(R, bn); };
  if (Co <= 32 && R > 64) return 6;
  if (Co <= 32 || R <= 64) return 5;
  // re-measured after the buffer-load loaders (kernel_bench --f32 --sweep, K = 33 / 100):
  // 1x1 shortcut convs (R <= 256) the 64x64 tile (l4sc 165 vs 97 TFLOP/s at K = 33); Co <= 64 the
  // 64x128 double-buffered tile; 3x3 layers with Co >= 256 and R >= 2048 the 256x128 tile (l3 / l4
  // 277-304 vs 256-291); the rest the double-buffered 128x128 (l2 / l3a 258-270 vs 238-268)
  (void)tiles;
  if (R <= 256 && Co > 64) return 5;
  if (Co <= 64) return 1;
  if (Co >= 256 && R >= 2048) return 3;
  // (the Transformer in_proj weight gradient, Co 1536 x R 512: 1.16 vs 1.24 ms for 128x128,
  // profiles/r6_c14_linear_f32_variants.log)
  if (Co >= 1024 && R >= 512) return 3;
  return 0;
}

int resolve_tn_f32_variant(int variant, int K, int Co, int R, int va, int vb) {
  if (variant < 0 || variant >= kTnF32Variants) variant = tn_f32_default_variant(K, Co, R);
  if ((va != 8 || vb != 8) && !(variant == 0 || variant == 1 || variant == 5 || variant == 6))
    variant = Co <= 64 ? 1 : 0;
  // (the all-widths tiles are the double-buffered 0 / 1 / 5 / 6)
  return variant;
}

void tn_f32_split(int K, int Co, int R, int M, int variant, int& splitk, int& mps) {
  // per-client decision (a reference cohort of 32): the deterministic fold's order must not
  // depend on how many clients share the launch (see conv_pl.hip tn_pl_split)
  (void)K;
  const TnTile t = kTnF32Tiles[variant];
  const long tiles = (long)32 * cdiv(Co, t.bm) * cdiv(R, t.bn);
  splitk = 1;
  const int target = 1024;  // >= 4 blocks per CU
  if (tiles < target) {
    splitk = (int)((target + tiles - 1) / tiles);
    splitk = min(splitk, max(1, M / (4 * TN_BKT_MAX)));
  }
  mps = cdiv(M, splitk);
  mps = ((mps + TN_BKT_MAX - 1) / TN_BKT_MAX) * TN_BKT_MAX;
  splitk = cdiv(M, mps);
}

}  // namespace

int conv_nt_f32_num_variants() { return 11; }

void conv_nt_f32(const ConvNTParams& p, int K, int variant, hipStream_t s) {
  if (p.x_lo != 0) {  // pre-split A (and B) planes: the LDS-DMA kernels of conv_halo / conv_pl.hip
    if (conv_nt_pl_variant() < 0 && conv_halo(p, K, s)) return;
    if (!conv_nt_pl(p, K, conv_nt_pl_variant(), s)) {
      fprintf(stderr, "conv_nt_f32: pre-split operands in an unsupported shape (C %d, ldx %d, N %d, R %d)\n", p.C,
              p.ldx, p.N, p.R);
      abort();
    }
    return;
  }
  const bool bkm = p.b_kmajor != 0;
  // the loaders address each client's operand window with 32-bit buffer offsets
  const long xb = (long)p.B * p.H * p.W * p.ldx * 4;
  const long wb = (bkm ? (long)p.C * p.wKH * p.wKW * p.N : (long)p.N * p.R) * 4;
  if (p.dil != 1) {  // (the dgrad launches use stride-1 parity classes, never input dilation)
    fprintf(stderr, "conv_nt_f32: input dilation is not supported\n");
    abort();
  }
  if (xb >= (long)OOB_OFF || wb >= (long)OOB_OFF || (p.wsplit && (p.ws_plane + wb / 4) * 2 >= (long)OOB_OFF)) {
    fprintf(stderr, "conv_nt_f32: per-client operand window over 2 GiB (x %ld B, w %ld B)\n", xb, wb);
    abort();
  }
  const int va = vw(std::gcd(p.C, p.ldx));
  int vb = bkm ? vw(p.N) : vw(p.R);
  if (variant < 0) {
    // measured (bench/kernel_bench.py --f32 --sweep, ResNet-18 layers, K = 100): the single-buffer
    // tiles win everywhere — 40-60 KB of LDS keeps 3 workgroups per CU, whose waves hide each
    // other's split (VALU) and global-load phases: 128x128 fwd/dgrad 275-299 TFLOP/s on l2-l4
    // (80 KB double-buffered v0: 262-276), 256x64 for N <= 64 (l1 fwd 211 vs 184, dgrad 209 vs 181)
    // (re-measured after the buffer-load loaders: for N <= 64 the 256x64 tile compiled for 3
    // waves per SIMD, v9: l1 dgrad 233-236 vs 205-222, strided-dgrad classes onto 64 channels
    // 157-179 vs 132-151, the 8-channel stem 118 vs 98-108; fwd equal)
    variant = p.N <= 64 ? 9 : 1;
    if (p.N <= 32) variant = 10;
    // linear-shaped GEMMs (1x1, no im2col: the Transformer's fp32-operand out_proj forward and
    // in_proj dgrad) on the 128x128 tile at 3 waves per SIMD as well: out_proj fwd 0.44 → 0.38 ms,
    // in_proj fwd / dgrad 1.25 / 1.10 → 1.09 / 1.02 (bench/linear_bench.py --f32-variants,
    // profiles/r6_c14_linear_f32_variants.log)
    if (p.N > 64 && p.KH * p.KW == 1) variant = 8;
  }
  // variants without the requested vector widths fall back to the all-widths 64x64 tile
  const bool v88 = va == 8 && vb == 8;
  const bool v84 = (va == 8 || va == 4) && (vb == 8 || vb == 4);
  if (!v88) {
    if (!v84 && variant != 3) variant = 3;
    if (v84 && !(variant == 0 || variant == 3 || variant == 4 || variant == 7 || variant == 10))
      variant = p.N <= 64 ? 4 : 0;
  }
  if (!launch_nt_f32_variant(variant, p, K, va, vb, bkm, s)) fprintf(stderr, "conv_nt_f32: bad variant %d\n", variant);
  if (p.yp) {
    // output planes: these kernels' epilogue has no plane stores (nt_f32_epilogue YP = false: the two
    // registers cost occupancy, 5 → 4 waves/SIMD on the 64x64 tiles), so split y afterwards
    if (p.yp_cs != 2 * p.y_cs || p.yp_lo != p.y_cs || p.ldy != p.N || p.out_s != 1) {
      fprintf(stderr, "conv_nt_f32: output planes need contiguous per-client rows\n");
      abort();
    }
    split_rows(reinterpret_cast<const float*>(p.y), p.yp, K, (long)p.M * p.N, p.y_cs, s);
  }
}

int conv_tn_f32_num_variants() { return kTnF32Variants; }

void conv_tn_f32(ConvTNParams p, int K, int variant, hipStream_t s) {
  if (p.sgd.theta && p.dy_lo == 0) {  // (the SGD epilogue exists in the plane kernels only)
    fprintf(stderr, "conv_tn_f32: the SGD epilogue needs pre-split operands\n");
    abort();
  }
  if (p.dy_lo != 0) {  // pre-split dY / X planes: the LDS-DMA kernels of conv_pl.hip
    if (!conv_tn_pl(p, K, variant, s)) {
      fprintf(stderr, "conv_tn_f32: pre-split operands in an unsupported shape (C %d, Co %d)\n", p.C, p.Co);
      abort();
    }
    return;
  }
  // the loaders address each client's operand window with 32-bit buffer offsets
  const long dyb = (long)p.M * (p.ldy ? p.ldy : p.Co) * 4, xb = (long)p.B * p.H * p.W * (p.ldx ? p.ldx : p.C) * 4;
  if (dyb >= (long)OOB_OFF || xb >= (long)OOB_OFF) {
    fprintf(stderr, "conv_tn_f32: per-client operand window over 2 GiB (dy %ld B, x %ld B)\n", dyb, xb);
    abort();
  }
  const int va = vw(std::gcd(p.Co, p.ldy));
  const int vb = vw(std::gcd(p.C, p.ldx));
  variant = resolve_tn_f32_variant(variant, K, p.Co, p.R, va, vb);
  tn_f32_split(K, p.Co, p.R, p.M, variant, p.splitk, p.m_per_split);
  const TnTile t = kTnF32Tiles[variant];
  const long tiles = (long)K * cdiv(p.Co, t.bm) * cdiv(p.R, t.bn);
  const int grid = (int)(tiles * p.splitk);
  if (!launch_tn_f32_variant(variant, p, va, vb, grid, s)) fprintf(stderr, "conv_tn_f32: bad variant %d\n", variant);
  if (p.splitk > 1 && p.part != nullptr) tn_fold(p.part, p.dw, p.dw_cs, K, p.splitk, (long)p.Co * p.R, s);
}

// gco / gc: the channel counts' gcd with their row strides (they set the vector widths)
int conv_tn_f32_splitk(int K, int Co, int R, int M, int gco, int gc, int variant) {
  int splitk, mps;
  variant = resolve_tn_f32_variant(variant, K, Co, R, vw(gco), vw(gc));
  tn_f32_split(K, Co, R, M, variant, splitk, mps);
  return splitk;
}
