// Client-batched implicit-GEMM convolution / linear, "NT" form, for gfx950 (MI355X, CDNA4).
//
//   Y[m][n] = Σ_r A[m][r] B[n][r]     A = im2col(X) gathered on the fly (NHWC per client)
//   forward : B = W [Co][KH][KW][Ci] (row-major, K contiguous)
//   dgrad   : conv of dY with input dilation = stride; B read STRAIGHT from the forward W:
//             the flip and the Co<->Ci transpose are folded into the loader (k-major LDS image,
//             fragments via ds_read_b64_tr_b16) so no transposed copy is materialised.
//
// Every launch covers ALL K clients of the rank (client = grid coordinate; weights selected
// per client via w_cs; `rep` virtual clients share one weight row for batched evaluation).
// MFMA v_mfma_f32_32x32x16_bf16; each wave owns a (TM·32)x(TN·32) output tile; LDS rows
// padded to (BK+8) bf16 ⇒ conflict-free ds_read_b128 fragment reads; incremental im2col
// state (no integer division in the K loop); XCD-aware tile order.
// DEPTH = 2 keeps two K tiles in flight in registers (loads for tile k+2 are issued before
// computing tile k and written to LDS after computing tile k+1); measured slower than
// DEPTH = 1 on every ResNet shape (≈190 VGPRs ⇒ 1 wave/SIMD), kept for the sweep only.
#include "dls.h"
#include "gemm_common.h"

#include <numeric>

namespace {

template <int BM, int BN, int BK, int WM, int WN, int VA, int VB, bool BKM, int DEPTH>
__global__ void __launch_bounds__(WM* WN * 64) conv_nt_kernel(ConvNTParams p) {
  constexpr int T = WM * WN * 64;
  constexpr int TM = BM / (WM * 32);
  constexpr int TN = BN / (WN * 32);
  constexpr int LDA = BK + 8;
  constexpr int KCA = BK / VA, RPA = T / KCA, PA = BM / RPA;
  constexpr int KCB = BK / VB, RPB = T / KCB, PB = BN / RPB;     // B row-major [n][k]
  constexpr int CCB = BN / VB, RPK = T / CCB, PK = BK / RPK;     // B k-major [k][n]
  constexpr int LDBK = BN + 32;                                 // row bytes ≡ 64 (mod 256)
  constexpr int NB = BKM ? PK : PB;
  static_assert(PA >= 1 && NB >= 1, "tile too small for thread count");
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  constexpr int NBUF = DEPTH == 0 ? 1 : 2;  // DEPTH 0: one LDS buffer, two barriers per K tile
  constexpr int B_ROWS = BKM ? BK : BN, B_COLS = BKM ? LDBK : LDA;
  constexpr int A_BYTES = NBUF * BM * LDA * 2, B_BYTES = NBUF * B_ROWS * B_COLS * 2;
  constexpr int SW = TN * 32 + 8;                   // epilogue slab row (bf16), 16-B padded
  constexpr int EPI_BYTES = WM * WN * 32 * SW * 2;  // one 32-row slab per wave
  constexpr int SMEM = (A_BYTES + B_BYTES) > EPI_BYTES ? (A_BYTES + B_BYTES) : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  auto& As = *reinterpret_cast<bf16_t(*)[NBUF][BM][LDA]>(smem);
  auto& Bs = *reinterpret_cast<bf16_t(*)[NBUF][B_ROWS][B_COLS]>(smem + A_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tilesM = (p.M + BM - 1) / BM, tilesN = (p.N + BN - 1) / BN;
  const int per_client = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  const int t = bid % per_client;
  const int m0 = (t / tilesN) * BM, n0 = (t % tilesN) * BN;
  const bf16_t* __restrict__ x = p.x + (long)client * p.x_cs;
  const bf16_t* __restrict__ w = p.w + (long)(client / p.rep) * p.w_cs;

  // --- A loader: PA rows per thread, one fixed K sub-chunk, incremental im2col state
  const int kca = tid % KCA;
  int a_ih0[PA], a_iw0[PA];
  const bf16_t* a_ptr[PA];
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
    a_ptr[j] = x + (long)b * p.H * p.W * p.ldx;
  }
  int r_cur = kca * VA;
  int kh, kw, c;
  {
    kh = (int)fdiv(r_cur, p.fd_kwc);
    const int rr = r_cur - kh * p.KW * p.C;
    kw = (int)fdiv(rr, p.fd_c);
    c = rr - kw * p.C;
  }
  const int kcb = tid % (BKM ? CCB : KCB);
  const int nk = (p.R + BK - 1) / BK;
  int k_next = 0;  // K offset of the next tile to load

  typedef typename VecT<VA>::T TA;
  typedef typename VecT<VB>::T TB;
  TA ra0[PA], ra1[PA];
  TB rb0[NB], rb1[NB];

  auto load_into = [&](TA* ra, TB* rb) {
    const int k0 = k_next;
    k_next += BK;
    const bool rok = r_cur < p.R;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      ra[j] = vzero<VA>();
      if (!(rok && a_ok[j])) continue;
      int qh = a_ih0[j] + kh, qw = a_iw0[j] + kw;
      if (p.dil > 1) {
        if ((qh % p.dil) != 0 || (qw % p.dil) != 0) continue;
        qh /= p.dil;
        qw /= p.dil;
      }
      if (qh < 0 || qh >= p.H || qw < 0 || qw >= p.W) continue;
      ra[j] = *reinterpret_cast<const TA*>(a_ptr[j] + ((long)qh * p.W + qw) * p.ldx + c);
    }
    if constexpr (!BKM) {
      const int rB = k0 + kcb * VB;
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int n = n0 + tid / KCB + j * RPB;
        rb[j] = vzero<VB>();
        if (n < p.N && rB < p.R) rb[j] = *reinterpret_cast<const TB*>(w + (long)n * p.R + rB);
      }
    } else {
      // k = (kh', kw', co) over the dY channels (p.C = conv Co); n = ci (p.N = conv Ci)
      const int nb = n0 + kcb * VB;
#pragma unroll
      for (int j = 0; j < PK; ++j) {
        const int k = k0 + tid / CCB + j * RPK;
        rb[j] = vzero<VB>();
        if (k >= p.R || nb >= p.N) continue;
        const int kh2 = (int)fdiv(k, p.fd_kwc);
        const int rr = k - kh2 * p.KW * p.C;
        const int kw2 = (int)fdiv(rr, p.fd_c);
        const int co = rr - kw2 * p.C;
        const int kh = p.kh_off - p.kh_step * kh2, kw = p.kw_off - p.kw_step * kw2;
        const long src = (((long)co * p.wKH + kh) * p.wKW + kw) * p.N + nb;
        rb[j] = *reinterpret_cast<const TB*>(w + src);
      }
    }
    r_cur += BK;
    c += BK;
    while (c >= p.C) {
      c -= p.C;
      if (++kw == p.KW) {
        kw = 0;
        ++kh;
      }
    }
  };
  auto store_from = [&](const TA* ra, const TB* rb, int buf) {
#pragma unroll
    for (int j = 0; j < PA; ++j) *reinterpret_cast<TA*>(&As[buf][tid / KCA + j * RPA][kca * VA]) = ra[j];
    if constexpr (!BKM) {
#pragma unroll
      for (int j = 0; j < PB; ++j) *reinterpret_cast<TB*>(&Bs[buf][tid / KCB + j * RPB][kcb * VB]) = rb[j];
    } else {
#pragma unroll
      for (int j = 0; j < PK; ++j) *reinterpret_cast<TB*>(&Bs[buf][tid / CCB + j * RPK][kcb * VB]) = rb[j];
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
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(&As[buf][wm0 + i * 32 + (lane & 31)][ks * 16 + 8 * h]);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (!BKM) {
          bfr[j] = *reinterpret_cast<const bf16x8*>(&Bs[buf][wn0 + j * 32 + (lane & 31)][ks * 16 + 8 * h]);
        } else {
          const int col = wn0 + j * 32 + 16 * (g & 1) + 4 * pp;
          const int krow = ks * 16 + 8 * h + q;
          bfr[j] = tr_frag(&Bs[buf][krow][col], &Bs[buf][krow + 4][col]);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (DEPTH == 0) {
    // half the LDS of the double-buffered loop ⇒ more resident workgroups per CU; the global
    // loads of tile k+1 are still in flight during compute(k)
    load_into(ra0, rb0);
    store_from(ra0, rb0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load_into(ra0, rb0);
      compute(0);
      if (kt + 1 < nk) {
        __syncthreads();
        store_from(ra0, rb0, 0);
        __syncthreads();
      }
    }
  } else if constexpr (DEPTH == 1) {
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
    // two tiles in flight: registers R0/R1 alternate, LDS buffers 0/1 alternate
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

  // --- epilogue: bias (+ReLU) → bf16 → per-wave 32-row LDS slab → 16-B coalesced global
  // stores (one 2-B store per element would make the epilogue store-issue-bound on wide
  // outputs such as the Transformer FFN: 1.9 M rows × 2048)
  bf16_t* __restrict__ y = p.y + (long)client * p.y_cs;
  const bf16_t* accp = p.acc ? p.acc + (long)client * p.y_cs : nullptr;
  const bf16_t* gatep = p.gate ? p.gate + (long)client * p.y_cs : nullptr;
  const bf16_t* bias = p.bias ? p.bias + (long)(client / p.rep) * p.b_cs : nullptr;
  // epilogue scale (dropout's 1/(1-p), or the dgrad gate's) and dropout mask of this client row
  const bool drop = p.drop_p > 0.f && p.drop_seeds != nullptr;
  const uint32_t dseed = drop ? p.drop_seeds[client] : 0u;
  const float oscale = (p.out_scale != 0.f ? p.out_scale : 1.f) * (drop ? 1.f / (1.f - p.drop_p) : 1.f);
  float bvals[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + j * 32 + (lane & 31);
    bvals[j] = (bias && n < p.N) ? bf2f(bias[n]) : 0.f;
  }
  bf16_t* slab = reinterpret_cast<bf16_t*>(smem) + wid * 32 * SW;
  const bool vec_ok = (p.N % 8) == 0 && (p.ldy % 8) == 0 && ((uintptr_t)y & 15) == 0;
  __syncthreads();  // every wave is done reading the K-loop tiles that the slabs overwrite
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float v = acc[i][j][e] + bvals[j];
        if (p.relu) v = fmaxf(v, 0.f);
        v *= oscale;
        if (drop) {
          const int rr = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          if (!drop_keep(dseed, m0 + wm0 + i * 32 + rr, p.N, n0 + wn0 + j * 32 + (lane & 31), p.drop_p)) v = 0.f;
        }
        slab[((e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * SW + j * 32 + (lane & 31)] = f2bf(v);
      }
    }
    __syncthreads();
    for (int qd = lane; qd < 32 * TN * 4; qd += 64) {
      const int r = qd / (TN * 4), cc = (qd % (TN * 4)) * 8;
      const int m = m0 + wm0 + i * 32 + r, n = n0 + wn0 + cc;
      if (m >= p.M || n >= p.N) continue;
      long row = m;
      if (p.out_s > 1) {
        const uint32_t b = fdiv(m, p.fd_ohw);
        const uint32_t rem = m - b * p.OH * p.OW;
        const uint32_t oh = fdiv(rem, p.fd_ow);
        const uint32_t ow = rem - oh * p.OW;
        row = ((long)b * p.out_H + oh * p.out_s + p.out_ph) * p.out_W + ow * p.out_s + p.out_pw;
      }
      bf16_t* dst = y + row * p.ldy + n;
      const bf16_t* acc_row = accp ? accp + row * p.ldy + n : nullptr;
      const bf16_t* gate_row = gatep ? gatep + row * p.ldy + n : nullptr;
      const bf16_t* src = slab + r * SW + cc;
      if (vec_ok && n + 8 <= p.N) {
        uint4 v = *reinterpret_cast<const uint4*>(src);
        if (gate_row) v = gate_bf16x8(v, *reinterpret_cast<const uint4*>(gate_row));
        if (acc_row) v = add_bf16x8(v, *reinterpret_cast<const uint4*>(acc_row));
        *reinterpret_cast<uint4*>(dst) = v;
      } else {
        for (int t = 0; t < 8 && n + t < p.N; ++t) {
          float o = bf2f(src[t]);
          if (gate_row && !(bf2f(gate_row[t]) > 0.f)) o = 0.f;
          if (acc_row) o += bf2f(acc_row[t]);
          dst[t] = f2bf(o);
        }
      }
    }
    __syncthreads();  // the slab is rewritten for the next row block
  }
}

// VSET: which (A, B) vector widths to instantiate — 0: the 16-B (8,8) gathers every wide layer
// uses; 1: + the 8-B combinations of channel counts ≡ 4 (mod 8) (Transformer d_model = 100);
// 2: every combination incl. scalar (stem-less narrow layers, LeNet).
template <int BM, int BN, int BK, int WM, int WN, int DEPTH, int VSET>
bool launch_cfg(const ConvNTParams& p, int K, int va, int vb, bool bkm, hipStream_t s) {
  const int grid = K * cdiv(p.M, BM) * cdiv(p.N, BN);
#define NT_CASE(A, B)                                                                                           \
  if (va == A && vb == B) {                                                                                     \
    if (bkm)                                                                                                    \
      hipLaunchKernelGGL((conv_nt_kernel<BM, BN, BK, WM, WN, A, B, true, DEPTH>), dim3(grid), dim3(WM * WN * 64), \
                         0, s, p);                                                                              \
    else                                                                                                        \
      hipLaunchKernelGGL((conv_nt_kernel<BM, BN, BK, WM, WN, A, B, false, DEPTH>), dim3(grid),                   \
                         dim3(WM * WN * 64), 0, s, p);                                                          \
    return true;                                                                                                \
  }
  NT_CASE(8, 8)
  if constexpr (VSET >= 1) { NT_CASE(4, 4) NT_CASE(8, 4) NT_CASE(4, 8) }  // d_model = 100 style widths
  if constexpr (VSET >= 2) { NT_CASE(8, 1) NT_CASE(4, 1) NT_CASE(1, 8) NT_CASE(1, 1) }
#undef NT_CASE
  return false;
}

// Tile configurations (variant ids are stable: the microbenchmark sweeps them)
bool launch_variant(int v, const ConvNTParams& p, int K, int va, int vb, bool bkm, hipStream_t s) {
  switch (v) {
    case 0: return launch_cfg<128, 128, 64, 2, 2, 1, 1>(p, K, va, vb, bkm, s);
    case 1: return launch_cfg<128, 64, 64, 4, 1, 1, 0>(p, K, va, vb, bkm, s);
    case 2: return launch_cfg<128, 64, 64, 4, 1, 2, 0>(p, K, va, vb, bkm, s);
    case 3: return launch_cfg<256, 128, 64, 4, 2, 1, 0>(p, K, va, vb, bkm, s);
    case 4: return launch_cfg<128, 128, 32, 2, 2, 1, 0>(p, K, va, vb, bkm, s);
    case 5: return launch_cfg<64, 64, 64, 2, 2, 1, 0>(p, K, va, vb, bkm, s);
    case 6: return launch_cfg<128, 128, 32, 2, 2, 1, 2>(p, K, va, vb, bkm, s);
    case 7: return launch_cfg<128, 64, 32, 2, 1, 1, 2>(p, K, va, vb, bkm, s);
    case 8: return launch_cfg<256, 64, 64, 4, 1, 1, 0>(p, K, va, vb, bkm, s);
    case 9: return launch_cfg<256, 64, 32, 4, 1, 1, 0>(p, K, va, vb, bkm, s);
    case 10: return launch_cfg<256, 128, 32, 4, 2, 1, 1>(p, K, va, vb, bkm, s);
    case 11: return launch_cfg<128, 128, 64, 2, 2, 0, 0>(p, K, va, vb, bkm, s);
    case 12: return launch_cfg<256, 128, 32, 4, 2, 0, 0>(p, K, va, vb, bkm, s);
    case 13: return launch_cfg<64, 64, 64, 2, 2, 0, 1>(p, K, va, vb, bkm, s);
    case 14: return launch_cfg<256, 64, 32, 4, 1, 0, 0>(p, K, va, vb, bkm, s);
    case 15: return launch_cfg<256, 128, 64, 4, 2, 0, 0>(p, K, va, vb, bkm, s);
    case 16: return launch_cfg<128, 128, 64, 2, 2, 0, 0>(p, K, va, vb, bkm, s);
    case 17: return launch_cfg<128, 64, 64, 2, 1, 0, 0>(p, K, va, vb, bkm, s);
    case 18: return launch_cfg<256, 32, 64, 4, 1, 0, 2>(p, K, va, vb, bkm, s);  // N <= 32 (DenseNet k=12)
    default: return false;
  }
}
// measured on MI355X (bench/kernel_bench.py --sweep, ResNet-18 shapes, K=100 clients):
// depth-2 register prefetch halves occupancy (≈190 VGPRs ⇒ 1 wave/SIMD) and loses ≈45%;
// the 128x128 BK64 depth-1 tile reaches 560-600 TFLOP/s on the 3x3 layers.

int vec_width(int c) { return (c % 8 == 0) ? 8 : (c % 4 == 0) ? 4 : 1; }


// Transposed, flipped split weight planes of a 3x3 conv for its stride-1 dgrad: wt[k][plane][ci][8 − t][co] =
// w[k][plane][co][t][ci] (t = 3·kh + kw). The dgrad then runs the FORWARD (row-major B) tiles:
// dX = conv(dY, wt) — the k-major B path of the dgrad tiles is 11-20 % slower on the same shapes
// (bench/epilogue_bench.py dgrad vs fwd, r4_c7_epi.log). 32 x 32 (co, ci) tiles through LDS.
__global__ void __launch_bounds__(256) wt_planes_kernel(const bf16_t* __restrict__ ws, long ws_cs, long ws_plane,
                                                        bf16_t* __restrict__ wt, int Co, int Ci) {
  __shared__ bf16_t tile[32][34];
  const int t = blockIdx.x % 9, kp = blockIdx.x / 9;  // (client row, plane)
  const int plane = kp & 1, k = kp >> 1;
  const int co0 = blockIdx.y * 32, ci0 = blockIdx.z * 32;
  const bf16_t* src = ws + (long)k * ws_cs + plane * ws_plane;
  bf16_t* dst = wt + ((long)k * 2 + plane) * 9L * Ci * Co;
  const int c = threadIdx.x & 31, r0 = threadIdx.x >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + 8 * j;
    tile[r][c] = src[((long)(co0 + r) * 9 + t) * Ci + ci0 + c];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + 8 * j;  // ci row of the output
    dst[((long)(ci0 + r) * 9 + (8 - t)) * Co + co0 + c] = tile[c][r];
  }
}
}  // namespace

int conv_nt_num_variants() { return 19; }

int conv_nt_default_variant(int M, int N, int R, int b_kmajor) {
  // measured (profiles/kernel_bench_resnet18_sweep.jsonl): forward wants 64-deep K tiles (B rows
  // are 128-B lines), dgrad's k-major B streams full lines at any depth and prefers 256-row tiles
  // N <= 64 (ResNet l1, stride-2 dgrad classes): single-LDS-buffer 64x64 tiles, 4 blocks/CU
  // (l1 fwd 428 vs 364, dgrad 376 vs 331 TFLOP/s for the double-buffered 64x64 / 256x64)
  if (N <= 64) return 13;  // (the 32-wide v18 measured slower on DenseNet's 12-channel outputs)
  if (b_kmajor) return 10;  // 256x128 BK32: l3 dgrad 672 vs 564 TFLOP/s (128x128)
  return 0;                 // 128x128 BK64 (l3 fwd 600)
}

void conv_nt(ConvNTParams p, int K, int variant, hipStream_t s) {
  if (p.wKH == 0) {  // plain launch: symmetric padding, full-flip dgrad tap order
    p.pad_w = p.pad;
    p.wKH = p.KH;
    p.wKW = p.KW;
    p.kh_off = p.KH - 1;
    p.kw_off = p.KW - 1;
    p.kh_step = p.kw_step = 1;
  }
  if (p.out_s == 0) p.out_s = 1;
  if (p.ldx == 0) p.ldx = p.C;
  if (p.ldy == 0) p.ldy = p.N;
  p.fd_ohw = make_fastdiv((uint32_t)(p.OH * p.OW));
  p.fd_ow = make_fastdiv((uint32_t)p.OW);
  p.fd_kwc = make_fastdiv((uint32_t)(p.KW * p.C));
  p.fd_c = make_fastdiv((uint32_t)p.C);
  if (p.f32) {  // reference precision: split-bf16 MFMA kernels (conv_f32.hip)
    conv_nt_f32(p, K, variant, s);
    return;
  }
  if (p.stats) {  // epilogue BN statistics exist in the fp32 kernels only (callers check)
    fprintf(stderr, "conv_nt: epilogue statistics need the fp32 kernels\n");
    abort();
  }
  const bool bkm = p.b_kmajor != 0;
  int va = vec_width(std::gcd(p.C, p.ldx));  // vectors must not straddle a channel-sliced pixel
  int vb = bkm ? vec_width(p.N) : vec_width(p.R);
  if (va == 1 && vb == 4) vb = 1;
  if (variant < 0) {
    variant = conv_nt_default_variant(p.M, p.N, p.R, p.b_kmajor);
    // (at 13 clients per launch the wide tiles stay faster even below 2 blocks/CU:
    // profiles/kernel_bench_resnet18_sweep_K13.jsonl)
    (void)K;
  }
  // narrow / scalar-gather layers (stem, LeNet, tiny linears) keep the small-K-tile config
  const bool w84 = (va == 8 || va == 4) && (vb == 8 || vb == 4);  // covered by VSET 1 variants
  if (w84 && !(va == 8 && vb == 8) && !(variant == 0 || variant == 10 || variant == 13 || variant == 6 ||
                                        variant == 7 || variant == 18)) {
    variant = (p.N <= 64) ? 13 : (bkm ? 10 : 0);
  } else if (!w84 && !(variant == 6 || variant == 7 || variant == 18)) {
    variant = (p.N <= 64) ? 7 : 6;
  }
  if (!launch_variant(variant, p, K, va, vb, bkm, s)) fprintf(stderr, "conv_nt: bad variant %d\n", variant);
}

void wt_planes(const bf16_t* wsplit, long ws_cs, long ws_plane, bf16_t* wt, int Kw, int Co, int Ci, hipStream_t s) {
  hipLaunchKernelGGL(wt_planes_kernel, dim3(Kw * 2 * 9, Co / 32, Ci / 32), dim3(256), 0, s, wsplit, ws_cs, ws_plane, wt,
                     Co, Ci);
}

void conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const bf16_t* acc, long w_cs, int K, int rep, int B, int OH, int OW,
                int Co, int H, int W, int Ci, int KH, int KW, int stride, int pad, int variant, int f32, hipStream_t s,
                int ld_dy, long dy_cs, const bf16_t* wsplit, long ws_cs, long ws_plane, long x_lo, int acc_compact,
                const BNBwdPartials* bnb, bf16_t* wt_buf, const uint8_t* acc_mask, int wt_ready) {
  ConvNTParams p{};
  p.acc_mask = acc_mask;
  if (bnb) {  // (the epilogue's partial rows are the dX rows of a single stride-1 launch)
    if (!f32 || stride != 1 || Ci % 4 != 0 || (bnb->mask && Ci % 8 != 0) || (bnb->xld && bnb->xld % 4 != 0)) {
      fprintf(stderr, "conv_dgrad: BN-backward partials need an fp32 stride-1 dgrad with Ci %% 4 == 0\n");
      abort();
    }
    p.bnb = bnb->part;
    p.bnb_x = bnb->x;
    p.bnb_xld = bnb->xld ? bnb->xld : Ci;
    p.bnb_y = bnb->y;
    p.bnb_mask = bnb->mask;
    p.bnb_mean = bnb->mean;
    p.bnb_rstd = bnb->rstd;
    p.bnb_valid = bnb->valid;
    // dX feeds that BatchNorm's backward alone, which stops at the valid rows (halo tiles past
    // them skip their MFMA work)
    if (stride == 1 && bnb->valid && native_option(g_opt_halo_skip, "DLS_SKIP_INVALID", 1)) {
      p.skip_valid = bnb->valid;
      p.skip_mul = 1;
    }
  }
  p.x_lo = x_lo;
  p.wsplit = wsplit;  // (fp32 kernels: pre-split weight planes, read k-major in place like w)
  p.ws_cs = ws_cs;
  p.ws_plane = ws_plane;
  p.f32 = f32;
  p.ldx = ld_dy;  // dY may be a channel slice of a wider buffer (DenseNet block)
  p.x = dy;
  p.w = w;
  p.y = dx;
  p.bias = nullptr;
  p.acc = acc;
  p.x_cs = dy_cs ? dy_cs : (long)B * OH * OW * (ld_dy ? ld_dy : Co);
  p.y_cs = (long)B * H * W * Ci;
  p.w_cs = w_cs;
  p.b_cs = 0;
  p.B = B;
  p.H = OH;  // the GEMM's A image is dY
  p.W = OW;
  p.C = Co;
  p.N = Ci;
  p.rep = rep;
  p.relu = 0;
  p.b_kmajor = 1;
  p.wKH = KH;
  p.wKW = KW;
  p.dil = 1;
  p.stride = 1;
  if (stride == 1) {
    // dX = full correlation of dY with the flipped kernel
    p.OH = H;
    p.OW = W;
    p.KH = KH;
    p.KW = KW;
    p.pad = KH - 1 - pad;
    p.pad_w = KW - 1 - pad;
    p.kh_off = KH - 1;
    p.kw_off = KW - 1;
    p.kh_step = p.kw_step = 1;
    p.out_s = 1;
    p.M = B * H * W;
    p.R = KH * KW * Co;
    // N <= 64 full-correlation dgrad (ResNet l1): the 256x64 BK32 single-buffer tile streams the
    // k-major weight rows best — l1 dgrad 420-435 vs 377-385 TFLOP/s for the 64x64 tile at 13 and
    // 100 clients (bench/kernel_bench.py --sweep); the stride-2 parity classes keep the 64x64 tile
    if (variant < 0 && !f32 && Ci <= 64 && vec_width(Ci) == 8 && vec_width(Co) == 8) variant = 14;
    if (wt_buf && f32 && x_lo != 0 && wsplit && KH == 3 && KW == 3 && pad == 1 && Co % 32 == 0 && Ci % 32 == 0) {
      // transposed flipped weight planes → the forward (row-major B) tiles
      // (wt_ready: built earlier by wt_planes — before a fused SGD step rewrote the weight planes)
      const int Kw = K / rep;
      if (!wt_ready)
        hipLaunchKernelGGL(wt_planes_kernel, dim3(Kw * 2 * 9, Co / 32, Ci / 32), dim3(256), 0, s, wsplit, ws_cs,
                           ws_plane, wt_buf, Co, Ci);
      p.b_kmajor = 0;
      p.wsplit = wt_buf;
      p.ws_cs = 2L * 9 * Ci * Co;
      p.ws_plane = 9L * Ci * Co;
      p.w = wt_buf;  // (unused by the plane kernels; never the k-major forward weight)
      p.w_cs = p.ws_cs;
    }
    conv_nt(p, K, variant, s);
    return;
  }
  // Parity class (ph, pw): dx pixels ih = s·oh' + ph receive only taps kh ≡ ph+pad (mod s):
  // kh = kh0 + s·j, dy row = oh' + (ph+pad-kh0)/s - j. Reversing j makes it a stride-1
  // correlation with pad' = nkh-1-(ph+pad-kh0)/s over the class subgrid.
  for (int ph = 0; ph < stride; ++ph) {
    const int Hc = (H - ph + stride - 1) / stride;
    if (Hc <= 0) continue;
    const int kh0 = (ph + pad) % stride;
    const int nkh = kh0 < KH ? (KH - kh0 + stride - 1) / stride : 0;
    const int dh = (ph + pad - kh0) / stride;
    for (int pw = 0; pw < stride; ++pw) {
      const int Wc = (W - pw + stride - 1) / stride;
      if (Wc <= 0) continue;
      const int kw0 = (pw + pad) % stride;
      const int nkw = kw0 < KW ? (KW - kw0 + stride - 1) / stride : 0;
      const int dw = (pw + pad - kw0) / stride;
      ConvNTParams q = p;
      q.OH = Hc;
      q.OW = Wc;
      q.M = B * Hc * Wc;
      if (acc_compact) {  // acc: the class-(0, 0) grid only, [K][B][Hc][Wc][Ci]
        q.acc = (ph == 0 && pw == 0) ? acc : nullptr;
        q.acc_compact = 1;
        q.acc_cs = (long)B * Hc * Wc * Ci;
      }
      q.out_s = stride;
      q.out_ph = ph;
      q.out_pw = pw;
      q.out_H = H;
      q.out_W = W;
      if (nkh == 0 || nkw == 0) {  // no tap reaches this class: dx = 0 (R = 0 ⇒ zero accumulators)
        q.KH = q.KW = 1;
        q.R = 0;
        q.pad = q.pad_w = 0;
        q.kh_off = q.kw_off = 0;
        q.kh_step = q.kw_step = 1;
      } else {
        q.KH = nkh;
        q.KW = nkw;
        q.pad = nkh - 1 - dh;
        q.pad_w = nkw - 1 - dw;
        q.kh_off = kh0 + stride * (nkh - 1);
        q.kw_off = kw0 + stride * (nkw - 1);
        q.kh_step = q.kw_step = stride;
        q.R = nkh * nkw * Co;
      }
      conv_nt(q, K, variant, s);
    }
  }
}
