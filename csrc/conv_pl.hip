// fp32-accurate implicit-GEMM convolution / linear on PRE-SPLIT operands for gfx950 (MI355X).
//
// Same arithmetic as conv_f32.hip (split bf16 "bf16x3": a·b ≈ ah·bh + al·bh + ah·bl on
// v_mfma_f32_32x32x16_bf16, fp32 accumulate; products in the same order, so the result is
// bit-identical for the same hi / lo values), but both operands arrive already split into two
// bf16 planes (hi = bf16(x), lo = bf16(x − hi), RNE):
//   A  — the activation (or dY) planes written by the producing BatchNorm (bn_fwd / bn_bwd
//        `planes` outputs): one extra 4-B/element write there replaces the per-workgroup split
//        of every tile that reads the element (3x3 im2col reads each element up to 9× per N tile);
//   B  — the weight planes the SGD step keeps current (sgd_step `split`).
// The loaders are then pure data movement: every 16-B piece goes HBM/L2 → LDS by LDS-DMA
// (`buffer_load_dwordx4 … lds`, per-lane source address, lane-linear LDS destination), so the
// main loop issues no split VALU, no ds_write and holds no staging registers; the DMA of
// stage k+1 (k+2) is in flight under the MFMAs of stage k (guide §5 "Pipelining across
// barriers": counted vmcnt + raw s_barrier, all LDS in ONE __shared__ array).
//
// Buffer resources bound each client's operand window: an out-of-window lane offset (image
// padding taps, M / N tails) makes the DMA write zeros, so no lane is ever masked (a masked
// lane would leave a hole in the lane-linear image).
//
// LDS images (per stage): A hi / lo [BM][32] and B hi / lo [BN][32] (row-major: 64-B rows,
// 16-B chunk c stored at c ^ ((row >> 2) & 3) → conflict-free ds_read_b128 fragment reads) or,
// for a k-major B (dgrad reading the forward weight in place), B hi / lo [32][BN] read by
// ds_read_b64_tr_b16 with the 32-element segment XOR-swizzled by k-row.
//
// Restrictions (the host dispatcher falls back to conv_f32.hip otherwise): C % 32 == 0 (one K
// tile never straddles a tap), pixel stride % 8 == 0, N % 8 == 0, per-client windows < 2 GiB.
#include "dls.h"
#include "epilogue_f32.h"
#include "sgd_epi.h"
#include "gemm_common.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int PK = 32;  // K tile: 32 bf16 per plane row (64 B)

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, 0, 0, 0);
}

// s_waitcnt with only vmcnt = N (expcnt / lgkmcnt left at their maxima), gfx9 encoding
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// conv_nt_pl_kernel<…, PIX>: pixel-major GEMM rows (ConvNTParams::pix). Row m is image m % B at
// pixel m / B, so a tile covers a few pixels of every image and each 32-row group (B % 32 == 0)
// one pixel. The K walk visits only the box of taps that lands inside the image for some row of
// the tile, and each wave skips the MFMAs (and A fragment reads) of its groups whose pixels the
// stage's tap misses. A skipped tap's rows are all out of the image, i.e. zeros: the sums are the
// ones the full walk forms, term for term. On 4x4 images with 3x3 taps the walk keeps 30 of 36
// taps per 256-row tile at B = 64 (every tap of a one-pixel tile past B = 256) and the MFMAs 100
// of 144.
template <int BM, int BN, int WM, int WN, bool BKM, int NST, int MINW, bool ILV, int PKT, bool PIX = false>
__global__ void __launch_bounds__(WM* WN * 64, MINW) conv_nt_pl_kernel(ConvNTParams p) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  static_assert(PKT == 16 || PKT == 32, "K tile");
  constexpr int A_PL = BM * PKT * 2, B_PL = BN * PKT * 2;  // bytes per plane image
  constexpr int STAGE = 2 * (A_PL + B_PL);
  // row-major images: PKT·2-byte rows, CR 16-B chunks per row, RI rows per 1-KiB DMA
  // instruction, RB rows per 256-B bank row; chunk c of row r stored at c ^ ((r / RB) % CR)
  constexpr int CR = PKT / 8, RI = 64 / CR, RB = 256 / (PKT * 2);
  constexpr int AI = BM / RI / NW;  // DMA instructions per wave per plane (1 KiB each)
  constexpr int BI = BN * PKT / 512 / NW;
  static_assert(AI * RI * NW == BM && BI * 512 * NW == BN * PKT, "DMA split");
  constexpr int G = 2 * (AI + BI);  // DMA instructions per wave per stage
  constexpr int SW = TN * 32 + 4;
  constexpr int EPI = NW * 32 * SW * 4;
  constexpr int SMEM = NST * STAGE > EPI ? NST * STAGE : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tilesM = (p.M + BM - 1) / BM, tilesN = (p.N + BN - 1) / BN;
  const int per_client = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  const int t = bid - client * per_client;
  int mt = t / tilesN;
  if constexpr (PIX) {
    // one-pixel tiles (B % BM == 0, >= 256 images per client): the tiles of every pixel of one image
    // chunk are consecutive, so they run together on one XCD and the input rows their taps share are
    // read from its L2
    if (p.B % BM == 0) {
      const int npix = p.OH * p.OW;
      mt = (mt % npix) * (p.B / BM) + mt / npix;
    }
  }
  const int m0 = mt * BM, n0 = (t % tilesN) * BN;

  // ---- operand windows (hi plane .. end of lo plane) as buffer resources
  const long a_img = (long)p.B * p.H * p.W * p.ldx;  // elements of one plane of a client's image
  const auto ar = make_rsrc(p.x + (long)client * p.x_cs, (uint32_t)((p.x_lo + a_img) * 2));
  const uint32_t a_lo = (uint32_t)(p.x_lo * 2);
  const long w_ext = BKM ? (long)p.C * p.wKH * p.wKW * p.N : (long)p.N * p.R;
  const auto br = make_rsrc(p.wsplit + (long)(client / p.rep) * p.ws_cs, (uint32_t)((p.ws_plane + w_ext) * 2));
  const uint32_t b_lo = (uint32_t)(p.ws_plane * 2);

  // ---- A loader: instruction i of wave w fills tile rows (i·NW + w)·RI + lane / CR, physical
  // chunk lane % CR, fetching logical chunk lc = (lane % CR) ^ ((row / RB) % CR) = … ^ ((lane >> 4) % CR)
  const int lc = (lane % CR) ^ ((lane >> 4) % CR);
  int a_off[AI], a_ih[AI], a_iw[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (i * NW + wid) * RI + lane / CR;
    if (m < p.M) {
      uint32_t b, oh, ow;
      if constexpr (PIX) {
        const uint32_t px = fdiv((uint32_t)m, p.fd_pb);
        b = (uint32_t)m - px * (uint32_t)p.B;
        oh = fdiv(px, p.fd_ow);
        ow = px - oh * (uint32_t)p.OW;
      } else {
        b = fdiv((uint32_t)m, p.fd_ohw);
        const uint32_t rem = (uint32_t)m - b * (uint32_t)(p.OH * p.OW);
        oh = fdiv(rem, p.fd_ow);
        ow = rem - oh * (uint32_t)p.OW;
      }
      a_ih[i] = (int)oh * p.stride - p.pad;
      a_iw[i] = (int)ow * p.stride - p.pad_w;
      a_off[i] = (((int)b * p.H + a_ih[i]) * p.W + a_iw[i]) * p.ldx + lc * 8;
    } else {
      a_ih[i] = -(1 << 28);  // never inside the image
      a_iw[i] = 0;
      a_off[i] = 0;
    }
  }
  // ---- B loader
  // row-major [N][R]: rows (i·NW + w)·16 + (lane >> 2), same chunk swizzle as A
  // k-major [k][N] (dgrad, the forward weight W[co][kh][kw][ci] read in place): instruction i
  // covers k-rows (i·NW + w)·RPI + lane / CPR, physical chunk lane % CPR
  constexpr int CPR = BN / 8, RPI = BKM ? 64 / CPR : RI;
  constexpr int SD = (128 / BN) > 1 ? 128 / BN : 1, SS = (BN / 32) < 4 ? BN / 32 : 4;  // k-major swizzle
  int b_off[BI];
  const long wkhwn = (long)p.wKH * p.wKW * p.N;  // element distance of one input channel (k-major)
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    if constexpr (!BKM) {
      const int n = n0 + (i * NW + wid) * RI + lane / CR;
      b_off[i] = n < p.N ? n * p.R + lc * 8 : -1;
    } else {
      const int kr = (i * NW + wid) * RPI + lane / CPR;
      const int f = SS > 1 ? (kr / SD) & (SS - 1) : 0;
      const int n = n0 + ((lane % CPR) ^ (f << 2)) * 8;
      b_off[i] = n < p.N ? (int)(kr * wkhwn) + n : -1;
    }
  }

  // PIX: the taps (kh, kw) that land inside the image for some row in rows [r0, r1] form a box
  // (the rows' pixels are a contiguous run in row-major pixel order); empty when r0 > r1
  struct TapBox {
    int h0, h1, w0, w1;
  };
  auto tap_box = [&](int r0, int r1) -> TapBox {
    if (r0 > r1) return TapBox{1, 0, 1, 0};
    const int p0 = r0 / p.B, p1 = r1 / p.B;
    const int oh0 = p0 / p.OW, oh1 = p1 / p.OW;
    const int ow0 = oh0 == oh1 ? p0 - oh0 * p.OW : 0, ow1 = oh0 == oh1 ? p1 - oh1 * p.OW : p.OW - 1;
    return TapBox{max(0, p.pad - oh1 * p.stride), min(p.KH - 1, p.H - 1 + p.pad - oh0 * p.stride),
                  max(0, p.pad_w - ow1 * p.stride), min(p.KW - 1, p.W - 1 + p.pad_w - ow0 * p.stride)};
  };
  TapBox tb{0, p.KH - 1, 0, p.KW - 1};
  if constexpr (PIX) tb = tap_box(m0, min(m0 + BM, p.M) - 1);

  // K-tile walk: taps (kh, kw) × 32-channel chunks kc of the GEMM's A image (C % 32 == 0).
  // prep() fixes the scalar part of the next stage's source offsets and advances the walk;
  // piece(n, buf) issues that stage's n-th DMA (n < G: A hi / lo per A instruction, then B hi /
  // lo per B instruction). A stage past the last K tile is issued with every lane out of window
  // (zeros into a buffer nobody reads again), so the loop needs no branch around its DMAs.
  // (PIX: the walk covers the tile's tap box only; k_next, the row-major B offset, follows it)
  int kc = 0, kh = tb.h0, kw = tb.w0, k_next = (tb.h0 * p.KW + tb.w0) * p.C;
  int s_toff = 0, s_boff = 0, s_kh = 0, s_kw = 0;
  bool s_live = false;
  auto prep = [&](bool live) {
    s_live = live;
    s_kh = kh;
    s_kw = kw;
    s_toff = (kh * p.W + kw) * p.ldx + kc;
    if constexpr (!BKM) {
      s_boff = k_next;
    } else {
      const int khh = p.kh_off - p.kh_step * kh, kww = p.kw_off - p.kw_step * kw;
      s_boff = (int)(kc * wkhwn) + (khh * p.wKW + kww) * p.N;
    }
    k_next += PKT;
    kc += PKT;
    if (kc == p.C) {
      kc = 0;
      if (++kw > tb.w1) {
        kw = tb.w0;
        ++kh;
        if constexpr (PIX) k_next = (kh * p.KW + kw) * p.C;
      }
    }
  };
  auto piece = [&](int n, int buf) {
    unsigned char* As = smem + buf * STAGE;
    unsigned char* Bs = As + 2 * A_PL;
    if (n < 2 * AI) {
      const int i = n >> 1;
      const bool ok = s_live && (unsigned)(a_ih[i] + s_kh) < (unsigned)p.H && (unsigned)(a_iw[i] + s_kw) < (unsigned)p.W;
      const uint32_t off = (uint32_t)(a_off[i] + s_toff) * 2u + ((n & 1) ? a_lo : 0u);
      dma16(ar, As + (n & 1) * A_PL + (i * NW + wid) * 1024, ok ? off : OOB_OFF);
    } else {
      const int i = (n - 2 * AI) >> 1;
      const bool ok = s_live && b_off[i] >= 0;
      const uint32_t off = (uint32_t)(b_off[i] + s_boff) * 2u + ((n & 1) ? b_lo : 0u);
      dma16(br, Bs + (n & 1) * B_PL + (i * NW + wid) * 1024, ok ? off : OOB_OFF);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const int wm0 = (wid / WN) * (TM * 32), wn0 = (wid % WN) * (TN * 32);
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = lane >> 5;
  const int rsw = ((lane & 31) / RB) % CR;  // row-major image key of fragment row (lane & 31)
  constexpr int KS = PKT / 16, NTRI = KS * TM * TN;  // MFMA triples per K tile
  // compute(buf, nb): the MFMAs of stage buf; with ILV the next stage's G DMAs (into buffer nb)
  // are spread over the MFMA triples (piece n after triple n·NTRI/G) instead of issued as one
  // burst after the barrier, so the DMA issue overlaps the matrix pipe
  // PIX: each 32-row group's tap box; the stage being computed is at tap (c_kh, c_kw)
  TapBox gb[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    gb[i] = TapBox{0, p.KH - 1, 0, p.KW - 1};
    if constexpr (PIX) gb[i] = tap_box(m0 + wm0 + i * 32, min(m0 + wm0 + i * 32 + 32, p.M) - 1);
  }
  int c_kc = 0, c_kh = tb.h0, c_kw = tb.w0;
  auto group_on = [&](int i) -> bool {
    if constexpr (!PIX) return true;
    return c_kh >= gb[i].h0 && c_kh <= gb[i].h1 && c_kw >= gb[i].w0 && c_kw <= gb[i].w1;
  };
  auto compute = [&](int buf, int nb) {
    const unsigned char* As = smem + buf * STAGE;
    const unsigned char* Bs = As + 2 * A_PL;
    bool on[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) on[i] = group_on(i);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int ch = ((ks * 2 + h) ^ rsw) * 16;
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (PIX && !on[i]) continue;
        const unsigned char* a = As + (wm0 + i * 32 + (lane & 31)) * (PKT * 2) + ch;
        ah[i] = *reinterpret_cast<const bf16x8*>(a);
        al[i] = *reinterpret_cast<const bf16x8*>(a + A_PL);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (!BKM) {
          const unsigned char* b = Bs + (wn0 + j * 32 + (lane & 31)) * (PKT * 2) + ch;
          bh[j] = *reinterpret_cast<const bf16x8*>(b);
          bl[j] = *reinterpret_cast<const bf16x8*>(b + B_PL);
        } else {
          const int kr = ks * 16 + 8 * h + q;  // (kr + 4 has the same swizzle key)
          const int f = SS > 1 ? (kr / SD) & (SS - 1) : 0;
          const int col = (wn0 + j * 32 + 16 * (g & 1) + 4 * pp) ^ (f << 5);
          const bf16_t* b0 = reinterpret_cast<const bf16_t*>(Bs) + kr * BN + col;
          bh[j] = tr_frag(b0, b0 + 4 * BN);
          bl[j] = tr_frag(b0 + B_PL / 2, b0 + B_PL / 2 + 4 * BN);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (PIX && !on[i]) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          if constexpr (ILV) {
            static_assert(!ILV || !PIX, "the interleaved DMAs must issue with every triple");
            const int tri = (ks * TM + i) * TN + j;
#pragma unroll
            for (int n = 0; n < G; ++n)
              if ((n * NTRI) / G == tri) {
                piece(n, nb);
                __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // the triple's MFMAs ...
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // ... then this DMA
              }
          }
        }
      }
    }
    if constexpr (PIX) {  // (the computed stage's walk position, one stage behind prep's)
      c_kc += PKT;
      if (c_kc == p.C) {
        c_kc = 0;
        if (++c_kw > tb.w1) {
          c_kw = tb.w0;
          ++c_kh;
        }
      }
    }
  };

  // ---- main loop: NST-stage LDS ring. Stage kt+NST-1 is issued after the barrier that retires
  // every wave's reads of its buffer (compute(kt-1)); stage kt is waited for by a counted vmcnt
  // that leaves the younger stage in flight (NST = 3)
  const int nk = PIX ? (tb.h1 - tb.h0 + 1) * (tb.w1 - tb.w0 + 1) * (p.C / PKT) : p.R / PKT;
#pragma unroll
  for (int st = 0; st < NST - 1; ++st) {
    prep(st < nk);
#pragma unroll
    for (int n = 0; n < G; ++n) piece(n, st);
  }
  for (int kt = 0; kt < nk; ++kt) {
    wait_vm<G*(NST - 2)>();
    __builtin_amdgcn_s_barrier();
    const int nb = (kt + NST - 1) % NST;
    prep(kt + NST - 1 < nk);
    if constexpr (!ILV) {
#pragma unroll
      for (int n = 0; n < G; ++n) piece(n, nb);
    }
    compute(kt % NST, nb);
  }
  wait_vm<0>();

  nt_f32_epilogue<TM, TN, NW, -1, true, PIX>(p, acc, smem, client, m0, n0, wm0, wn0, wid, lane);
}

template <int BM, int BN, int WM, int WN, int NST, bool ILV = false, int PKT = 32, int MINW = 1, bool PIX = false>
void launch_pl(const ConvNTParams& p, int K, bool bkm, hipStream_t s) {
  const int grid = K * cdiv(p.M, BM) * cdiv(p.N, BN);
  if (bkm)
    hipLaunchKernelGGL((conv_nt_pl_kernel<BM, BN, WM, WN, true, NST, MINW, ILV, PKT, PIX>), dim3(grid),
                       dim3(WM * WN * 64), 0, s, p);
  else
    hipLaunchKernelGGL((conv_nt_pl_kernel<BM, BN, WM, WN, false, NST, MINW, ILV, PKT, PIX>), dim3(grid),
                       dim3(WM * WN * 64), 0, s, p);
}

}  // namespace

static int g_pl_variant = -1;
int conv_nt_pl_variant() { return g_pl_variant; }
void conv_nt_pl_set_variant(int v) { g_pl_variant = v; }

// variant ids are stable (bench/kernel_bench.py --planes sweeps them)
int conv_nt_pl_num_variants() { return 8; }

bool conv_nt_pl_supported(const ConvNTParams& p) {
  return p.x_lo != 0 && p.wsplit != nullptr && p.dil == 1 && p.C % PK == 0 && p.ldx % 8 == 0 &&
         p.N % 8 == 0 && (p.R == p.KH * p.KW * p.C || p.R == 0);
}

// measured (bench/kernel_bench.py --f32 --planes, ResNet-18 layers at 50 clients): N <= 64 the
// 256x64 tile (l1 fwd / dgrad 253 / 238 TFLOP/s vs 168 / 165 for 128x128); N >= 512 the 256x256
// tile (l4 354 / 297 vs 333 / 278); otherwise 128x128 at 2 blocks per CU (l3 331 / 291 vs 309 /
// 249 for 256x128)
// Small cohorts (a rank's share of a multi-GPU round: 100 clients / 8 ranks / 2 streams ≈ 6-7 per
// launch) leave the 256x256 grid far below the 256 CUs: below 192 workgroups N >= 512 takes the
// 128x128 tile (l4 at 7 clients: fwd / dgrad 282 / 213 vs 127 / 107 TFLOP/s; at 50 clients the
// 256x256 tile keeps 380 / 325 vs 350 / 303, profiles/r3_kernel_bench_small_cohort_kref.log).
// 192 rather than 256 since the pixel-major walk: a 2-rank share (25 clients per launch, 200 l4
// workgroups) runs 1779 → 1732 ms per round on the 256x256 tile, while the 4- and 8-rank shares
// (96-104 and 56 workgroups) stay on 128x128 (threshold 96 / 48 measured +1.4 / +7.6 % there,
// profiles/r6_c17_pl_min_wg.txt). DLS_PL_MIN_WG overrides it (0 = always 256x256)
static int pl_min_wg() {
  return native_option(g_opt_pl_min_wg, "DLS_PL_MIN_WG", 192);
}

// Large-M launches (>= 128 K rows per client: ResNet-50's 56x56 layers at 128 images per client;
// bench/eval_tiles_bench.py at 8192 images, bench/r50_kernel_bench.py --nt-variants,
// profiles/r6_c11_eval_tiles.log, r6_c11_r50_layer_variants.log): N = 256 also takes the 256x256
// tile (l3a 3.63 vs 4.06 ms; ResNet-50 l1.c3 fwd 0.97 vs 1.07) and the 3x3 N = 128 conv the 3-stage
// interleaved 256x128 tile (l2a 2.36 vs 2.53; the 1x1 shortcut keeps 128x128, 0.84 vs 0.97)
int conv_nt_pl_default_variant(const ConvNTParams& p, int K) {
  if (p.N <= 64) return 2;
  if (p.N >= 512) return (long)K * cdiv(p.M, 256) * cdiv(p.N, 256) < pl_min_wg() ? 1 : 3;
  if (p.M >= (1 << 17)) {
    if (p.N >= 256) return 3;
    if (p.KH * p.KW > 1) return 4;
  }
  return 1;
}

// pixel-major rows with tap skipping (conv_nt_pl_kernel PIX) for stride-1 convs on small images,
// where the image border holds a large share of the tap-pixels: 3x3 on 4x4 (ResNet-18 l4) keeps 100
// of 144. Measured (bench/pix_bench.py, profiles/r6_c10_pix_bench.log): the 256x256 tile gains on l4
// (fwd / dgrad 1.03 / 1.06x at 50 clients, 1.15x at 8192 images per client); the 128x128 tile of small cohorts loses
// (0.87 / 0.94x at 7 clients: a 2-pixel tile's tap box is mostly the full 3x3) and so do the strided
// forwards (l4a 0.97x, 0.91x at 8192 images), which keep the plain walk. Not for the sub-pixel dgrad classes,
// compact shortcut gradients or dropout (their epilogues index GEMM rows). conv_pix = 0 turns it off
static bool pix_ok(const ConvNTParams& p, int variant) {
  return native_option(g_opt_conv_pix, "DLS_CONV_PIX", 1) != 0 && variant == 3 && p.stride == 1 &&
         p.OH * p.OW <= 64 && p.KH * p.KW > 1 && (p.pad > 0 || p.pad_w > 0) && p.out_s <= 1 && !p.acc_compact &&
         !(p.drop_p > 0.f) && p.M == p.B * p.OH * p.OW;
}

bool conv_nt_pl(const ConvNTParams& p0, int K, int variant, hipStream_t s) {
  if (!conv_nt_pl_supported(p0)) return false;
  const long ab = (p0.x_lo + (long)p0.B * p0.H * p0.W * p0.ldx) * 2;
  const long wb = (p0.ws_plane + (p0.b_kmajor ? (long)p0.C * p0.wKH * p0.wKW * p0.N : (long)p0.N * p0.R)) * 2;
  if (ab >= (long)OOB_OFF || wb >= (long)OOB_OFF) return false;
  if (variant < 0) variant = conv_nt_pl_default_variant(p0, K);
  const bool bkm = p0.b_kmajor != 0;
  ConvNTParams p = p0;
  p.pix = pix_ok(p0, variant) ? 1 : 0;
  if (p.pix) {
    p.fd_pb = make_fastdiv((uint32_t)p.B);
    launch_pl<256, 256, 2, 4, 2, false, 32, 1, true>(p, K, bkm, s);
    return true;
  }
  switch (variant) {
    case 0: launch_pl<256, 128, 4, 2, 2>(p, K, bkm, s); break;  // 96 KB, 8 waves
    case 1: launch_pl<128, 128, 2, 2, 2>(p, K, bkm, s); break;  // 64 KB, 2 blocks/CU
    case 2: launch_pl<256, 64, 4, 1, 2>(p, K, bkm, s); break;   // 80 KB, 2 blocks/CU
    case 3: launch_pl<256, 256, 2, 4, 2>(p, K, bkm, s); break;  // 128 KB, 8 waves, 128x64 wave tiles
    // 3 stages, the next-but-one stage's DMAs interleaved with the MFMAs (ILV)
    case 4: launch_pl<256, 128, 4, 2, 3, true>(p, K, bkm, s); break;  // 144 KB
    case 5: launch_pl<256, 256, 2, 4, 4, false, 16>(p, K, bkm, s); break;  // 128 KB: BK 16, 4 stages
    case 6: launch_pl<256, 256, 2, 4, 3, false, 16>(p, K, bkm, s); break;  // 96 KB: BK 16, 3 stages
    case 7: launch_pl<256, 128, 4, 2, 3>(p, K, bkm, s); break;  // 144 KB, 3 stages, DMA burst
    default: return false;
  }
  return true;
}

// ============================================================================ TN (weight gradient)
//   dW[co][r] = Σ_m dY[m][co] · X̃[m][r]   (X̃ = im2col of the layer input, r = (kh, kw, c))
// Both operands are k-major (k = m, the pixel reduction): LDS images A hi / lo [32][BMc] and
// B hi / lo [32][BNr], 32-element segments XOR-swizzled by k-row, fragments by
// ds_read_b64_tr_b16. Each DMA lane keeps one fixed 8-column chunk for the whole kernel (its
// (kh, kw, c) for B), so only the pixel walk m → (b, oh, ow) advances, 32 rows per K tile,
// with carries instead of divisions. Split-K over pixels writes per-split slabs (ConvTNParams::part)
// folded in order by tn_fold: no atomics, bitwise-reproducible.
namespace {

template <int W>
struct KmSwz {  // k-major image of W-element rows: segment key of k-row kr
  static constexpr int SD = (128 / W) > 1 ? 128 / W : 1, SS = (W / 32) < 4 ? W / 32 : 4;
  static __device__ __forceinline__ int f(int kr) { return SS > 1 ? (kr / SD) & (SS - 1) : 0; }
};

// SGD: the direct-store epilogue applies the optimiser step (SgdEpi) instead of storing dW — its
// own instantiation, so the plain kernels compile as if it did not exist (the merged branch cost
// the 128x128 tile 96 → 178 VGPRs and +59 % time in the ResNet-50 sign-SGD profile)
// PIX (ConvTNParams::pix; C % BNr == 0, so the workgroup's columns share one tap (kh, kw)): the
// pixel reduction walks K tiles of (output pixel, 32 images) over only the pixels whose tap input
// lies inside the image — a box — instead of 32 consecutive GEMM rows over every pixel; the
// deterministic split-K cuts that walk into splitk equal runs
template <int BMc, int BNr, int WM, int WN, int NST, bool ILV, bool SGD = false, bool PIX = false>
__global__ void __launch_bounds__(WM* WN * 64) conv_tn_pl_kernel(ConvTNParams p) {
  constexpr int NW = WM * WN;
  constexpr int TM = BMc / (WM * 32), TN = BNr / (WN * 32);
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  constexpr int A_PL = PK * BMc * 2, B_PL = PK * BNr * 2;
  constexpr int STAGE = 2 * (A_PL + B_PL);
  constexpr int AI = BMc / 16 / NW, BI = BNr / 16 / NW;
  static_assert(AI * 16 * NW == BMc && BI * 16 * NW == BNr, "DMA split");
  constexpr int G = 2 * (AI + BI);
  constexpr int CPA = BMc / 8, RPA = 64 / CPA, CPB = BNr / 8, RPB = 64 / CPB;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NST * STAGE];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tilesM = (p.Co + BMc - 1) / BMc, tilesN = (p.R + BNr - 1) / BNr;
  const int per_client = tilesM * tilesN * p.splitk;
  const int nclients = gridDim.x / per_client;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  int t = bid - client * per_client;
  const int split = t % p.splitk;
  t /= p.splitk;
  const int co0 = (t / tilesN) * BMc, r0 = (t % tilesN) * BNr;
  const int mbeg = PIX ? 0 : split * p.m_per_split;
  const int mend = PIX ? p.M : min(p.M, mbeg + p.m_per_split);
  // PIX walk: this tile's tap, the box of output pixels it lands inside for, nbc 32-image chunks per
  // pixel, and this split's run [t_beg, t_end) of the nv·nbc K tiles
  int x_kh = 0, x_kw = 0, x_oh0 = 0, x_ow0 = 0, x_nw = 1, x_nbc = 1, t_beg = 0, t_end = 0;
  if constexpr (PIX) {
    const int tap = r0 / p.C;
    x_kh = tap / p.KW;
    x_kw = tap - x_kh * p.KW;
    int oh1 = p.OH - 1, ow1 = p.OW - 1;
    while (x_oh0 < p.OH && x_oh0 * p.stride - p.pad + x_kh < 0) ++x_oh0;
    while (oh1 >= 0 && oh1 * p.stride - p.pad + x_kh > p.H - 1) --oh1;
    while (x_ow0 < p.OW && x_ow0 * p.stride - p.pad + x_kw < 0) ++x_ow0;
    while (ow1 >= 0 && ow1 * p.stride - p.pad + x_kw > p.W - 1) --ow1;
    x_nw = max(ow1 - x_ow0 + 1, 1);
    const int nv = max(oh1 - x_oh0 + 1, 0) * max(ow1 - x_ow0 + 1, 0);
    x_nbc = (p.B + PK - 1) / PK;
    const int T = nv * x_nbc, tps = (T + p.splitk - 1) / p.splitk;
    t_beg = min(T, split * tps);
    t_end = min(T, t_beg + tps);
  }

  const auto ar = make_rsrc(p.dy + (long)client * p.dy_cs, (uint32_t)((p.dy_lo + (long)p.M * p.ldy) * 2));
  const uint32_t a_lo = (uint32_t)(p.dy_lo * 2);
  const auto br = make_rsrc(p.x + (long)client * p.x_cs, (uint32_t)((p.x_lo + (long)p.B * p.H * p.W * p.ldx) * 2));
  const uint32_t b_lo = (uint32_t)(p.x_lo * 2);

  // ---- A (dY) loader: k-row ka_i, columns co0 + chunk·8
  int a_kr[AI], a_off[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int kr = (i * NW + wid) * RPA + lane / CPA;
    const int co = co0 + ((lane % CPA) ^ (KmSwz<BMc>::f(kr) << 2)) * 8;
    a_kr[i] = co < p.Co ? kr : (1 << 29);  // a column past Co never loads
    a_off[i] = PIX ? kr * p.OH * p.OW * p.ldy + co : (mbeg + kr) * p.ldy + co;  // (PIX: image kr of the chunk)
  }
  // ---- B (im2col X) loader: fixed column chunk → fixed (kh, kw, c); pixel walk per k-row
  constexpr int S = PK;  // pixels per K tile
  const int q_b = S / (p.OH * p.OW), rem_b = S - q_b * p.OH * p.OW;
  const int q_oh = rem_b / p.OW, r_ow = rem_b - q_oh * p.OW;
  const int s_ldx = p.stride * p.ldx, s_row = p.stride * p.W * p.ldx, img = p.H * p.W * p.ldx;
  const int d_iw = r_ow * p.stride, d_off = r_ow * s_ldx + q_oh * s_row + q_b * img;
  const int w_wrap = p.OW * p.stride, off_c1 = s_row - p.OW * s_ldx;
  const int d_ih0 = q_oh * p.stride, d_ih1 = (q_oh + 1) * p.stride;
  const int h_wrap = p.OH * p.stride, off_c2 = img - p.OH * s_row;
  int b_kr[BI], b_ow[BI], b_oh[BI], b_ih[BI], b_iw[BI], b_off[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int kr = (i * NW + wid) * RPB + lane / CPB;
    const int r = r0 + ((lane % CPB) ^ (KmSwz<BNr>::f(kr) << 2)) * 8;
    int kh = 0, kw = 0, c = 0;
    if (r < p.R) {
      kh = r / (p.KW * p.C);
      const int rr = r - kh * p.KW * p.C;
      kw = rr / p.C;
      c = rr - kw * p.C;
    }
    b_kr[i] = r < p.R ? kr : (1 << 29);
    if constexpr (PIX) {  // (image kr of the chunk, channel c; the pixel part is per stage)
      b_off[i] = kr * p.H * p.W * p.ldx + c;
      continue;
    }
    const uint32_t m = mbeg + kr;
    const uint32_t b = fdiv(m, p.fd_ohw);
    const uint32_t rem = m - b * p.OH * p.OW;
    const uint32_t oh = fdiv(rem, p.fd_ow);
    const uint32_t ow = rem - oh * p.OW;
    b_ow[i] = ow;
    b_oh[i] = oh;
    b_ih[i] = (int)oh * p.stride - p.pad + kh;
    b_iw[i] = (int)ow * p.stride - p.pad + kw;
    b_off[i] = (((int)b * p.H + b_ih[i]) * p.W + b_iw[i]) * p.ldx + c;
  }

  int k_rows = mbeg;  // first pixel of the stage being prepared
  bool s_live = false;
  int s_m0 = 0;
  int sa_off[AI], sb_off[BI];
  bool sb_ok[BI];
  // PIX stage state: the scalar offsets of (pixel, first image) in dY and X, the images left
  int t_j = 0, t_bc = 0, s_pa = 0, s_pb = 0, s_left = 0;
  if constexpr (PIX) {
    t_j = t_beg / x_nbc;
    t_bc = t_beg - t_j * x_nbc;
  }
  auto prep = [&](bool live) {
    if constexpr (PIX) {
      s_live = live;
      const int jh = t_j / x_nw, oh = x_oh0 + jh, ow = x_ow0 + (t_j - jh * x_nw);
      const int b0 = t_bc * PK;
      s_left = p.B - b0;
      s_pa = (b0 * p.OH * p.OW + oh * p.OW + ow) * p.ldy;
      s_pb = ((b0 * p.H + oh * p.stride - p.pad + x_kh) * p.W + ow * p.stride - p.pad + x_kw) * p.ldx;
      if (++t_bc == x_nbc) {
        t_bc = 0;
        ++t_j;
      }
      return;
    }
    s_live = live;
    s_m0 = k_rows;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      sa_off[i] = a_off[i];
      a_off[i] += S * p.ldy;
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      sb_ok[i] = (unsigned)b_ih[i] < (unsigned)p.H && (unsigned)b_iw[i] < (unsigned)p.W;
      sb_off[i] = b_off[i];
      // advance this k-row's pixel by S (wave-uniform step constants, carries as selects)
      b_ow[i] += r_ow;
      b_iw[i] += d_iw;
      b_off[i] += d_off;
      const bool c1 = b_ow[i] >= p.OW;
      b_ow[i] -= c1 ? p.OW : 0;
      b_oh[i] += c1 ? q_oh + 1 : q_oh;
      b_iw[i] -= c1 ? w_wrap : 0;
      b_ih[i] += c1 ? d_ih1 : d_ih0;
      b_off[i] += c1 ? off_c1 : 0;
      const bool c2 = b_oh[i] >= p.OH;
      b_oh[i] -= c2 ? p.OH : 0;
      b_ih[i] -= c2 ? h_wrap : 0;
      b_off[i] += c2 ? off_c2 : 0;
    }
    k_rows += S;
  };
  auto piece = [&](int n, int buf) {
    unsigned char* As = smem + buf * STAGE;
    unsigned char* Bs = As + 2 * A_PL;
    if constexpr (PIX) {
      if (n < 2 * AI) {
        const int i = n >> 1;
        const bool ok = s_live && a_kr[i] < s_left;
        const uint32_t off = (uint32_t)(a_off[i] + s_pa) * 2u + ((n & 1) ? a_lo : 0u);
        dma16(ar, As + (n & 1) * A_PL + (i * NW + wid) * 1024, ok ? off : OOB_OFF);
      } else {
        const int i = (n - 2 * AI) >> 1;
        const bool ok = s_live && b_kr[i] < s_left;
        const uint32_t off = (uint32_t)(b_off[i] + s_pb) * 2u + ((n & 1) ? b_lo : 0u);
        dma16(br, Bs + (n & 1) * B_PL + (i * NW + wid) * 1024, ok ? off : OOB_OFF);
      }
      return;
    }
    if (n < 2 * AI) {
      const int i = n >> 1;
      const bool ok = s_live && s_m0 + a_kr[i] < mend;
      const uint32_t off = (uint32_t)sa_off[i] * 2u + ((n & 1) ? a_lo : 0u);
      dma16(ar, As + (n & 1) * A_PL + (i * NW + wid) * 1024, ok ? off : OOB_OFF);
    } else {
      const int i = (n - 2 * AI) >> 1;
      const bool ok = s_live && s_m0 + b_kr[i] < mend && sb_ok[i];
      const uint32_t off = (uint32_t)sb_off[i] * 2u + ((n & 1) ? b_lo : 0u);
      dma16(br, Bs + (n & 1) * B_PL + (i * NW + wid) * 1024, ok ? off : OOB_OFF);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const int wm0 = (wid / WN) * (TM * 32), wn0 = (wid % WN) * (TN * 32);
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = lane >> 5;
  constexpr int KS = PK / 16, NTRI = KS * TM * TN;
  auto compute = [&](int buf, int nb) {
    const bf16_t* As = reinterpret_cast<const bf16_t*>(smem + buf * STAGE);
    const bf16_t* Bs = As + A_PL;  // (element offset 2·A_PL bytes)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int kr = ks * 16 + 8 * h + q;  // (kr + 4 has the same swizzle key)
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
      const int fa = KmSwz<BMc>::f(kr), fb = KmSwz<BNr>::f(kr);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16_t* a0 = As + kr * BMc + ((wm0 + i * 32 + 16 * (g & 1) + 4 * pp) ^ (fa << 5));
        ah[i] = tr_frag(a0, a0 + 4 * BMc);
        al[i] = tr_frag(a0 + A_PL / 2, a0 + A_PL / 2 + 4 * BMc);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bf16_t* b0 = Bs + kr * BNr + ((wn0 + j * 32 + 16 * (g & 1) + 4 * pp) ^ (fb << 5));
        bh[j] = tr_frag(b0, b0 + 4 * BNr);
        bl[j] = tr_frag(b0 + B_PL / 2, b0 + B_PL / 2 + 4 * BNr);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          if constexpr (ILV) {
            const int tri = (ks * TM + i) * TN + j;
#pragma unroll
            for (int n = 0; n < G; ++n)
              if ((n * NTRI) / G == tri) {
                piece(n, nb);
                __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
              }
          }
        }
    }
  };

  const int nk = PIX ? t_end - t_beg : (mend - mbeg + PK - 1) / PK;
#pragma unroll
  for (int st = 0; st < NST - 1; ++st) {
    prep(st < nk);
#pragma unroll
    for (int n = 0; n < G; ++n) piece(n, st);
  }
  for (int kt = 0; kt < nk; ++kt) {
    wait_vm<G*(NST - 2)>();
    __builtin_amdgcn_s_barrier();
    const int nb = (kt + NST - 1) % NST;
    prep(kt + NST - 1 < nk);
    if constexpr (!ILV) {
#pragma unroll
      for (int n = 0; n < G; ++n) piece(n, nb);
    }
    compute(kt % NST, nb);
  }
  wait_vm<0>();

  // ---- epilogue: direct stores (splitk == 1) or this split's slab (deterministic fold)
  const bool slab = p.splitk > 1;
  float* __restrict__ dst = slab ? p.part + ((long)split * nclients + client) * p.Co * p.R
                                 : p.dw + (long)client * p.dw_cs;
  if constexpr (SGD) {  // the optimiser step in place of the dW store (SgdEpi), a tile at a time via LDS
    if (!p.sgd.active[client]) return;
    __syncthreads();  // (every wave's main-loop LDS reads retired: the slabs reuse the stage buffers)
    float* sl = reinterpret_cast<float*>(smem) + wid * 32 * 36;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int rb = co0 + wm0 + i * 32, cbk = r0 + wn0 + j * 32;
        sgd_epi_tile32(p.sgd, client, sl, acc[i][j], (long)rb * p.R + cbk, p.R, p.Co - rb, p.R - cbk);
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = r0 + wn0 + j * 32 + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wm0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (co < p.Co && r < p.R) dst[(long)co * p.R + r] = acc[i][j][e];
      }
    }
}

// deterministic split-K fold: dw[k][i] = Σ_s part[(s·K + k)·CoR + i], s ascending
// (sgd.theta: the fold steps the weights instead of storing dw, SgdEpi)
__global__ void __launch_bounds__(256) tn_fold_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                      long dw_cs, int K, int splitk, long CoR, SgdEpi sgd) {
  const long n4 = CoR / 4;
  const int k = blockIdx.y;
  if (sgd.theta && !sgd.active[k]) return;
  const bool vec = sgd.theta ? (CoR % 4 == 0 && sgd.th_cs % 4 == 0 && sgd.sp_cs % 4 == 0 && sgd.sp_lo % 4 == 0 &&
                                ((uintptr_t)sgd.theta & 15) == 0 && ((uintptr_t)sgd.split & 7) == 0)
                             : (CoR % 4 == 0) && (dw_cs % 4 == 0) && (((uintptr_t)dw & 15) == 0);
  if (vec) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
      float4 a = reinterpret_cast<const float4*>(part + (long)k * CoR)[i];
      for (int sp = 1; sp < splitk; ++sp) {
        const float4 b = reinterpret_cast<const float4*>(part + ((long)sp * K + k) * CoR)[i];
        a.x += b.x;
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
      }
      if (sgd.theta)
        sgd_epi4(sgd, k, 4 * i, a);
      else
        reinterpret_cast<float4*>(dw + (long)k * dw_cs)[i] = a;
    }
  } else {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < CoR; i += (long)gridDim.x * 256) {
      float a = part[(long)k * CoR + i];
      for (int sp = 1; sp < splitk; ++sp) a += part[((long)sp * K + k) * CoR + i];
      if (sgd.theta)
        sgd_epi1(sgd, k, i, a);
      else
        dw[(long)k * dw_cs + i] = a;
    }
  }
}

struct TnPlTile {
  int bm, bn;
};
// (all 64x64 wave tiles: 128x64 / 64x128 wave tiles — half the LDS fragment reads per MFMA, one
// wave per SIMD — measured slower on every ResNet-18 layer at 50 clients: l3 243-271 vs 328,
// l4 253-285 vs 318 TFLOP/s, profiles/r3_kernel_bench_tn_wave_tiles_K50.jsonl)
// 6: 256x256, 8 waves of 128x64 (the NT 256x256 shape: two waves per SIMD, 128 KB)
constexpr TnPlTile kTnPlTiles[] = {{128, 128}, {64, 128}, {128, 128}, {64, 128}, {256, 128}, {128, 256}, {256, 256}};
constexpr int kTnPlVariants = sizeof(kTnPlTiles) / sizeof(kTnPlTiles[0]);

// Co >= 512 at >= 16 clients per launch: the 8-wave 256x256 tile (l4 364 vs 343 TFLOP/s at 50
// clients; a small cohort's split-K reference — tn_kref — would split it, 246)
int tn_pl_default_variant(int K, int Co, int R) {
  (void)R;
  if (Co >= 512 && K >= 16) return 6;
  return Co <= 64 ? 1 : 0;
}

// split-K factor from per-client quantities and a reference cohort KREF (as if KREF clients shared
// the launch): a client's weight gradient — summation order included — is the same whatever
// stream, rank or cohort size trains it, as long as the launch is in the same cohort class.
// KREF = 32 for launches of >= 16 clients (one GPU: 50 per stream; two ranks: 25), 8 below (a rank
// of an 8-GPU round: 6-7 per stream), where KREF 32 leaves the grid a few dozen workgroups:
// at 7 clients l1 / l2 / l3 wgrad 223 / 308 / 324 vs 85 / 125 / 233 TFLOP/s, while at 50 clients
// KREF 8 would cost l2 / l3 6-7 % in slab traffic (profiles/r3_kernel_bench_small_cohort_kref.log).
// So 1-rank and 2-rank runs train bitwise alike; an 8-rank run's weight gradients differ from
// them by summation order only. Co <= 64 (5 tiles per client: l1) takes 8 at any cohort size (236
// vs 216 TFLOP/s at 50 clients).
static int tn_kref(int K, int Co) {
  return (K >= 16 && Co > 64) ? 32 : 8;
}
void tn_pl_split(int K, int Co, int R, int M, int variant, int& splitk, int& mps) {
  const TnPlTile t = kTnPlTiles[variant];
  const long tiles = (long)tn_kref(K, Co) * cdiv(Co, t.bm) * cdiv(R, t.bn);
  splitk = 1;
  const int target = 512;  // ≥ 2 blocks per CU
  if (tiles < target) {
    splitk = (int)((target + tiles - 1) / tiles);
    splitk = min(splitk, max(1, M / (8 * PK)));  // ≥ 8 K tiles per split
  }
  mps = cdiv(M, splitk);
  mps = ((mps + PK - 1) / PK) * PK;
  splitk = cdiv(M, mps);
}

static int g_tn_pl_variant = -1;

}  // namespace

int conv_tn_pl_num_variants() { return kTnPlVariants; }
int conv_tn_pl_variant() { return g_tn_pl_variant; }
void conv_tn_pl_set_variant(int v) { g_tn_pl_variant = v; }

bool conv_tn_pl_supported(const ConvTNParams& p) {
  return p.dy_lo != 0 && p.x_lo != 0 && p.C % 8 == 0 && p.Co % 8 == 0 && p.ldy == p.Co && p.ldx == p.C;
}

static int resolve_tn_pl(int variant, int K, int Co, int R) {
  if (variant < 0 || variant >= kTnPlVariants) variant = tn_pl_default_variant(K, Co, R);
  return variant;
}

int conv_tn_pl_splitk(int K, int Co, int R, int M, int variant) {
  int splitk, mps;
  tn_pl_split(K, Co, R, M, resolve_tn_pl(variant, K, Co, R), splitk, mps);
  return splitk;
}

void tn_fold(const float* part, float* dw, long dw_cs, int K, int splitk, long CoR, hipStream_t s, const SgdEpi* sgd) {
  const long n = (CoR + 3) / 4;
  const int gx = (int)std::min<long>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(tn_fold_kernel, dim3(gx, K), dim3(256), 0, s, part, dw, dw_cs, K, splitk, CoR,
                     sgd ? *sgd : SgdEpi{});
}

bool conv_tn_pl(ConvTNParams p, int K, int variant, hipStream_t s) {
  if (!conv_tn_pl_supported(p)) return false;
  const long ab = (p.dy_lo + (long)p.M * p.ldy) * 2, bb = (p.x_lo + (long)p.B * p.H * p.W * p.ldx) * 2;
  if (ab >= (long)OOB_OFF || bb >= (long)OOB_OFF) return false;
  variant = resolve_tn_pl(variant < 0 ? g_tn_pl_variant : variant, K, p.Co, p.R);
  tn_pl_split(K, p.Co, p.R, p.M, variant, p.splitk, p.m_per_split);
  if (p.splitk > 1 && p.part == nullptr) return false;  // (the caller sizes the slabs)
  const TnPlTile t = kTnPlTiles[variant];
  const int grid = (int)((long)K * cdiv(p.Co, t.bm) * cdiv(p.R, t.bn) * p.splitk);
  // (the SGD epilogue instantiation where the kernel itself stores: no split-K slabs)
  const bool sgd = p.sgd.theta != nullptr && p.splitk == 1;
  // the pixel walk (PIX) on small images, the 128x128 and 256x256 tiles: l4 / l4a / l3a wgrad 1.31 /
  // 1.13 / 1.06x at 50 clients, l4 1.08x at 7 (bench/pix_bench.py, profiles/r6_c10_pix_bench.log)
  p.pix = native_option(g_opt_conv_pix, "DLS_CONV_PIX", 1) != 0 && (variant == 0 || variant == 6) &&
          p.C % t.bn == 0 && p.OH * p.OW <= 64 && p.KH * p.KW > 1 && p.pad > 0 && p.R == p.KH * p.KW * p.C &&
          p.M == p.B * p.OH * p.OW;
#define TN_PL_LAUNCH_X(BM_, BN_, WM_, WN_, NST_, ILV_, NT_, PIX_)                                                 \
  if (sgd)                                                                                                 \
    hipLaunchKernelGGL((conv_tn_pl_kernel<BM_, BN_, WM_, WN_, NST_, ILV_, true, PIX_>), dim3(grid), dim3(NT_), 0, s, p); \
  else                                                                                                     \
    hipLaunchKernelGGL((conv_tn_pl_kernel<BM_, BN_, WM_, WN_, NST_, ILV_, false, PIX_>), dim3(grid), dim3(NT_), 0, s, p);
#define TN_PL_LAUNCH(BM_, BN_, WM_, WN_, NST_, ILV_, NT_) TN_PL_LAUNCH_X(BM_, BN_, WM_, WN_, NST_, ILV_, NT_, false)
  if (p.pix) {
    if (variant == 0) {
      TN_PL_LAUNCH_X(128, 128, 2, 2, 2, false, 256, true)
    } else {
      TN_PL_LAUNCH_X(256, 256, 2, 4, 2, false, 512, true)
    }
  } else switch (variant) {
    case 0: TN_PL_LAUNCH(128, 128, 2, 2, 2, false, 256) break;
    case 1: TN_PL_LAUNCH(64, 128, 2, 2, 2, false, 256) break;
    case 2: TN_PL_LAUNCH(128, 128, 2, 2, 3, true, 256) break;
    case 3: TN_PL_LAUNCH(64, 128, 2, 2, 3, true, 256) break;
    case 4: TN_PL_LAUNCH(256, 128, 4, 2, 2, false, 512) break;
    case 5: TN_PL_LAUNCH(128, 256, 2, 4, 2, false, 512) break;
    case 6: TN_PL_LAUNCH(256, 256, 2, 4, 2, false, 512) break;
    default: return false;
  }
#undef TN_PL_LAUNCH
#undef TN_PL_LAUNCH_X
  if (p.splitk > 1) tn_fold(p.part, p.dw, p.dw_cs, K, p.splitk, (long)p.Co * p.R, s, &p.sgd);
  return true;
}
