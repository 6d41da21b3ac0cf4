// 3x3 / stride-1 / pad-1 weight gradient with LDS halo reuse (gfx950, MI355X): the ResNet
// layer-1..3 convolutions (64-256 channels, 32² / 16² / 8² images).
//
// dW[n][tap][c] = Σ_p dY[p][n] · X[p + tap][c] per client. The implicit-GEMM TN kernel
// (conv_pl.hip) makes the 9·C im2col columns its GEMM N dimension: every input pixel is gathered
// from L2 nine times, and at 32² the gathers spill out of the XCD's L2 — the layer-1 weight
// gradient read 2.5x its operand bytes from HBM (PMC TCC_EA0_RDREQ, r4_c16 summary) and ran
// HBM-bound at 44 % MFMA-busy. Here a workgroup owns one client, one 64 x 64 (n, c) block and a
// strided set of pixel tiles (IMG images × TH rows × the full width TW):
//   * per tile the X halo (IMG·(TH+2)·(TW+2) pixels × 64 channels) and the dY tile (TP pixels × 64
//     channels) are loaded ONCE, split to bf16 hi / lo planes while staged (or copied as planes),
//     into LDS — HBM reads ≈ dY + (1 + halo) · X;
//   * twelve waves: wave (kh, n-half, c-half) runs the three taps (kh, 0..2) of one 32 x 32
//     output block on v_mfma_f32_32x32x16_bf16 with the pixel as the reduction index; its dYᵀ
//     fragment is shared by the three taps, and both operands are read k-major with the
//     transposed LDS read (ds_read_b64_tr_b16);
//   * products are bf16x3 like every fp32 GEMM here (al·bh + ah·bl + ah·bh, fp32 accumulate);
//   * the next tile's global loads are issued into registers before the current tile's MFMAs.
// X modes: bf16 planes (the producing BatchNorm wrote them), fp32, or fp32 with the BatchNorm
// (+ReLU) applied while staging — relu(scale·x + shift), zero outside the image and past the
// client's valid rows: the exact operand bits of bn_apply's planes, from the RAW conv output, so
// training never has to store the normalised activation for this weight gradient.
// Each workgroup writes its 64 x 9 x 64 partial to its own slab; a fold sums a (client, block)'s
// G slabs in slab order — no atomics, bitwise reproducible, and G depends on the per-client shape
// only (so N ranks give the bits of one). G = 1 writes dW directly.
// LDS rows are 128 B (64 bf16); the 64-B half of a row a 16-lane group's transposed read lands in
// is flipped by bit 1 of the row, so the four consecutive rows one LDS cycle reads hit 4 disjoint
// 64-B bank windows at any starting row (tap shifts move the start by 0..2).
#include "dls.h"
#include "sgd_epi.h"
#include "gemm_common.h"

namespace {

__device__ __forceinline__ uint32_t wh_off(int row, int slot) {
  return (uint32_t)(row * 128 + ((slot ^ (((row >> 1) & 1) << 2)) << 4));
}

constexpr int kSlab = 64 * 9 * 64;  // floats of one workgroup's partial dW block

// XM: 0 X as bf16 planes, 1 fp32, 2 fp32 + BatchNorm(+ReLU) in the loader; DM: 0 dY planes, 1 fp32,
// 2 the BatchNorm backward of an fp32 output gradient applied in the loader (HaloWgradParams bb_*):
// the consumer of a BN's input gradient stages it from (dy, x, ReLU bits) itself, and writes its
// split planes for the dgrad on the way — no separate BN-backward apply pass over HBM.
// Tiles of TH rows × TW columns of one image (TW ≤ W: a 32-wide image is two column tiles).
// LDS holds two tiles (X halo + dY, hi and lo planes each): tile t + 1 is written from registers
// into the other buffer halfway through tile t's MFMAs, and tile t + 2's global loads are issued
// right after — one barrier per tile, the staging spread over the compute instead of a phase of
// its own, and only one tile's loads (≈ 40 KB per workgroup) held in registers.
template <int TH, int TW, int XM, int DM, int U>
__global__ void __launch_bounds__(768, 1) halo_wgrad_kernel(HaloWgradParams p) {
  constexpr int NT = 768;
  constexpr int HW2 = TW + 2, HH2 = TH + 2;
  constexpr int TP = TH * TW, HP = HH2 * HW2;
  constexpr int X_PL = HP * 128, D_PL = TP * 128;
  constexpr int BUF = 2 * X_PL + 2 * D_PL;
  constexpr int XT = (HP * 8 + NT - 1) / NT, DT = (TP * 8 + NT - 1) / NT;
  constexpr int KS = TP / 16;
  static_assert(TP % 16 == 0 && TW % 8 == 0 && XT <= 32 && KS >= 2, "tile");
  constexpr int COEF = XM == 2 ? 512 : 0, DCOEF = DM == 2 ? 768 : 0;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF + COEF + DCOEF];
  float* const coef_s = reinterpret_cast<float*>(smem + 2 * BUF);
  float* const dcoef_s = reinterpret_cast<float*>(smem + 2 * BUF + COEF);  // (DM 2) (a, d, e) × 64

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbc = p.nblk * p.cblk;
  const int per_client = p.G * nbc;
  // consecutive remapped ids share an XCD: the (n, c) blocks of one (client, pixel group) read the
  // same tiles, so their re-reads hit that XCD's L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  const int rem = bid - client * per_client;
  const int g = rem / nbc, nc = rem - g * nbc;
  const int nb = nc / p.cblk, cb = nc - nb * p.cblk;
  const int n0 = nb * 64, c0 = cb * 64;
  const int tcols = p.W / TW;
  const int tpi = (p.H / TH) * tcols;  // tiles per image
  // (tiles of images past the client's valid samples hold zero dY and X: skipped)
  const int tiles = p.valid_img ? min(p.B, max(p.valid_img[client], 0)) * tpi : p.B * tpi;

  const long npix = (long)p.B * p.H * p.W;
  const auto xr = make_rsrc(reinterpret_cast<const unsigned char*>(p.x) + client * p.x_cs * (XM == 0 ? 2 : 4),
                            (uint32_t)(XM == 0 ? (p.x_lo + npix * p.ldx) * 2 : npix * p.ldx * 4));
  const auto dr = make_rsrc(reinterpret_cast<const unsigned char*>(p.dy) + client * p.dy_cs * (DM == 0 ? 2 : 4),
                            (uint32_t)(DM == 0 ? (p.dy_lo + npix * p.ldy) * 2 : npix * p.ldy * 4));
  // (DM 2) the BN's raw input rows share dy's layout; its ReLU bits: one byte per 8 channels
  const auto br = make_rsrc(DM == 2 ? reinterpret_cast<const unsigned char*>(p.bb_x) + client * p.dy_cs * 4
                                    : reinterpret_cast<const unsigned char*>(p.dy),
                            (uint32_t)(DM == 2 ? npix * p.ldy * 4 : 0));
  const uint8_t* const bmk = DM == 2 && p.bb_mask ? p.bb_mask + client * npix * (p.N >> 3) + (n0 >> 3) : nullptr;
  const int brows = DM == 2 ? (p.bb_valid ? p.bb_valid[client] : (int)npix) : 0;
  bf16_t* const bdx = DM == 2 && p.bb_dxp && cb == 0 ? p.bb_dxp + client * 2 * npix * p.N + n0 : nullptr;
  const uint32_t x_lo = (uint32_t)(p.x_lo * 2), d_lo = (uint32_t)(p.dy_lo * 2);
  const int xrows = XM == 2 ? (p.x_valid ? p.x_valid[client] : (int)npix) : 0;
  if constexpr (XM == 2) {
    if (tid < 128) coef_s[tid] = p.coef[((long)client * p.C + c0) * 2 + tid];
  }
  if constexpr (DM == 2) {
    if (tid < 192) dcoef_s[tid] = p.bb_coef[((long)client * p.N + n0) * 3 + tid];
  }
  if constexpr (XM == 2 || DM == 2) __syncthreads();

  // ---- global → registers (one tile), registers → the LDS planes of a buffer
  u32x4_t xa[XT], xb[XT], da[DT], db[DT];
  uint32_t xok = 0;  // (XM 2) staged halo row inside the image and a valid sample
  // (DM 2) the BN's raw input, the task's ReLU byte (bit 8: a valid row) and pixel
  u32x4_t ba[DM == 2 ? DT : 1], bb[DM == 2 ? DT : 1];
  uint32_t bm[DM == 2 ? DT : 1];
  int bpix[DM == 2 ? DT : 1];
  auto load_tile = [&](int t) {
    const int b = t / tpi, r = t - b * tpi;
    const int h0 = (r / tcols) * TH, w0 = (r - (r / tcols) * tcols) * TW;
    xok = 0;
#pragma unroll
    for (int i = 0; i < XT; ++i) {
      const int task = tid + i * NT;
      const int hr = task >> 3, slot = task & 7;
      const int hh = hr / HW2, ww = hr - hh * HW2;
      const int ih = h0 - 1 + hh, iw = w0 - 1 + ww;
      const bool ok = task < HP * 8 && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const int pix = (b * p.H + ih) * p.W + iw;
      if constexpr (XM == 2) xok |= (ok && pix < xrows ? 1u : 0u) << i;
      if constexpr (XM == 0) {
        const uint32_t off = (uint32_t)(pix * p.ldx + c0 + slot * 8) * 2u;
        xa[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? off : OOB_OFF, 0, 0);
        xb[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? off + x_lo : OOB_OFF, 0, 0);
      } else {
        const uint32_t off = (uint32_t)(pix * p.ldx + c0 + slot * 8) * 4u;
        xa[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? off : OOB_OFF, 0, 0);
        xb[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? off + 16 : OOB_OFF, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < DT; ++i) {
      const int task = tid + i * NT;
      const int pt = task >> 3, slot = task & 7;
      const int th = pt / TW, tw = pt - th * TW;
      const bool ok = task < TP * 8;
      const int pix = (b * p.H + h0 + th) * p.W + w0 + tw;
      if constexpr (DM == 0) {
        const uint32_t off = (uint32_t)(pix * p.ldy + n0 + slot * 8) * 2u;
        da[i] = __builtin_amdgcn_raw_buffer_load_b128(dr, ok ? off : OOB_OFF, 0, 0);
        db[i] = __builtin_amdgcn_raw_buffer_load_b128(dr, ok ? off + d_lo : OOB_OFF, 0, 0);
      } else {
        // (DM 2: rows past the BN's valid ones are zero whatever dy and x hold — not loaded)
        const bool okv = ok && (DM != 2 || pix < brows);
        const uint32_t off = (uint32_t)(pix * p.ldy + n0 + slot * 8) * 4u;
        da[i] = __builtin_amdgcn_raw_buffer_load_b128(dr, okv ? off : OOB_OFF, 0, 0);
        db[i] = __builtin_amdgcn_raw_buffer_load_b128(dr, okv ? off + 16 : OOB_OFF, 0, 0);
        if constexpr (DM == 2) {
          ba[i] = __builtin_amdgcn_raw_buffer_load_b128(br, okv ? off : OOB_OFF, 0, 0);
          bb[i] = __builtin_amdgcn_raw_buffer_load_b128(br, okv ? off + 16 : OOB_OFF, 0, 0);
          bm[i] = okv ? (bmk ? (uint32_t)bmk[(long)pix * (p.N >> 3) + slot] : 0xffu) | 0x100u : 0u;
          bpix[i] = pix;
        }
      }
    }
  };
  // fp32 values (channels 0-3, 4-7) → 16-B hi and lo slots
  auto split8 = [](const float* v, uint4& hi, uint4& lo) {
    split_pair(v[0], v[1], hi.x, lo.x);
    split_pair(v[2], v[3], hi.y, lo.y);
    split_pair(v[4], v[5], hi.z, lo.z);
    split_pair(v[6], v[7], hi.w, lo.w);
  };
  auto store_tile = [&](unsigned char* buf) {
    unsigned char* const Xs = buf;
    unsigned char* const Ds = buf + 2 * X_PL;
#pragma unroll
    for (int i = 0; i < XT; ++i) {
      const int task = tid + i * NT;
      if (task < HP * 8) {
        const int hr = task >> 3, slot = task & 7;
        uint4 hi, lo;
        if constexpr (XM == 0) {
          hi = make_uint4(xa[i].x, xa[i].y, xa[i].z, xa[i].w);
          lo = make_uint4(xb[i].x, xb[i].y, xb[i].z, xb[i].w);
        } else {
          float v[8] = {__uint_as_float(xa[i].x), __uint_as_float(xa[i].y), __uint_as_float(xa[i].z),
                        __uint_as_float(xa[i].w), __uint_as_float(xb[i].x), __uint_as_float(xb[i].y),
                        __uint_as_float(xb[i].z), __uint_as_float(xb[i].w)};
          if constexpr (XM == 2) {
            const float4* cf = reinterpret_cast<const float4*>(coef_s + slot * 16);  // (scale, shift) pairs
            const float4 c0v = cf[0], c1v = cf[1], c2v = cf[2], c3v = cf[3];
            const bool okv = (xok >> i) & 1u;
            v[0] = fmaf(v[0], c0v.x, c0v.y);
            v[1] = fmaf(v[1], c0v.z, c0v.w);
            v[2] = fmaf(v[2], c1v.x, c1v.y);
            v[3] = fmaf(v[3], c1v.z, c1v.w);
            v[4] = fmaf(v[4], c2v.x, c2v.y);
            v[5] = fmaf(v[5], c2v.z, c2v.w);
            v[6] = fmaf(v[6], c3v.x, c3v.y);
            v[7] = fmaf(v[7], c3v.z, c3v.w);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              if (p.relu) v[j] = fmaxf(v[j], 0.f);
              if (!okv) v[j] = 0.f;
            }
          }
          split8(v, hi, lo);
        }
        const uint32_t o = wh_off(hr, slot);
        *reinterpret_cast<uint4*>(Xs + o) = hi;
        *reinterpret_cast<uint4*>(Xs + X_PL + o) = lo;
      }
    }
#pragma unroll
    for (int i = 0; i < DT; ++i) {
      const int task = tid + i * NT;
      if (task < TP * 8) {
        const int pt = task >> 3, slot = task & 7;
        uint4 hi, lo;
        if constexpr (DM == 0) {
          hi = make_uint4(da[i].x, da[i].y, da[i].z, da[i].w);
          lo = make_uint4(db[i].x, db[i].y, db[i].z, db[i].w);
        } else {
          float v[8] = {__uint_as_float(da[i].x), __uint_as_float(da[i].y), __uint_as_float(da[i].z),
                        __uint_as_float(da[i].w), __uint_as_float(db[i].x), __uint_as_float(db[i].y),
                        __uint_as_float(db[i].z), __uint_as_float(db[i].w)};
          if constexpr (DM == 2) {
            const float xv[8] = {__uint_as_float(ba[i].x), __uint_as_float(ba[i].y), __uint_as_float(ba[i].z),
                                 __uint_as_float(ba[i].w), __uint_as_float(bb[i].x), __uint_as_float(bb[i].y),
                                 __uint_as_float(bb[i].z), __uint_as_float(bb[i].w)};
            const float* cf = dcoef_s + slot * 24;  // (a, d, e) of the slot's 8 channels
            const uint32_t m = bm[i];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float gd = ((m >> j) & 1u) ? v[j] : 0.f;
              v[j] = (m & 0x100u) ? fmaf(cf[3 * j], gd, fmaf(cf[3 * j + 2], xv[j], cf[3 * j + 1])) : 0.f;
            }
          }
          split8(v, hi, lo);
          if constexpr (DM == 2) {
            if (bdx) {  // (dY's planes for the dgrad: the hi / lo slots bn_bwd_apply would have stored)
              bf16_t* const hp = bdx + (long)bpix[i] * p.N + slot * 8;
              *reinterpret_cast<uint4*>(hp) = hi;
              *reinterpret_cast<uint4*>(hp + npix * p.N) = lo;
            }
          }
        }
        const uint32_t o = wh_off(pt, slot);
        *reinterpret_cast<uint4*>(Ds + o) = hi;
        *reinterpret_cast<uint4*>(Ds + D_PL + o) = lo;
      }
    }
  };

  // ---- MFMA operand addressing: wave (kh, n-half, c-half); lane 16·g4 + 4q + pp supplies pixel
  // row 16·ks + 8·hf + q (and + 4) of the transposed reads, channels 16·(g4 & 1) + 4·pp of its half
  const int kh = wid >> 2, nh = (wid >> 1) & 1, chh = wid & 1;
  const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, hf = lane >> 5;
  const int aslot = nh * 4 + 2 * (g4 & 1) + (pp >> 1), bslot = chh * 4 + 2 * (g4 & 1) + (pp >> 1);
  const int sb = (pp & 1) * 8;
  f32x16 acc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) acc[j] = f32x16{};
  auto kstep = [&](const unsigned char* buf, int ks) {
    const unsigned char* const Xs = buf;
    const unsigned char* const Ds = buf + 2 * X_PL;
    const int kq = 16 * ks + 8 * hf + q;  // (kq and kq + 4: one 8-aligned run of one tile row)
    const int th = kq / TW, tw = kq - th * TW;
    const int hr = (th + kh) * HW2 + tw;  // halo row of tap (kh, 0)
    const bf16_t* a1 = reinterpret_cast<const bf16_t*>(Ds + wh_off(kq, aslot) + sb);
    const bf16_t* a2 = reinterpret_cast<const bf16_t*>(Ds + wh_off(kq + 4, aslot) + sb);
    const bf16x8 ah = tr_frag(a1, a2);
    const bf16x8 al = tr_frag(a1 + D_PL / 2, a2 + D_PL / 2);
    bf16x8 bh[3], bl[3];
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const bf16_t* b1 = reinterpret_cast<const bf16_t*>(Xs + wh_off(hr + kw, bslot) + sb);
      const bf16_t* b2 = reinterpret_cast<const bf16_t*>(Xs + wh_off(hr + kw + 4, bslot) + sb);
      bh[kw] = tr_frag(b1, b2);
      bl[kw] = tr_frag(b1 + X_PL / 2, b2 + X_PL / 2);
    }
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[kw], acc[kw], 0, 0, 0);
      acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[kw], acc[kw], 0, 0, 0);
      acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[kw], acc[kw], 0, 0, 0);
    }
  };

  // a contiguous range of tiles per workgroup (consecutive tiles of one image: the halo rows and
  // columns shared with the previous tile come from L2, not HBM)
  const int t_beg = (int)((long)tiles * g / p.G), t_end = (int)((long)tiles * (g + 1) / p.G);
  if (t_beg < t_end) {
    load_tile(t_beg);
    store_tile(smem);
    if (t_beg + 1 < t_end) load_tile(t_beg + 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __syncthreads();
  }
  for (int t = t_beg; t < t_end; ++t) {
    unsigned char* const cur = smem + ((t - t_beg) & 1) * BUF;
    unsigned char* const nxt = smem + (((t - t_beg) & 1) ^ 1) * BUF;
#pragma unroll U
    for (int ks = 0; ks < KS / 2; ++ks) kstep(cur, ks);
    // (the other buffer's last readers passed the previous tile's closing barrier)
    if (t + 1 < t_end) {
      store_tile(nxt);
      if (t + 2 < t_end) load_tile(t + 2);
    }
#pragma unroll U
    for (int ks = KS / 2; ks < KS; ++ks) kstep(cur, ks);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS stores landed
    __syncthreads();
  }

  if constexpr (DM == 2) {
    // (the images past the valid samples were skipped: their dY planes are zeros, as the BN
    // backward writes there; the pixel groups split those tiles like the valid ones)
    const int all = p.B * tpi;
    if (bdx && tiles < all) {
      const int z_beg = tiles + (int)((long)(all - tiles) * g / p.G), z_end = tiles + (int)((long)(all - tiles) * (g + 1) / p.G);
      for (int task = tid; task < (z_end - z_beg) * TP * 8; task += NT) {
        const int t = z_beg + task / (TP * 8), r = task - (task / (TP * 8)) * (TP * 8);
        const int b = t / tpi, rt = t - b * tpi;
        const int h0 = (rt / tcols) * TH, w0 = (rt - (rt / tcols) * tcols) * TW;
        const int pt = r >> 3, slot = r & 7;
        const int th = pt / TW, tw = pt - th * TW;
        bf16_t* const hp = bdx + (long)((b * p.H + h0 + th) * p.W + w0 + tw) * p.N + slot * 8;
        *reinterpret_cast<uint4*>(hp) = make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(hp + npix * p.N) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }

  // ---- this wave's three 32 x 32 blocks: lane holds rows n = (e & 3) + 8(e >> 2) + 4·hf, column
  // c = lane & 31 of each. G = 1: straight into dW, else into the workgroup's slab [64 n][9][64 c]
  const int cc = chh * 32 + (lane & 31);
  if (p.G == 1 && p.sgd.theta) {  // the optimiser step in place of the dW store (SgdEpi)
    if (p.sgd.active[client]) {
      // (each wave's 32 x 32 blocks through its own LDS slab: the main loop's last barrier retired
      // every read of the tile buffers)
      float* sl = reinterpret_cast<float*>(smem) + wid * 32 * 36;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)  // (rows n of dW [n][tap][c]: stride 9·C)
        sgd_epi_tile32(p.sgd, client, sl, acc[kw], ((long)(n0 + nh * 32) * 9 + kh * 3 + kw) * p.C + c0 + chh * 32,
                       9L * p.C, 32, 32);
    }
  } else if (p.G == 1) {
    float* dw = p.dw + (long)client * p.dw_cs;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int nn = nh * 32 + (e & 3) + 8 * (e >> 2) + 4 * hf;
        dw[((long)(n0 + nn) * 9 + kh * 3 + kw) * p.C + c0 + cc] = acc[kw][e];
      }
  } else {
    float* slab = p.part + ((((long)client * p.nblk + nb) * p.cblk + cb) * p.G + g) * kSlab;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int nn = nh * 32 + (e & 3) + 8 * (e >> 2) + 4 * hf;
        slab[(nn * 9 + kh * 3 + kw) * 64 + cc] = acc[kw][e];
      }
  }
}

// dW[k][n][tap][c] = Σ_g slab[k][n / 64][c / 64][g][n % 64][tap][c % 64], g in order; 4 columns
// per thread (C % 64 == 0)
__global__ void __launch_bounds__(256) halo_wgrad_fold_kernel(HaloWgradParams p) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long per4 = (long)p.N * 9 * p.C / 4;
  if (idx >= per4 * p.K) return;
  const int k = (int)(idx / per4);
  const long r = (idx - (long)k * per4) * 4;
  const int n = (int)(r / (9 * p.C));
  const int r2 = (int)(r - (long)n * 9 * p.C);
  const int tap = r2 / p.C, c = r2 - tap * p.C;
  const float* src = p.part + ((((long)k * p.nblk + n / 64) * p.cblk + c / 64) * p.G) * kSlab +
                     ((n & 63) * 9 + tap) * 64 + (c & 63);
  float4 s = *reinterpret_cast<const float4*>(src);
  for (int gg = 1; gg < p.G; ++gg) {
    const float4 v = *reinterpret_cast<const float4*>(src + (long)gg * kSlab);
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  if (p.sgd.theta) {
    if (p.sgd.active[k]) sgd_epi4(p.sgd, k, r, s);
  } else {
    *reinterpret_cast<float4*>(p.dw + (long)k * p.dw_cs + r) = s;
  }
}

// tile shapes: TH rows × TW columns of one image, two LDS buffers of (halo + dY) hi / lo planes
// (32² and 16²: 8 × 16, 157.7 KB; 8²: 8 × 8); 64 x 64 (n, c) blocks
int halo_wgrad_cfg(int B, int H, int W, int C, int N) {
  if (C % 64 || N % 64 || C > 512 || N > 512 || B < 1) return -1;
  if (W % 16 == 0 && H % 8 == 0 && W <= 64) return 0;  // 8 × 16 tiles
  if (W == 8 && H == 8) return 1;                       // 8 × 8
  return -1;
}

int halo_wgrad_tiles(int cfg, int B, int H, int W) { return cfg == 0 ? B * (H / 8) * (W / 16) : B; }

// pixel groups per (client, block): about 16 workgroups per client, whatever the block count
int halo_wgrad_G(int cfg, int B, int H, int W, int C, int N) {
  const int nbc = (C / 64) * (N / 64);
  int G = 16 / nbc;
  if (G < 1) G = 1;
  const int tiles = halo_wgrad_tiles(cfg, B, H, W);
  return G < tiles ? G : tiles;
}

}  // namespace

bool halo_wgrad_supported(int B, int H, int W, int C, int N) { return halo_wgrad_cfg(B, H, W, C, N) >= 0; }

long halo_wgrad_part_floats(int K, int B, int H, int W, int C, int N) {
  const int cfg = halo_wgrad_cfg(B, H, W, C, N);
  if (cfg < 0) return 0;
  const int G = halo_wgrad_G(cfg, B, H, W, C, N);
  return G > 1 ? (long)K * (C / 64) * (N / 64) * G * kSlab : 0;
}

bool halo_wgrad(HaloWgradParams p, int xm, int dm, hipStream_t s) {
  const int cfg = halo_wgrad_cfg(p.B, p.H, p.W, p.C, p.N);
  if (cfg < 0 || xm < 0 || xm > 2 || dm < 0 || dm > 2) return false;
  if (p.ldx % 8 || p.ldy % 8 || (xm == 2 && p.coef == nullptr)) return false;
  if (dm == 2 && (p.bb_x == nullptr || p.bb_coef == nullptr || p.ldy != p.N)) return false;
  if (((uintptr_t)p.dw & 15) || p.dw_cs % 4) return false;  // (the fold's 16-B stores)
  if (p.sgd.theta && (((uintptr_t)p.sgd.theta & 15) || ((uintptr_t)p.sgd.split & 7) || p.sgd.th_cs % 4 ||
                      p.sgd.sp_cs % 4 || p.sgd.sp_lo % 4 || (p.sgd.momentum != 0.f && ((uintptr_t)p.sgd.mom & 15))))
    return false;  // (the fold's float4 step)
  const long npix = (long)p.B * p.H * p.W;
  const long xb = xm == 0 ? (p.x_lo + npix * p.ldx) * 2 : npix * p.ldx * 4;
  const long db = dm == 0 ? (p.dy_lo + npix * p.ldy) * 2 : npix * p.ldy * 4;
  if (dm == 2 && npix * p.N * 2 * 2 >= (1L << 31)) return false;  // (bb_dxp: 32-bit element offsets)
  if (xb >= (long)OOB_OFF || db >= (long)OOB_OFF) return false;
  p.nblk = p.N / 64;
  p.cblk = p.C / 64;
  p.G = halo_wgrad_G(cfg, p.B, p.H, p.W, p.C, p.N);
  if (p.G > 1 && p.part == nullptr) return false;
  const int grid = p.K * p.G * p.nblk * p.cblk;
#define HW_LAUNCH_XD(TH, TW, U, XM, DM) \
  hipLaunchKernelGGL((halo_wgrad_kernel<TH, TW, XM, DM, U>), dim3(grid), dim3(768), 0, s, p)
#define HW_LAUNCH1(TH, TW, U)                               \
  switch (xm * 3 + dm) {                                        \
    case 0: HW_LAUNCH_XD(TH, TW, U, 0, 0); break;          \
    case 1: HW_LAUNCH_XD(TH, TW, U, 0, 1); break;          \
    case 2: HW_LAUNCH_XD(TH, TW, U, 0, 2); break;          \
    case 3: HW_LAUNCH_XD(TH, TW, U, 1, 0); break;          \
    case 4: HW_LAUNCH_XD(TH, TW, U, 1, 1); break;          \
    case 5: HW_LAUNCH_XD(TH, TW, U, 1, 2); break;          \
    case 6: HW_LAUNCH_XD(TH, TW, U, 2, 0); break;          \
    case 7: HW_LAUNCH_XD(TH, TW, U, 2, 1); break;          \
    default: HW_LAUNCH_XD(TH, TW, U, 2, 2); break;         \
  }
#define HW_LAUNCH(TH, TW) \
  if (unroll == 2) {          \
    HW_LAUNCH1(TH, TW, 2) \
  } else {                    \
    HW_LAUNCH1(TH, TW, 1) \
  }
  // (k-step unroll: 2 lets the compiler fetch the next step's fragments under this step's MFMAs)
  const int unroll = native_option(g_opt_halo_wgrad_unroll, "DLS_HALO_WGRAD_UNROLL", 1);
  if (cfg == 0) {
    HW_LAUNCH(8, 16)
  } else {
    HW_LAUNCH(8, 8)
  }
#undef HW_LAUNCH
#undef HW_LAUNCH1
#undef HW_LAUNCH_XD
  if (p.G > 1) {
    const long total4 = (long)p.K * p.N * 9 * p.C / 4;
    hipLaunchKernelGGL(halo_wgrad_fold_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, p);
  }
  return true;
}
