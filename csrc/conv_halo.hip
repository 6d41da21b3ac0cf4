// 3x3 / stride-1 / pad-1 fp32-accurate convolution on pre-split operands with LDS halo reuse
// (gfx950, MI355X).
//
// The implicit-GEMM kernels (conv_pl.hip) stage a fresh A tile for every (tap, channel chunk):
// each input pixel crosses the L2 → LDS path up to 9 times per output-channel tile, and that
// path (≈60 GB/s per CU for LDS-DMA gathers) is what bounds them. Here a workgroup owns a block
// of whole output rows — IMG images × TH rows × the full width TW, BM = IMG·TH·TW GEMM rows —
// and per 32-channel chunk DMAs the block's input HALO once ((TH+2)·(TW+2) pixels per image,
// zeros outside the image) into LDS; the nine taps then read their A fragments from that halo
// at a uniform row shift (dh·(TW+2) + dw). Only the weight tile is staged per tap. A-side bytes
// per chunk drop from 9·BM rows to IMG·(TH+2)·(TW+2) rows: 2.6–8.5× fewer for ResNet-18's
// 32², 16², 8², 4² layers.
//
// Arithmetic, split planes and product order are those of conv_pl.hip (bf16x3 on
// v_mfma_f32_32x32x16_bf16), so outputs are bit-identical to it, and it serves
//   forward : B = W[n][kh][kw][c] row-major;
//   dgrad   : stride-1 full correlation of dY with the flipped kernel, B read k-major in place
//             (ConvNTParams kh_off / kh_step mapping).
// Pipeline (per wave, all in one __shared__ array): halo double-buffered — chunk c+1's halo is
// issued at chunk c's first tap step; weight tiles in a 3-slot ring, tile s+2 issued at step s.
// Counted vmcnt before each step's barrier: the step's weight tile and its chunk's halo are
// older than everything left in flight (see the wait comments in the loop).
#include "dls.h"
#include "epilogue_f32.h"
#include "gemm_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void hdma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void hwait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// HB: halo buffers (2: chunk c+1's halo in flight during chunk c; 1: loaded at the chunk start
// behind a barrier — half the LDS, so two workgroups share a CU); NBS: weight-tile slots (3 or 2)
// BNF: the A operand is BatchNorm(+ReLU) of the raw fp32 input, applied while the halo is staged
// (ConvNTParams::bn_x): each lane loads its 8 channels of a halo row into registers, applies the
// per-channel (scale, shift) and ReLU, splits to hi / lo and writes the same 16-B LDS slots the
// plane DMA would fill — bit-identical operands to BN-apply-then-planes, without the normalised
// tensor ever reaching HBM. Forward (row-major B) with one halo buffer only.
// BNM: 0 plain; 1 fused BN (ResNet block: bn_x contiguous [.., C], training writes split planes +
// ReLU bits); 2 fused BN over a DenseNet channel prefix (bn_x rows at stride ldx inside the block
// buffer, bn_c ≤ C real channels — the rest of the 32-channel chunk stages as zero — training
// writes the normalised activation in fp32 at row stride bn_ldy)
// TPS (one halo buffer only): taps per pipeline step — each weight slot holds TPS taps' tiles,
// so a barrier covers TPS taps' MFMAs (the 64-channel l1 shape has only 12 MFMAs per wave per tap)
template <int IMG, int TH, int TW, int BN, int WM, int WN, bool BKM, int MINW, int HB, int NBS, int BNM = 0,
          int TPS = 1>
__global__ void __launch_bounds__(WM* WN * 64) __attribute__((amdgpu_waves_per_eu(MINW * WM * WN / 4)))
conv_halo_kernel(ConvNTParams p) {
  constexpr bool BNF = BNM != 0, DENSE = BNM == 2;
  static_assert((HB == 2 && NBS == 3) || (HB == 1 && (NBS == 2 || NBS == 3)), "pipeline shape");
  static_assert(TPS == 1 || (HB == 1 && TPS == 2 && NBS == 2), "taps per step");
  constexpr int SPC = (9 + TPS - 1) / TPS;  // pipeline steps per 32-channel chunk
  static_assert(!BNF || (HB == 1 && !BKM), "fused BN input: forward, one halo buffer");
  constexpr int BM = IMG * TH * TW;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(TM >= 1 && TN >= 1 && TM * WM * 32 == BM, "wave tile");
  constexpr int HW2 = TW + 2, HH2 = TH + 2;
  // LDS row pitch of one halo image row, and the chunk-swizzle key of halo row hr:
  //   key(hr) = ((hr >> 2) + (hr / PITCH) * KC) & 3
  // The A fragment rows of a tap are TW-pixel runs of consecutive halo rows that jump by
  // PITCH - TW at each image row. With the plain key ((hr >> 2) & 3) and pitch TW + 2, the 16
  // rows one ds_read_b128 lane group reads collide on banks for TW = 16 / 8 (PMC: 33-40 % of
  // LDS cycles were conflicts). Pitch TW + 4 with KC = 3 makes every group of every tap shift
  // conflict-free (searched exhaustively over the 9 taps and both lane groups); TW = 32 already
  // is with the plain key. The pad columns are never loaded (DMA offset out of window).
  constexpr int PITCH = TW == 32 ? HW2 : TW + 4, KC = TW == 32 ? 0 : 3;
  constexpr int HP = IMG * HH2 * PITCH;            // halo rows of the A image (pads included)
  constexpr int HI = (HP + 16 * NW - 1) / (16 * NW);  // halo DMA instructions per wave per plane
  constexpr int H_PL = HI * 16 * NW * 64;          // bytes per halo plane (64-B rows)
  constexpr int B_PL = BN * 64;                    // bytes per weight plane ([BN][32] or [32][BN])
  constexpr int NBI = BN / 16;                     // 1-KiB weight DMA instructions per plane
  constexpr int BI = (NBI + NW - 1) / NW;          // per wave (the surplus ones go to a scratch KiB)
  constexpr int GH = 2 * HI, GB = 2 * BI;          // DMA instructions per wave: halo / weight tile
  constexpr int H_OFF = 0, B_OFF = HB * 2 * H_PL;  // halo buffers (hi, lo each), then the weight slots
  constexpr int SCR = B_OFF + NBS * TPS * 2 * B_PL;  // scratch KiB of the surplus weight DMAs
  // (TPS > 1: every step waits for all its DMAs (NBS 2), so the surplus waves issue no weight DMAs
  // instead of keeping their counts uniform through the scratch KiB — which would not fit two
  // workgroups per CU)
  constexpr int LOOP = SCR + (BI * NW > NBI && TPS == 1 ? 1024 : 0);
  constexpr int SW = TN * 32 + 4;
  constexpr int EPI = NW * 32 * SW * 4;
  // (BNF) channels whose (scale, shift) pairs sit in LDS, copied once per workgroup so the loader
  // reads them without ordering against its output stores — sized where two workgroups still fit
  // per CU (0: read from global memory; halo_config keeps C within it)
  constexpr int COEF_C =
      !BNF ? 0 : DENSE ? (TW == 8 ? 0 : 512) : (TW == 32 && TPS == 1 ? 128 : TW == 8 ? 256 : 0);
  constexpr int SMEM = LOOP + COEF_C * 8 > EPI ? LOOP + COEF_C * 8 : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tpi = p.OH / TH;  // row blocks per image (IMG == 1), 1 otherwise
  const int tilesM = IMG == 1 ? p.B * tpi : p.B / IMG, tilesN = (p.N + BN - 1) / BN;
  const int per_client = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  const int t = bid - client * per_client;
  const int tm = t / tilesN, n0 = (t % tilesN) * BN;
  const int b0 = IMG == 1 ? tm / tpi : tm * IMG;
  const int h0 = IMG == 1 ? (tm % tpi) * TH : 0;
  const int m0 = tm * BM;
  if (!DENSE && p.skip_valid && m0 >= p.skip_valid[client] * p.skip_mul) {
    // a row block of samples past the client's valid ones (an epoch's last, partial batch): its
    // readers stop at the valid rows, so only the epilogue's partial sums must exist (as zeros)
    const int parts = (p.M + 31) / 32;
    for (int i = threadIdx.x; i < (BM / 32) * BN; i += NW * 64) {
      const int g = m0 / 32 + i / BN, n = n0 + i % BN;
      if (g < parts && n < p.N) {
        const long o = ((long)client * parts + g) * 2 * p.N + n;
        if (p.stats) {
          p.stats[o] = 0.f;
          p.stats[o + p.N] = 0.f;
        }
        if (p.bnb) {
          p.bnb[o] = 0.f;
          p.bnb[o + p.N] = 0.f;
        }
      }
    }
    return;
  }

  const long a_img = (long)p.B * p.H * p.W * p.ldx;
  const auto ar = make_rsrc(p.x + (long)client * p.x_cs, (uint32_t)((p.x_lo + a_img) * 2));
  const uint32_t a_lo = (uint32_t)(p.x_lo * 2);
  const long w_ext = BKM ? (long)p.C * p.wKH * p.wKW * p.N : (long)p.N * p.R;
  const auto br = make_rsrc(p.wsplit + (long)(client / p.rep) * p.ws_cs, (uint32_t)((p.ws_plane + w_ext) * 2));
  const uint32_t b_lo = (uint32_t)(p.ws_plane * 2);

  // ---- halo loader: instruction i of wave w fills halo rows (i·NW + w)·16 + lane/4, physical
  // chunk lane & 3 ← logical chunk lc = (lane & 3) ^ key(row)
  int h_off[HI], h_ch[HI];  // (h_ch: BNF, the lane's first channel within a 32-channel chunk)
  // (BNF) rows of samples past the BN's valid rows read as zero, like the padding; h_ctr: the halo
  // row is one of this row block's own output pixels (written out when bn_yp is set)
  bool h_bnok[HI], h_ctr[HI];
  int h_pix[DENSE ? HI : 1];  // (DENSE: the halo row's pixel index, for the fp32 activation rows)
  const int bn_rows = BNF ? (p.bn_valid ? p.bn_valid[client] : p.B * p.H * p.W) : 0;
#pragma unroll
  for (int i = 0; i < HI; ++i) {
    const int hr = (i * NW + wid) * 16 + (lane >> 2);
    const int img = hr / (HH2 * PITCH), rem = hr - img * (HH2 * PITCH);
    const int hh = rem / PITCH, ww = rem - hh * PITCH;
    const int ih = h0 - p.pad + hh, iw = ww - p.pad_w;
    const int lc = (lane & 3) ^ (((hr >> 2) + (hr / PITCH) * KC) & 3);
    const int pix = ((b0 + img) * p.H + ih) * p.W + iw;
    const bool ok = hr < HP && ww < HW2 && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    h_off[i] = ok ? pix * p.ldx + lc * 8 : -1;
    h_ch[i] = lc * 8;
    h_bnok[i] = !BNF || pix < bn_rows;
    h_ctr[i] = ok && hh >= 1 && hh <= TH && ww >= 1 && ww <= TW;
    if constexpr (DENSE) h_pix[i] = pix;
  }
  // ---- weight loader (as conv_pl.hip): row-major rows (i·NW + w)·16 + lane/4; k-major k-rows
  // (i·NW + w)·RPI + lane/CPR with the 32-element segment swizzle of the k-major image
  constexpr int CPR = BN / 8, RPI = 64 / CPR;
  constexpr int SD = (128 / BN) > 1 ? 128 / BN : 1, SS = (BN / 32) < 4 ? BN / 32 : 4;
  const long wkhwn = (long)p.wKH * p.wKW * p.N;
  const int wlc = (lane & 3) ^ ((lane >> 4) & 3);  // row-major weight rows: key (row >> 2) & 3
  int b_off[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    if constexpr (!BKM) {
      const int n = n0 + (i * NW + wid) * 16 + (lane >> 2);
      b_off[i] = n < p.N ? n * p.R + wlc * 8 : -1;
    } else {
      const int kr = (i * NW + wid) * RPI + lane / CPR;
      const int f = SS > 1 ? (kr / SD) & (SS - 1) : 0;
      const int n = n0 + ((lane % CPR) ^ (f << 2)) * 8;
      b_off[i] = n < p.N ? (int)(kr * wkhwn) + n : -1;
    }
    if (i * NW + wid >= NBI) b_off[i] = -1;
  }

  const int nchunks = p.C / 32, nsteps = nchunks * SPC;
  const float* bxc = BNF ? p.bn_x + (long)client * p.bn_x_cs : nullptr;
  const float* bcoef = BNF ? p.bn_coef + (long)client * p.C * 2 : nullptr;
  const long bn_rc = (long)p.B * p.H * p.W * p.C;  // (elements of one plane of one client)
  bf16_t* bn_yph = (BNF && p.bn_yp && n0 == 0) ? p.bn_yp + (long)client * 2 * bn_rc : nullptr;
  uint8_t* bn_mk = (BNF && p.bn_mask && n0 == 0)
                      ? p.bn_mask + (long)client * ((DENSE ? (long)p.M * p.bn_ldy : bn_rc) >> 3)
                      : nullptr;
  float* bn_ny = (DENSE && p.bn_y && n0 == 0) ? p.bn_y + (long)client * p.bn_y_cs : nullptr;
  const int bn_creal = DENSE ? p.bn_c : p.C;
  float* coef_s = reinterpret_cast<float*>(smem + LOOP);
  auto issue_halo = [&](int c, int buf) {
    const bool live = c < nchunks;
    unsigned char* Hs = smem + H_OFF + buf * 2 * H_PL;
    if constexpr (BNF) {
      // the raw x of RG rows first, so their HBM round trips overlap (one wait per RG rows, not one
      // per row: the output stores of a row would otherwise order the next row's loads after
      // them), then per row: (scale, shift), ReLU, split, LDS store (+ the outputs)
      // (RG 1 where the accumulators leave no VGPRs for it: TM·TN = 4 tiles, the l2 shape)
      constexpr int RG = TM * TN >= 4 ? 1 : (HI < 3 ? HI : 3);
#pragma unroll
      for (int i0 = 0; i0 < HI; i0 += RG) {
      float4 xa[RG], xb[RG];
#pragma unroll
      for (int i = i0; i < i0 + RG && i < HI; ++i) {
        const bool ok = live && h_off[i] >= 0;
        const int e = (ok ? h_off[i] : 0) + c * 32;  // lane's 8 channels: h_off = pixel·ldx + lc·8
        // (DENSE) real channels of the lane's 8: ≥ 8 all, 4 the first half (bn_c % 4 == 0), ≤ 0
        // none — channels past the prefix are other layers' (maybe unwritten) slots: never read
        const int cv = bn_creal - (c * 32 + h_ch[i]);
        xa[i - i0] = make_float4(0.f, 0.f, 0.f, 0.f);
        xb[i - i0] = xa[i - i0];
        if (!DENSE || cv > 0) xa[i - i0] = *reinterpret_cast<const float4*>(bxc + e);
        if (!DENSE || cv >= 8) xb[i - i0] = *reinterpret_cast<const float4*>(bxc + e + 4);
      }
#pragma unroll
      for (int i = i0; i < i0 + RG && i < HI; ++i) {
        const bool ok = live && h_off[i] >= 0;
        unsigned char* d = Hs + (i * NW + wid) * 1024;
        const bool inimg = ok;
        const bool okv = ok && h_bnok[i];
        const int e = (ok ? h_off[i] : 0) + c * 32;
        const int ch = c * 32 + h_ch[i];
        const int cv = bn_creal - ch;
        const float4 x0 = xa[i - i0], x1 = xb[i - i0];
        const float4* cf = reinterpret_cast<const float4*>((COEF_C ? coef_s : bcoef) + 2 * ch);  // (scale, shift)
        const float4 c0 = cf[0], c1 = cf[1], c2 = cf[2], c3 = cf[3];
        float v[8] = {fmaf(x0.x, c0.x, c0.y), fmaf(x0.y, c0.z, c0.w), fmaf(x0.z, c1.x, c1.y), fmaf(x0.w, c1.z, c1.w),
                      fmaf(x1.x, c2.x, c2.y), fmaf(x1.y, c2.z, c2.w), fmaf(x1.z, c3.x, c3.y), fmaf(x1.w, c3.z, c3.w)};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (p.bn_relu) v[j] = fmaxf(v[j], 0.f);
          if (!okv || (DENSE && cv <= (j < 4 ? 0 : 4))) v[j] = 0.f;
        }
        uint32_t hi[4], lo[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) split_pair(v[2 * j], v[2 * j + 1], hi[j], lo[j]);
        *reinterpret_cast<uint4*>(d + lane * 16) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
        *reinterpret_cast<uint4*>(d + H_PL + lane * 16) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
        // this row block's own pixels: planes (unless the weight gradient applies the BN itself,
        // conv_halo_wgrad.hip x mode 2) + ReLU bits out
        if (!DENSE && (bn_yph || bn_mk) && inimg && h_ctr[i]) {
          if (bn_yph) {
            *reinterpret_cast<uint4*>(bn_yph + e) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
            *reinterpret_cast<uint4*>(bn_yph + bn_rc + e) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
          }
          if (bn_mk) {
            uint32_t m = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) m |= (v[j] > 0.f ? 1u : 0u) << j;
            bn_mk[e >> 3] = (uint8_t)m;
          }
        }
        if constexpr (DENSE) {
          if (bn_ny && inimg && h_ctr[i] && cv > 0) {  // own pixels: the fp32 activation (bn_apply's bits)
            const long o = (long)h_pix[i] * p.bn_ldy + ch;
            *reinterpret_cast<float4*>(bn_ny + o) = make_float4(v[0], v[1], v[2], v[3]);
            if (cv >= 8) *reinterpret_cast<float4*>(bn_ny + o + 4) = make_float4(v[4], v[5], v[6], v[7]);
            if (bn_mk) {  // (bn_ldy % 8 == 0: whole bytes) the ReLU bits bn_apply would have written
              uint32_t m = 0;
#pragma unroll
              for (int j = 0; j < 8; ++j) m |= (v[j] > 0.f ? 1u : 0u) << j;
              bn_mk[o >> 3] = (uint8_t)m;
            }
          }
        }
      }
      }
      // (the LDS writes of a register-staged halo must land before the barrier that publishes it)
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    } else {
#pragma unroll
      for (int i = 0; i < HI; ++i) {
        const bool ok = live && h_off[i] >= 0;
        unsigned char* d = Hs + (i * NW + wid) * 1024;
        const uint32_t off = (uint32_t)(h_off[i] + c * 32) * 2u;
        hdma16(ar, d, ok ? off : OOB_OFF);
        hdma16(ar, d + H_PL, ok ? off + a_lo : OOB_OFF);
      }
    }
  };
  auto issue_w = [&](int s, int slot) {
    const int c = s / SPC, j = s - c * SPC;
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      const int tap = j * TPS + u;
      const bool live = s < nsteps && tap < 9;  // (a step past the chunk's last tap loads zeros)
      int boff;
      if constexpr (!BKM) {
        boff = tap * p.C + c * 32;
      } else {
        const int kh2 = tap / 3, kw2 = tap - kh2 * 3;
        const int khh = p.kh_off - p.kh_step * kh2, kww = p.kw_off - p.kw_step * kw2;
        boff = (int)(c * 32 * wkhwn) + (khh * p.wKW + kww) * p.N;
      }
      unsigned char* Bs = smem + B_OFF + (slot * TPS + u) * 2 * B_PL;
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        const bool ok = live && b_off[i] >= 0;
        const uint32_t off = (uint32_t)(b_off[i] + boff) * 2u;
        const bool real = BI * NW == NBI || i * NW + wid < NBI;  // (wave-uniform)
        if (TPS > 1 && !real) continue;
        unsigned char* d = real ? Bs + (i * NW + wid) * 1024 : smem + SCR;
        hdma16(br, d, ok ? off : OOB_OFF);
        hdma16(br, real ? d + B_PL : d, ok ? off + b_lo : OOB_OFF);
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
  // halo row of each A fragment row at tap (0, 0); tap (dh, dw) adds dh·PITCH + dw
  int hbase[TM], hkey[TM];  // (hkey: the image-row term of key(hr) at tap row 0, premultiplied)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int pix = wm0 + i * 32 + (lane & 31);
    const int img = pix / (TH * TW), rr = pix - img * (TH * TW);
    const int th = rr / TW, tw = rr - th * TW;
    hbase[i] = img * HH2 * PITCH + th * PITCH + tw;
    hkey[i] = (img * HH2 + th) * KC;  // = (hbase + dh·PITCH + dw) / PITCH · KC − dh·KC (tw + dw < PITCH)
  }
  const int rsw = (lane >> 2) & 3;  // row-major weight image key of fragment row (lane & 31)
  auto compute = [&](int hb, int slot, int shift, int dh) {
    const unsigned char* Hs = smem + H_OFF + hb * 2 * H_PL;
    const unsigned char* Bs = smem + B_OFF + slot * 2 * B_PL;  // (slot: the tile index, slot·TPS + u)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int hr = hbase[i] + shift;
        const unsigned char* a = Hs + hr * 64 + (((ks * 2 + h) ^ (((hr >> 2) + hkey[i] + dh * KC) & 3)) << 4);
        ah[i] = *reinterpret_cast<const bf16x8*>(a);
        al[i] = *reinterpret_cast<const bf16x8*>(a + H_PL);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (!BKM) {
          const unsigned char* b = Bs + (wn0 + j * 32 + (lane & 31)) * 64 + (((ks * 2 + h) ^ rsw) << 4);
          bh[j] = *reinterpret_cast<const bf16x8*>(b);
          bl[j] = *reinterpret_cast<const bf16x8*>(b + B_PL);
        } else {
          const int kr = ks * 16 + 8 * h + q;
          const int f = SS > 1 ? (kr / SD) & (SS - 1) : 0;
          const int col = (wn0 + j * 32 + 16 * (g & 1) + 4 * pp) ^ (f << 5);
          const bf16_t* b0p = reinterpret_cast<const bf16_t*>(Bs) + kr * BN + col;
          bh[j] = tr_frag(b0p, b0p + 4 * BN);
          bl[j] = tr_frag(b0p + B_PL / 2, b0p + B_PL / 2 + 4 * BN);
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

  // issue order: halo(0), w(0) [, w(1)] | step s: [wait, barrier] w(s+NBS-1), (HB 2, tap 0)
  // halo(c+1), MFMAs; HB 1: a chunk start first retires the old halo's reads (barrier), loads
  // the new one and waits for everything
  if constexpr (COEF_C > 0) {
    for (int i = threadIdx.x; i < 2 * p.C; i += NW * 64) coef_s[i] = bcoef[i];
    __syncthreads();
  }
  issue_halo(0, 0);
  issue_w(0, 0);
  if constexpr (NBS == 3) issue_w(1, 1);
  if constexpr (TPS > 1) {
    // (one halo buffer) steps of TPS taps: the chunk's halo at its first step, as below
    int c = 0, j = 0;
    for (int s = 0; s < nsteps; ++s) {
      if (j == 0 && c > 0) {
        __builtin_amdgcn_s_barrier();
        issue_halo(c, 0);
        hwait_vm<0>();
      } else {
        hwait_vm<TPS * GB*(NBS - 2)>();
      }
      __builtin_amdgcn_s_barrier();
      issue_w(s + NBS - 1, (s + NBS - 1) % NBS);
#pragma unroll
      for (int u = 0; u < TPS; ++u) {
        const int tap = j * TPS + u;
        if (tap < 9) {
          const int dh = tap / 3;
          compute(0, (s % NBS) * TPS + u, dh * PITCH + (tap - dh * 3), dh);
        }
      }
      if (++j == SPC) {
        j = 0;
        ++c;
      }
    }
  } else {
  int c = 0, tap = 0;
  for (int s = 0; s < nsteps; ++s) {
    if constexpr (HB == 2) {
      // w(s) and halo(c) are older than every DMA still allowed in flight: w(s+1) always, and
      // halo(c+1) at taps 1 and 2 (issued at tap 0 right after w(s+2))
      if (tap == 1 || tap == 2)
        hwait_vm<GB + GH>();
      else
        hwait_vm<GB>();
    } else {
      if (tap == 0 && c > 0) {
        __builtin_amdgcn_s_barrier();
        issue_halo(c, 0);
        hwait_vm<0>();
      } else {
        hwait_vm<GB*(NBS - 2)>();
      }
    }
    __builtin_amdgcn_s_barrier();
    issue_w(s + NBS - 1, (s + NBS - 1) % NBS);
    if constexpr (HB == 2)
      if (tap == 0) issue_halo(c + 1, (c + 1) & 1);
    const int dh = tap / 3;
    compute(HB == 2 ? (c & 1) : 0, s % NBS, dh * PITCH + (tap - dh * 3), dh);
    if (++tap == 9) {
      tap = 0;
      ++c;
    }
  }
  }
  hwait_vm<0>();

  // (epilogue operand prefetch where the accumulators leave the VGPRs for it: the l1 shape, whose
  // dgrads carry a residual gradient and BN partials over 64 channels)
  nt_f32_epilogue<TM, TN, NW, (TM * TN <= 2 ? 2 : -1), false>(p, acc, smem, client, m0, n0, wm0, wn0, wid, lane);
}

template <int IMG, int TH, int TW, int BN, int WM, int WN, int HB, int NBS, int TPS = 1, int MINW = 1>
void launch_halo(const ConvNTParams& p, int K, hipStream_t s) {
  const int tilesM = IMG == 1 ? p.B * (p.OH / TH) : p.B / IMG;
  const int grid = K * tilesM * cdiv(p.N, BN);
  if (p.b_kmajor)
    hipLaunchKernelGGL((conv_halo_kernel<IMG, TH, TW, BN, WM, WN, true, MINW, HB, NBS, 0, TPS>), dim3(grid),
                       dim3(WM * WN * 64), 0, s, p);
  else
    hipLaunchKernelGGL((conv_halo_kernel<IMG, TH, TW, BN, WM, WN, false, MINW, HB, NBS, 0, TPS>), dim3(grid),
                       dim3(WM * WN * 64), 0, s, p);
}

// MINW 2: two workgroups per CU asked of the register allocator (the l1 fused-BN tile otherwise
// lands at 129 VGPRs: one workgroup per CU)
template <int IMG, int TH, int TW, int BN, int WM, int WN, int NBS, int BNM = 1, int TPS = 1, int MINW = 1>
void launch_halo_bnf(const ConvNTParams& p, int K, hipStream_t s) {
  const int tilesM = IMG == 1 ? p.B * (p.OH / TH) : p.B / IMG;
  const int grid = K * tilesM * cdiv(p.N, BN);
  hipLaunchKernelGGL((conv_halo_kernel<IMG, TH, TW, BN, WM, WN, false, MINW, 1, NBS, BNM, TPS>), dim3(grid),
                     dim3(WM * WN * 64), 0, s, p);
}

// two taps per pipeline step: the 32² / 64-channel ResNet shape (headline −2.6 %,
// profiles/r5_c12_ab_halo_tps2.txt); the DenseNet growth convs (32-wide N tiles) measured even with
// it (9.45 / 9.48 vs 9.46 / 9.53 s per DenseNet-40 round) and keep one tap per step

int g_halo_mode = -1;  // -1 shape rule, 0 never, 1 whenever supported (tests / A-B)
int g_halo_variant = -1;

}  // namespace

void conv_halo_set_mode(int m) { g_halo_mode = m; }
void conv_halo_set_variant(int v) { g_halo_variant = v; }

// one of the compiled tile shapes fits this launch: full-width row blocks of 256 GEMM rows
static int halo_config(const ConvNTParams& p) {
  if (p.KH != 3 || p.KW != 3 || p.stride != 1 || p.pad != 1 || p.pad_w != 1 || p.dil != 1) return -1;
  const bool dense = p.bn_x != nullptr && p.bn_c > 0;
  if (p.OH != p.H || p.OW != p.W || p.out_s > 1 || p.C % 32 || p.N % (dense ? 4 : 8) || p.ldx % 8 || p.R != 9 * p.C)
    return -1;
  if ((p.x_lo == 0 && p.bn_x == nullptr) || p.wsplit == nullptr) return -1;
  if (p.bn_x != nullptr && (p.b_kmajor || (!dense && p.ldx != p.C))) return -1;
  // (the LDS copy of the BN coefficients: kernel COEF_C)
  if (p.bn_x != nullptr && p.C > (dense ? (p.OW == 8 ? 1 << 30 : 512) : (p.OW == 32 ? 128 : p.OW == 8 ? 256 : 1 << 30)))
    return -1;
  if (dense) {  // DenseNet growth conv (N = growth ≤ 32): 32-wide N tiles, 4 waves of 64 x 32
    if (p.N > 32 || p.bn_c % 4 || p.bn_c > p.C || p.bn_c > p.ldx || (p.bn_y && p.bn_ldy % 4)) return -1;
    if (p.bn_mask && (!p.bn_y || p.bn_ldy % 8 || p.bn_c % 8)) return -1;
    if (p.OW == 32 && p.OH % 8 == 0) return 4;            // 1 × 8 × 32
    if (p.OW == 16 && p.OH == 16) return 5;               // 1 × 16 × 16
    if (p.OW == 8 && p.OH == 8 && p.B % 4 == 0) return 6;  // 4 × 8 × 8
    return -1;
  }
  if (p.OW == 32 && p.OH % 8 == 0 && p.N <= 64) return 0;  // 1 × 8 × 32, BN 64
  if (p.OW == 16 && p.OH == 16) return 1;                   // 1 × 16 × 16, BN 128
  if (p.OW == 8 && p.OH == 8 && p.B % 2 == 0) return 2;     // 2 × 8 × 8, BN 128
  // (4 × 4 images: the 256 x 256 implicit-GEMM tile of conv_pl.hip is as fast forward and faster
  // in dgrad — l4 387 / 310 vs 385 / 331 TFLOP/s — so the halo shape serves it only on request)
  if (p.OW == 4 && p.OH == 4 && p.B % 8 == 0 && g_halo_mode == 1) return 3;  // 8 × 4 × 4, BN 128
  return -1;
}

bool conv_halo(const ConvNTParams& p, int K, hipStream_t s) {
  if (g_halo_mode == 0 || p.yp) return false;  // (no output-planes stores in the halo epilogue)
  const int cfg = halo_config(p);
  if (cfg < 0) return false;
  const long ab = (p.x_lo + (long)p.B * p.H * p.W * p.ldx) * 2;
  const long wb = (p.ws_plane + (p.b_kmajor ? (long)p.C * p.wKH * p.wKW * p.N : (long)p.N * p.R)) * 2;
  if (ab >= (long)OOB_OFF || wb >= (long)OOB_OFF) return false;
  // variants (bench/kernel_bench.py --planes sweeps them): 0 = two halo buffers + 3 weight slots;
  // 1 / 2 = one halo buffer (two workgroups per CU where the LDS allows), 8 waves
  // measured (kernel_bench --f32 --planes, 50 clients; fwd / dgrad TFLOP/s vs the implicit-GEMM
  // plane kernels): l1 v1 302 / 275 (259 / 247), l2 v1 441 / 396 (338 / 310), l3 v2 409 / 344
  // (361 / 321)
  if (p.bn_x != nullptr) {  // fused BN input: the default one-halo-buffer shapes only
    if (g_halo_variant >= 0 || cfg == 3) return false;
    switch (cfg) {
      case 0: launch_halo_bnf<1, 8, 32, 64, 4, 2, 2, 1, 2, 2>(p, K, s); break;
      case 1: launch_halo_bnf<1, 16, 16, 128, 4, 2, 2>(p, K, s); break;
      case 2: launch_halo_bnf<2, 8, 8, 128, 4, 2, 2>(p, K, s); break;
      case 4: launch_halo_bnf<1, 8, 32, 32, 4, 1, 3, 2>(p, K, s); break;   // 62 KB
      case 5: launch_halo_bnf<1, 16, 16, 32, 4, 1, 3, 2>(p, K, s); break;  // 62 KB
      case 6: launch_halo_bnf<4, 8, 8, 32, 4, 1, 3, 2>(p, K, s); break;    // 78 KB
      // (8 waves of 32 x 32 per tile: bitwise the same, no faster — r4_c14_dn_w*.log)
      default: return false;
    }
    return true;
  }
  // (measured at 32² / 64 channels and removed: 16 waves with two halo buffers, one workgroup per
  // CU, +42 % forward; 4-row blocks with three workgroups per CU, +15 %,
  // profiles/r6_c9_halo_l1_variant5_rejected.log)
  const int v = g_halo_variant >= 0 ? g_halo_variant : (cfg == 2 ? 2 : 1);
  if (cfg > 3) return false;
  if (cfg == 0 && (v == 1 || v == 3)) {  // 32² / 64 channels: two taps per step
    launch_halo<1, 8, 32, 64, 4, 2, 1, 2, 2>(p, K, s);      // 74 KB
    return true;
  }
  if (v > 2) return false;
  switch (cfg * 3 + v) {
    case 0: launch_halo<1, 8, 32, 64, 4, 1, 2, 3>(p, K, s); break;    // 120 KB, 4 waves
    case 2: launch_halo<1, 8, 32, 64, 4, 2, 2, 3>(p, K, s); break;    // 121 KB
    case 3: launch_halo<1, 16, 16, 128, 4, 2, 2, 3>(p, K, s); break;  // 144 KB
    case 4: launch_halo<1, 16, 16, 128, 4, 2, 1, 2>(p, K, s); break;  // 80 KB
    case 5: launch_halo<1, 16, 16, 128, 4, 2, 1, 3>(p, K, s); break;  // 96 KB
    case 6: launch_halo<2, 8, 8, 128, 2, 2, 2, 3>(p, K, s); break;    // 112 KB, 4 waves
    case 7: launch_halo<2, 8, 8, 128, 4, 2, 1, 3>(p, K, s); break;    // 80 KB, 8 waves
    case 8: launch_halo<2, 8, 8, 128, 4, 2, 1, 2>(p, K, s); break;    // 64 KB
    case 9: launch_halo<8, 4, 4, 128, 2, 2, 2, 3>(p, K, s); break;    // 144 KB, 4 waves
    case 10: launch_halo<8, 4, 4, 128, 4, 2, 1, 3>(p, K, s); break;   // 96 KB, 8 waves
    case 11: launch_halo<8, 4, 4, 128, 4, 2, 1, 2>(p, K, s); break;   // 80 KB
    default: return false;
  }
  return true;
}

bool conv_halo_bn_supported(int B, int H, int W, int C, int N) {
  ConvNTParams p{};
  p.bn_x = reinterpret_cast<const float*>(16);  // (shape check only)
  p.wsplit = reinterpret_cast<const bf16_t*>(16);
  p.B = B; p.H = H; p.W = W; p.C = C; p.OH = H; p.OW = W; p.KH = 3; p.KW = 3;
  p.stride = 1; p.pad = 1; p.pad_w = 1; p.dil = 1; p.N = N; p.R = 9 * C; p.ldx = C; p.out_s = 1;
  const int cfg = halo_config(p);
  return g_halo_mode != 0 && g_halo_variant < 0 && cfg >= 0 && cfg != 3 && (long)B * H * W * C * 4 < (1L << 31);
}

static ConvNTParams halo_bn_params(const float* x, long x_cs, int ldx, const float* coef, int relu,
                                   const int* valid_rows, const bf16_t* wsplit, long ws_cs, long ws_plane, int rep,
                                   float* y, long y_cs, int ldy, int B, int H, int W, int C, int N, float* stats,
                                   const int* stats_valid) {
  ConvNTParams p{};
  p.f32 = 1;
  p.bn_x = x;
  p.bn_x_cs = x_cs;
  p.bn_coef = coef;
  p.bn_relu = relu;
  p.bn_valid = valid_rows;
  p.wsplit = wsplit;
  p.ws_cs = ws_cs;
  p.ws_plane = ws_plane;
  p.rep = rep;
  p.y = reinterpret_cast<bf16_t*>(y);
  p.y_cs = y_cs;
  p.B = B; p.H = H; p.W = W; p.C = C; p.OH = H; p.OW = W; p.KH = 3; p.KW = 3;
  p.stride = 1; p.pad = 1; p.pad_w = 1; p.dil = 1;
  p.M = B * H * W; p.N = N; p.R = 9 * C;
  p.wKH = 3; p.wKW = 3; p.kh_off = 2; p.kw_off = 2; p.kh_step = 1; p.kw_step = 1;
  p.out_s = 1;
  p.ldx = ldx; p.ldy = ldy;
  p.fd_ohw = make_fastdiv((uint32_t)(H * W));
  p.fd_ow = make_fastdiv((uint32_t)W);
  p.fd_kwc = make_fastdiv((uint32_t)(3 * C));
  p.fd_c = make_fastdiv((uint32_t)C);
  p.stats = stats;
  p.stats_valid = stats_valid;
  return p;
}

bool conv_halo_bn_fwd(const float* x, long x_cs, const float* coef, int relu, const int* valid_rows,
                      const bf16_t* wsplit, long ws_cs, long ws_plane, int rep, float* y, long y_cs, int K, int B,
                      int H, int W, int C, int N, float* stats, const int* stats_valid, hipStream_t s,
                      bf16_t* yp, uint8_t* mask) {
  ConvNTParams p = halo_bn_params(x, x_cs, C, coef, relu, valid_rows, wsplit, ws_cs, ws_plane, rep, y, y_cs, N, B, H,
                                  W, C, N, stats, stats_valid);
  p.bn_yp = yp;
  p.bn_mask = mask;
  if (stats && stats_valid && !yp && native_option(g_opt_halo_skip, "DLS_SKIP_INVALID", 1)) {
    // (not with planes: an implicit-GEMM weight gradient would read them whole)
    p.skip_valid = stats_valid;
    p.skip_mul = H * W;
  }
  const long wb = (ws_plane + (long)N * p.R) * 2;
  if (wb >= (long)OOB_OFF || (long)p.M * C * 4 >= (1L << 31)) return false;
  return conv_halo(p, K, s);
}

bool conv_halo_bn_dense_supported(int B, int H, int W, int C, int N) {
  ConvNTParams p{};
  p.bn_x = reinterpret_cast<const float*>(16);  // (shape check only)
  p.wsplit = reinterpret_cast<const bf16_t*>(16);
  p.bn_c = 4;
  p.B = B; p.H = H; p.W = W; p.C = C; p.OH = H; p.OW = W; p.KH = 3; p.KW = 3;
  p.stride = 1; p.pad = 1; p.pad_w = 1; p.dil = 1; p.N = N; p.R = 9 * C; p.ldx = C; p.out_s = 1;
  return g_halo_mode != 0 && g_halo_variant < 0 && halo_config(p) >= 4;
}

bool conv_halo_bn_dense_fwd(const float* x, long x_cs, int ldx, int creal, const float* coef, int relu,
                            const int* valid_rows, const bf16_t* wsplit, long ws_cs, long ws_plane, int rep, float* y,
                            long y_cs, int ldy, int K, int B, int H, int W, int C, int N, float* stats,
                            const int* stats_valid, float* ny, long ny_cs, int ldny, uint8_t* mask, hipStream_t s) {
  ConvNTParams p = halo_bn_params(x, x_cs, ldx, coef, relu, valid_rows, wsplit, ws_cs, ws_plane, rep, y, y_cs, ldy, B,
                                  H, W, C, N, stats, stats_valid);
  p.bn_c = creal;
  p.bn_y = ny;
  p.bn_y_cs = ny_cs;
  p.bn_ldy = ldny;
  p.bn_mask = mask;
  const long wb = (ws_plane + (long)N * p.R) * 2;
  if (wb >= (long)OOB_OFF || (long)p.M * ldx * 4 >= (1L << 31)) return false;
  if (halo_config(p) < 4) return false;
  return conv_halo(p, K, s);
}
