// DenseNet growth-conv weight gradient with LDS halo reuse (gfx950, MI355X).
//
// dW[n][tap][c] = Σ_pixels dY[p][n] · Y[p + tap][c] for a 3x3 / stride-1 / pad-1 conv with few
// output channels (the growth rate, N ≤ 16) over a wide channel prefix (c < C). The implicit-GEMM
// TN kernel (conv_f32.hip, 32-row tile) gathers every Y element nine times through L2 and splits it
// nine times in registers, and 20 of its 32 MFMA rows are padding: it ran at ≈ 10 % of the MFMA
// rate (DenseNet-40 profile: 19 % of the round). Here a workgroup owns one client, one 32-channel
// chunk of the prefix and a strided set of pixel tiles (IMG images × TH rows × full width):
//   * per tile the Y halo ((TH+2)·(TW+2) pixels per image, 32 channels) and the dY tile (TP
//     pixels × N) are loaded ONCE, split to bf16 hi / lo while staged, into LDS;
//   * nine waves, one per tap, run v_mfma_f32_16x16x32_bf16 (16 rows: N ≤ 16, 12 used) with the
//     pixel as the reduction index: A = dYᵀ and B = the tap-shifted halo, both read k-major with
//     ds_read_b64_tr_b16 (lane i of a 16-lane group gets column i of 4 pixel rows);
//   * products are bf16x3 like every fp32 GEMM here (al·bh + ah·bl + ah·bh, fp32 accumulate).
// Each workgroup writes its 16 x 9 x 32 partial to its own slab; a fold sums the G slabs of a
// (client, chunk) in slab order into dW — no atomics, bitwise reproducible, and the pixel split G
// depends on the per-client shape only (so N ranks give the bits of one).
// LDS rows are 64 B (32 bf16); the 32-byte half a channel (or n) range lands in is XORed with bit
// 3 of the row, so the two 16-lane groups of a transposed read (rows 8 apart) hit disjoint banks.
#include "dls.h"
#include "gemm_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_off(int row, int half) { return (uint32_t)(row * 64 + ((half ^ ((row >> 3) & 1)) << 5)); }

template <int IMG, int TH, int TW, bool REC>
__global__ void __launch_bounds__(576) __attribute__((amdgpu_waves_per_eu(5, 8))) dense_wgrad_kernel(DenseWgradParams p) {
  constexpr int TP = IMG * TH * TW;  // GEMM k rows (pixels) per tile
  static_assert(TP % 32 == 0 && TW % 8 == 0, "tile");
  constexpr int HW2 = TW + 2, HH2 = TH + 2;
  constexpr int HP = IMG * HH2 * HW2;  // halo rows
  constexpr int Y_PL = HP * 64, D_PL = TP * 64;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * Y_PL + 2 * D_PL];
  unsigned char* Yh = smem;
  unsigned char* Yl = smem + Y_PL;
  unsigned char* Dh = smem + 2 * Y_PL;
  unsigned char* Dl = Dh + D_PL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int tap = __builtin_amdgcn_readfirstlane(tid >> 6);  // one wave per tap
  const int per_client = p.nchunks * p.G;
  const int client = blockIdx.x / per_client;
  const int rem = blockIdx.x - client * per_client;
  const int chunk = rem / p.G, g = rem - chunk * p.G;
  const int c0 = chunk * 32;
  const float* __restrict__ yb_ = p.y + (long)client * p.y_cs;
  const float* __restrict__ db = p.dy + (long)client * p.dy_cs;
  const int tpi = p.H / TH;  // row blocks per image (IMG == 1)
  const int tiles = IMG == 1 ? p.B * tpi : p.B / IMG;

  // MFMA operand addressing (per lane, per k-step s: pixel pt = 32s + 8·(lane>>4) + q and pt + 4)
  const int i16 = lane & 15, q = i16 >> 2, pp = i16 & 3, g4 = lane >> 4;
  const int kh = tap / 3, kw = tap - kh * 3;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  // REC: the chunk's (scale, shift) pairs in LDS (zeros past the prefix: y = relu(0·x + 0) = 0
  // there); a halo pixel outside the image or past the client's valid samples stages as zeros
  // (its live bit, taken at load time)
  __shared__ __attribute__((aligned(16))) float sc_s[REC ? 64 : 1];
  const int ldy = REC ? p.ldy_x : p.C;
  const int nvalid = REC && p.valid_rows ? min(p.valid_rows[client], p.B * p.H * p.W) : p.B * p.H * p.W;
  if constexpr (REC) {
    if (tid < 64) {
      const int c = c0 + (tid >> 1);
      sc_s[tid] = c < p.C ? p.bn_sc[((long)client * p.C + c) * 2 + (tid & 1)] : 0.f;
    }
  }
  uint32_t live_bits = 0;

  // global → registers for tile t (issued one tile ahead: the loads of tile t + G fly while
  // tile t's MFMAs run), registers → split bf16 planes in LDS
  constexpr int YR = (HP * 4 + 575) / 576, DR = (TP * 4 + 575) / 576;
  float4 ya[YR], yb[YR], dv[DR];
  auto load_tile = [&](int t) {
    const int b0 = IMG == 1 ? t / tpi : t * IMG;
    const int h0 = IMG == 1 ? (t - (t / tpi) * tpi) * TH : 0;
#pragma unroll
    for (int r = 0; r < YR; ++r) {  // Y halo: (halo row, 8-channel group) tasks
      const int task = tid + r * 576;
      const int hr = task >> 2, cg = task & 3;
      const int img = hr / (HH2 * HW2), r2 = hr - img * (HH2 * HW2);
      const int hh = r2 / HW2, ww = r2 - hh * HW2;
      const int ih = h0 - 1 + hh, iw = ww - 1;
      const bool ok = task < HP * 4 && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const int c = c0 + cg * 8, cv = p.C - c;  // zeros outside the image / past the prefix
      const long pix = (long)((b0 + img) * p.H + (ok ? ih : 0)) * p.W + (ok ? iw : 0);
      const long e = pix * ldy + c;
      ya[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      yb[r] = ya[r];
      if (ok && cv > 0) ya[r] = *reinterpret_cast<const float4*>(yb_ + e);
      if (ok && cv >= 8) yb[r] = *reinterpret_cast<const float4*>(yb_ + e + 4);
      if constexpr (REC) {
        if (r == 0) live_bits = 0;
        live_bits |= (ok && pix < nvalid ? 1u : 0u) << r;
      }
    }
#pragma unroll
    for (int r = 0; r < DR; ++r) {  // dY tile: (pixel, 4-channel group) tasks, n ≥ N zero
      const int task = tid + r * 576;
      const int pt = task >> 2, ng = task & 3;
      const int img = pt / (TH * TW), r2 = pt - img * (TH * TW);
      const int th = r2 / TW, tw = r2 - th * TW;
      const long pix = (long)((b0 + img) * p.H + h0 + th) * p.W + tw;
      dv[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (task < TP * 4 && ng * 4 < p.N) dv[r] = *reinterpret_cast<const float4*>(db + pix * p.ldy + ng * 4);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int r = 0; r < YR; ++r) {
      const int task = tid + r * 576;
      if (task < HP * 4) {
        const int hr = task >> 2, cg = task & 3;
        if constexpr (REC) {  // y = relu(BN(x)) as the forward's halo loader computes it (conv_halo.hip BNM 2)
          const float4* cs = reinterpret_cast<const float4*>(sc_s + cg * 16);
          const float4 k0 = cs[0], k1 = cs[1], k2 = cs[2], k3 = cs[3];
          const bool lv = (live_bits >> r) & 1u;
          ya[r] = lv ? make_float4(fmaxf(fmaf(ya[r].x, k0.x, k0.y), 0.f), fmaxf(fmaf(ya[r].y, k0.z, k0.w), 0.f),
                                   fmaxf(fmaf(ya[r].z, k1.x, k1.y), 0.f), fmaxf(fmaf(ya[r].w, k1.z, k1.w), 0.f))
                     : make_float4(0.f, 0.f, 0.f, 0.f);
          yb[r] = lv ? make_float4(fmaxf(fmaf(yb[r].x, k2.x, k2.y), 0.f), fmaxf(fmaf(yb[r].y, k2.z, k2.w), 0.f),
                                   fmaxf(fmaf(yb[r].z, k3.x, k3.y), 0.f), fmaxf(fmaf(yb[r].w, k3.z, k3.w), 0.f))
                     : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        uint32_t hi[4], lo[4];
        split_pair(ya[r].x, ya[r].y, hi[0], lo[0]);
        split_pair(ya[r].z, ya[r].w, hi[1], lo[1]);
        split_pair(yb[r].x, yb[r].y, hi[2], lo[2]);
        split_pair(yb[r].z, yb[r].w, hi[3], lo[3]);
        const uint32_t off = lds_off(hr, cg >> 1) + ((cg & 1) << 4);
        *reinterpret_cast<uint4*>(Yh + off) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
        *reinterpret_cast<uint4*>(Yl + off) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
      }
    }
#pragma unroll
    for (int r = 0; r < DR; ++r) {
      const int task = tid + r * 576;
      if (task < TP * 4) {
        const int pt = task >> 2, ng = task & 3;
        uint32_t hi0, lo0, hi1, lo1;
        split_pair(dv[r].x, dv[r].y, hi0, lo0);
        split_pair(dv[r].z, dv[r].w, hi1, lo1);
        const uint32_t off = lds_off(pt, 0) + (ng << 3);
        *reinterpret_cast<uint2*>(Dh + off) = make_uint2(hi0, hi1);
        *reinterpret_cast<uint2*>(Dl + off) = make_uint2(lo0, lo1);
      }
    }
  };

  if (g < tiles) load_tile(g);
  for (int t = g; t < tiles; t += p.G) {
    __syncthreads();  // the previous tile's reads are done
    store_tile();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS stores landed
    __syncthreads();
    if (t + p.G < tiles) load_tile(t + p.G);
    // ---- this wave's tap over the tile's pixels
#pragma unroll 1
    for (int s = 0; s < TP / 32; ++s) {
      const int pt = 32 * s + 8 * g4 + q;  // (pt and pt + 4: one 8-aligned run of one image row)
      const int img = pt / (TH * TW), r2 = pt - img * (TH * TW);
      const int th = r2 / TW, tw = r2 - th * TW;
      const int hr = img * HH2 * HW2 + (th + kh) * HW2 + tw + kw;
      const bf16_t* a1 = reinterpret_cast<const bf16_t*>(Dh + lds_off(pt, 0) + pp * 8);
      const bf16_t* a2 = reinterpret_cast<const bf16_t*>(Dh + lds_off(pt + 4, 0) + pp * 8);
      const bf16x8 ah = tr_frag(a1, a2);
      const bf16x8 al = tr_frag(a1 + D_PL / 2, a2 + D_PL / 2);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const bf16_t* b1 = reinterpret_cast<const bf16_t*>(Yh + lds_off(hr, hf) + pp * 8);
        const bf16_t* b2 = reinterpret_cast<const bf16_t*>(Yh + lds_off(hr + 4, hf) + pp * 8);
        const bf16x8 bh = tr_frag(b1, b2);
        const bf16x8 bl = tr_frag(b1 + Y_PL / 2, b2 + Y_PL / 2);
        acc[hf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[hf], 0, 0, 0);
        acc[hf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[hf], 0, 0, 0);
        acc[hf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[hf], 0, 0, 0);
      }
    }
  }
  // ---- partial slab [16 n][9 taps][32 c] of this workgroup: lane holds rows n = 4·(lane>>4) + e,
  // column c = hf·16 + (lane & 15)
  float* slab = p.part + ((long)(client * p.nchunks + chunk) * p.G + g) * (16 * 9 * 32);
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int e = 0; e < 4; ++e) slab[((4 * g4 + e) * 9 + tap) * 32 + hf * 16 + i16] = acc[hf][e];
}

// dW[k][n][tap][c] = Σ_g slab[k][c / 32][g][n][tap][c % 32], g in order
__global__ void __launch_bounds__(256) dense_wgrad_fold_kernel(DenseWgradParams p) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long per = (long)p.N * 9 * p.C;
  if (idx >= per * p.K) return;
  const int k = (int)(idx / per);
  const long r = idx - (long)k * per;
  const int n = (int)(r / (9 * p.C));
  const int r2 = (int)(r - (long)n * 9 * p.C);
  const int tap = r2 / p.C, c = r2 - tap * p.C;
  const float* src = p.part + ((long)(k * p.nchunks + c / 32) * p.G) * (16 * 9 * 32) + (n * 9 + tap) * 32 + (c & 31);
  float s = 0.f;
  for (int gg = 0; gg < p.G; ++gg) s += src[(long)gg * (16 * 9 * 32)];
  p.dw[(long)k * p.dw_cs + r] = s;
}

}  // namespace

// shape rule: full-width tiles of 256 (128 for 8 x 8) pixels, growth ≤ 16 in 4-channel groups
static int dense_wgrad_cfg(int B, int H, int W, int N) {
  if (N > 16 || N % 4 || H != W) return -1;
  if (H == 32) return 0;
  if (H == 16) return 1;
  if (H == 8 && B % 2 == 0) return 2;
  return -1;
}

bool dense_wgrad_supported(int B, int H, int W, int C, int N) {
  return dense_wgrad_cfg(B, H, W, N) >= 0 && C % 4 == 0;
}

int dense_wgrad_groups(int B, int H, int W) {
  const int tiles = H == 32 ? B * 4 : H == 16 ? B : B / 2;
  return tiles < 16 ? tiles : 16;
}

long dense_wgrad_part_floats(int K, int B, int H, int W, int C) {
  return (long)K * ((C + 31) / 32) * dense_wgrad_groups(B, H, W) * 16 * 9 * 32;
}

bool dense_wgrad(const float* dy, long dy_cs, int ldy, const float* y, long y_cs, float* dw, long dw_cs, float* part,
                 int K, int B, int H, int W, int C, int N, hipStream_t s, const float* bn_sc, int ldy_x,
                 const int* valid_rows) {
  const int cfg = dense_wgrad_cfg(B, H, W, N);
  if (cfg < 0 || C % 4 || ldy % 4 || (bn_sc && ldy_x % 4)) return false;
  DenseWgradParams p{};
  p.dy = dy;
  p.dy_cs = dy_cs;
  p.ldy = ldy;
  p.y = y;
  p.y_cs = y_cs;
  p.dw = dw;
  p.dw_cs = dw_cs;
  p.part = part;
  p.K = K;
  p.B = B;
  p.H = H;
  p.W = W;
  p.C = C;
  p.N = N;
  p.nchunks = (C + 31) / 32;
  p.G = dense_wgrad_groups(B, H, W);
  p.bn_sc = bn_sc;
  p.ldy_x = ldy_x;
  p.valid_rows = valid_rows;
  const int grid = K * p.nchunks * p.G;
#define DW_LAUNCH(REC_)                                                                                 \
  switch (cfg) {                                                                                     \
    case 0: hipLaunchKernelGGL((dense_wgrad_kernel<1, 8, 32, REC_>), dim3(grid), dim3(576), 0, s, p); break;  \
    case 1: hipLaunchKernelGGL((dense_wgrad_kernel<1, 16, 16, REC_>), dim3(grid), dim3(576), 0, s, p); break; \
    default: hipLaunchKernelGGL((dense_wgrad_kernel<2, 8, 8, REC_>), dim3(grid), dim3(576), 0, s, p); break;  \
  }
  if (bn_sc) {
    DW_LAUNCH(true)
  } else {
    DW_LAUNCH(false)
  }
#undef DW_LAUNCH
  const long total = (long)K * N * 9 * C;
  hipLaunchKernelGGL(dense_wgrad_fold_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
  return true;
}
