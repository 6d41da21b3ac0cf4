// 3x3 / stride-1 / pad-1 convolution WEIGHT GRADIENT on pre-split operands with LDS halo reuse
// (gfx950, MI355X).
//
//   dW[co][kh][kw][c] = Σ_pixels dY[pix][co] · X[pix shifted by (kh − 1, kw − 1)][c]
//
// The implicit-GEMM wgrad (conv_pl.hip conv_tn_pl_kernel) stages the im2col B operand
// X̃[pix][(kh, kw, c)] tap by tap: every input pixel crosses L2 → LDS up to 9 times, and with
// the dY tile besides that the LDS-DMA path (≈60–70 GB/s per CU) bounds it below half the
// MFMA rate (PMC: 31–41 % MFMA busy). Here a workgroup owns an output tile of BMc output
// channels × ALL 9 taps × a 32-channel input chunk (BMc × 288) and walks the pixels 32 at a
// time — R = 32 / W whole output rows of one image per K step. Per step it DMAs the dY tile
// [32 px][BMc] and the input HALO of those rows once ((R + 2) × (W + 2) pixels × 32 channels);
// the 9 taps read their B fragments from the halo at a uniform row shift. Bytes per MAC drop
// 2–3× against the implicit GEMM.
//
// Waves: (BMc / 32) × 3 — wave (wm, kh) computes co rows wm·32.. × taps (kh, 0..2) × 32
// channels: three 32×32 accumulators. Arithmetic is split-bf16 "bf16x3" on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation, operands pre-split into (hi, lo) bf16 planes
// by the producing BatchNorms (as conv_pl.hip). Fragments of both k-major images come from
// ds_read_b64_tr_b16 (tr_frag); the halo image needs no swizzle: a quad of k-rows is 4
// consecutive pixels of one image row, i.e. 4 consecutive 64-B halo rows (all 64 banks).
//
// Pipeline: NST-stage LDS ring, every DMA piece (1 KiB, one wave-instruction) of a stage
// assigned round-robin to the waves (a wave's surplus pieces write zeros to a scratch KiB, so
// every wave issues the same count); counted vmcnt + raw s_barrier (guide "Pipelining across
// barriers"). Split-K over pixels writes per-split slabs folded in order by tn_fold
// (conv_pl.hip): deterministic, no atomics.
//
// Contract (host checks, else conv_pl.hip serves): 3x3, stride 1, pad 1, W ∈ {8, 16, 32},
// OH·OW % 32 == 0, C % 32 == 0, Co % BMc == 0, contiguous planes, windows < 2 GiB.
#include "dls.h"
#include "gemm_common.h"

#include <algorithm>

namespace {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void wdma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wwait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int W>
struct HaloGeo {
  static constexpr int R = 32 / W;                 // output rows per K step
  static constexpr int PITCH = W + 2;              // halo pixels per halo row
  static constexpr int ROWS = (R + 2) * PITCH;     // halo pixels (64-B LDS rows per plane)
  static constexpr int HI = (ROWS + 15) / 16;      // 1-KiB DMA pieces per halo plane
};

template <int BMc>
struct KmSwzW {  // k-major [32][BMc] image: segment key of k-row kr (as conv_pl.hip KmSwz)
  static constexpr int SD = (128 / BMc) > 1 ? 128 / BMc : 1, SS = (BMc / 32) < 4 ? BMc / 32 : 4;
  static __device__ __forceinline__ int f(int kr) { return SS > 1 ? (kr / SD) & (SS - 1) : 0; }
};

template <int BMc, int TMW, int W, int NST>
__global__ void __launch_bounds__((BMc / (32 * TMW)) * 3 * 64) conv_wgrad_halo_kernel(ConvTNParams p) {
  using G = HaloGeo<W>;
  constexpr int WM = BMc / (32 * TMW), NW = WM * 3;
  constexpr int A_PL = 32 * BMc * 2;  // bytes of one dY plane image
  constexpr int AI = A_PL / 1024;     // 1-KiB pieces per dY plane
  constexpr int H_PL = G::HI * 1024;  // bytes of one halo plane image
  constexpr int STAGE = 2 * (A_PL + H_PL);
  constexpr int NP = 2 * (AI + G::HI);       // pieces per stage
  constexpr int GP = (NP + NW - 1) / NW;     // pieces per wave per stage
  constexpr int SCR = NST * STAGE;           // scratch KiB for surplus pieces
  constexpr int CPA = BMc / 8, RPA = 64 / CPA;  // dY image: 16-B chunks per k-row, k-rows per piece
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SCR + 1024];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tilesM = p.Co / BMc, tilesC = p.C / 32;
  const int per_client = tilesM * tilesC * p.splitk;
  const int nclients = gridDim.x / per_client;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  int t = bid - client * per_client;
  const int split = t % p.splitk;
  t /= p.splitk;
  const int co0 = (t / tilesC) * BMc, c0 = (t % tilesC) * 32;
  const int mbeg = split * p.m_per_split;
  const int mend = min(p.M, mbeg + p.m_per_split);

  const auto ar = make_rsrc(p.dy + (long)client * p.dy_cs, (uint32_t)((p.dy_lo + (long)p.M * p.ldy) * 2));
  const uint32_t a_lo = (uint32_t)(p.dy_lo * 2);
  const auto xr = make_rsrc(p.x + (long)client * p.x_cs, (uint32_t)((p.x_lo + (long)p.B * p.H * p.W * p.ldx) * 2));
  const uint32_t x_lo = (uint32_t)(p.x_lo * 2);

  // ---- this wave's GP pieces of every stage: piece j = n·NW + wid of the list
  //   [dY hi 0..AI-1 | dY lo 0..AI-1 | halo hi 0..HI-1 | halo lo 0..HI-1], j ≥ NP: scratch
  // static per-lane parts: dY pieces — k-row kr and column co (offset kr·ldy + co, advanced by
  // 32·ldy per step); halo pieces — halo row (hh, ww) → input pixel (oh0 − 1 + hh, ww − 1)
  int pc_kind[GP];  // 0 dY, 1 halo, 2 scratch (wave-uniform)
  int pc_plane[GP], pc_dst[GP], pc_off[GP], pc_hh[GP], pc_ww[GP];
#pragma unroll
  for (int n = 0; n < GP; ++n) {
    const int j = n * NW + wid;
    pc_hh[n] = 0;
    pc_ww[n] = 0;
    if (j < 2 * AI) {
      const int plane = j / AI, a = j % AI;
      const int kr = a * RPA + lane / CPA;
      const int co = co0 + ((lane % CPA) ^ (KmSwzW<BMc>::f(kr) << 2)) * 8;
      pc_kind[n] = 0;
      pc_plane[n] = plane;
      pc_dst[n] = plane * A_PL + a * 1024;
      pc_off[n] = kr * p.ldy + co;
    } else if (j < NP) {
      const int jj = j - 2 * AI;
      const int plane = jj / G::HI, h = jj % G::HI;
      const int hr = h * 16 + (lane >> 2);
      const int hh = hr / G::PITCH, ww = hr - hh * G::PITCH;
      pc_kind[n] = 1;
      pc_plane[n] = plane;
      pc_dst[n] = 2 * A_PL + plane * H_PL + h * 1024;
      pc_hh[n] = hr < G::ROWS ? hh : -(1 << 20);  // (rows past the halo: never in the image)
      pc_ww[n] = ww;
      pc_off[n] = (hh * p.W + ww) * p.ldx + c0 + (lane & 3) * 8;  // + image base − (W + 1)·ldx per step
    } else {
      pc_kind[n] = 2;
      pc_plane[n] = 0;
      pc_dst[n] = 0;
      pc_off[n] = 0;
    }
  }

  // stage state (wave-uniform): first pixel of the step, its image and first output row
  const int ohw = p.OH * p.OW;
  int k_m = mbeg;
  bool s_live = false;
  int s_m0 = 0, s_oh0 = 0;
  long s_img = 0;
  auto prep = [&](bool live) {
    s_live = live;
    s_m0 = k_m;
    const int b = k_m / ohw;
    s_oh0 = (k_m - b * ohw) / p.W;
    s_img = (long)b * p.H * p.W;
    k_m += 32;
  };
  auto piece = [&](int n, int buf) {
    unsigned char* base = smem + buf * STAGE;
    if (pc_kind[n] == 0) {
      const uint32_t off = (uint32_t)(pc_off[n] + s_m0 * p.ldy) * 2u + (pc_plane[n] ? a_lo : 0u);
      wdma16(ar, base + pc_dst[n], s_live ? off : OOB_OFF);
    } else if (pc_kind[n] == 1) {
      const int ih = s_oh0 - 1 + pc_hh[n], iw = pc_ww[n] - 1;
      const bool ok = s_live && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const long off = (s_img + (long)(s_oh0 - 1) * p.W - 1) * p.ldx + pc_off[n];
      wdma16(xr, base + pc_dst[n], ok ? (uint32_t)off * 2u + (pc_plane[n] ? x_lo : 0u) : OOB_OFF);
    } else {
      wdma16(xr, smem + SCR, OOB_OFF);
    }
  };

  f32x16 acc[TMW][3];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x16{};

  const int wm = wid % WM, kh = wid / WM;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3, h = lane >> 5;
  auto compute = [&](int buf) {
    const bf16_t* As = reinterpret_cast<const bf16_t*>(smem + buf * STAGE);
    const bf16_t* Hs = reinterpret_cast<const bf16_t*>(smem + buf * STAGE + 2 * A_PL);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kr = ks * 16 + 8 * h + q;  // pixel of the step (kr + 4: same image row, +4 halo rows)
      bf16x8 ah[TMW], al[TMW];
#pragma unroll
      for (int i = 0; i < TMW; ++i) {
        const bf16_t* a0 = As + kr * BMc + (((wm * TMW + i) * 32 + 16 * (g & 1) + 4 * pp) ^ (KmSwzW<BMc>::f(kr) << 5));
        ah[i] = tr_frag(a0, a0 + 4 * BMc);
        al[i] = tr_frag(a0 + A_PL / 2, a0 + A_PL / 2 + 4 * BMc);
      }
      const int hrow = (kr / W + kh) * G::PITCH + (kr % W);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const bf16_t* b0 = Hs + (hrow + kw) * 32 + 16 * (g & 1) + 4 * pp;
        const bf16x8 bh = tr_frag(b0, b0 + 4 * 32);
        const bf16x8 bl = tr_frag(b0 + H_PL / 2, b0 + H_PL / 2 + 4 * 32);
#pragma unroll
        for (int i = 0; i < TMW; ++i) {
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh, acc[i][kw], 0, 0, 0);
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl, acc[i][kw], 0, 0, 0);
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh, acc[i][kw], 0, 0, 0);
        }
      }
    }
  };

  const int nk = (mend - mbeg) / 32;
#pragma unroll
  for (int st = 0; st < NST - 1; ++st) {
    prep(st < nk);
#pragma unroll
    for (int n = 0; n < GP; ++n) piece(n, st);
  }
  for (int kt = 0; kt < nk; ++kt) {
    wwait_vm<GP*(NST - 2)>();
    __builtin_amdgcn_s_barrier();
    prep(kt + NST - 1 < nk);
#pragma unroll
    for (int n = 0; n < GP; ++n) piece(n, (kt + NST - 1) % NST);
    compute(kt % NST);
  }
  wwait_vm<0>();

  // ---- epilogue: dW[co][(kh·3 + kw)·C + c] (or this split's slab, folded in order by tn_fold)
  const bool slab = p.splitk > 1;
  float* __restrict__ dst = slab ? p.part + ((long)split * nclients + client) * p.Co * p.R : p.dw + (long)client * p.dw_cs;
  const int c = c0 + (lane & 31);
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int r = (kh * 3 + kw) * p.C + c;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + (wm * TMW + i) * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        dst[(long)co * p.R + r] = acc[i][kw][e];
      }
    }
}

template <int BMc, int TMW, int W>
void launch_wh(const ConvTNParams& p, int K, hipStream_t s) {
  const int grid = K * (p.Co / BMc) * (p.C / 32) * p.splitk;
  hipLaunchKernelGGL((conv_wgrad_halo_kernel<BMc, TMW, W, 3>), dim3(grid), dim3((BMc / (32 * TMW)) * 3 * 64), 0, s, p);
}

template <int BMc, int TMW>
void launch_wh_w(const ConvTNParams& p, int K, hipStream_t s) {
  if (p.W == 32) launch_wh<BMc, TMW, 32>(p, K, s);
  else if (p.W == 16) launch_wh<BMc, TMW, 16>(p, K, s);
  else launch_wh<BMc, TMW, 8>(p, K, s);
}

// -1 shape rule (off: measured slower than the implicit GEMM at 32 co per wave — l1 / l2 / l3
// 187 / 288 / 286 vs 221 / 316 / 346 TFLOP/s at 50 clients — LDS-read bound: 1.8 transposed
// reads per MFMA), 0 never, 1 = 32 co per wave, 2 = 64 co per wave (tests / A-B)
int g_wh_mode = -1;

}  // namespace

void conv_wgrad_halo_set_mode(int m) { g_wh_mode = m; }

// split-K from per-client quantities only (bitwise the same whatever the cohort: see conv_pl.hip)
static void wh_split(int Co, int C, int M, int bm, int& splitk, int& mps) {
  constexpr int KREF = 32;
  const long tiles = (long)KREF * (Co / bm) * (C / 32);
  splitk = 1;
  if (tiles < 768) splitk = (int)std::min<long>((768 + tiles - 1) / tiles, std::max(1, M / (32 * 16)));
  mps = ((M + splitk - 1) / splitk + 31) / 32 * 32;
  splitk = (M + mps - 1) / mps;
}

static int wh_bm(const ConvTNParams& p) { return p.Co % 128 == 0 ? 128 : 64; }

bool conv_wgrad_halo_supported(const ConvTNParams& p) {
  if (g_wh_mode <= 0) return false;
  if (p.KH != 3 || p.KW != 3 || p.stride != 1 || p.pad != 1 || p.OH != p.H || p.OW != p.W) return false;
  if (p.dy_lo == 0 || p.x_lo == 0 || p.C % 32 || p.Co % 64 || p.ldy != p.Co || p.ldx != p.C) return false;
  if (!(p.W == 8 || p.W == 16 || p.W == 32) || (p.OH * p.OW) % 32) return false;
  const long ab = (p.dy_lo + (long)p.M * p.ldy) * 2, bb = (p.x_lo + (long)p.B * p.H * p.W * p.ldx) * 2;
  return ab < (long)OOB_OFF && bb < (long)OOB_OFF;
}

int conv_wgrad_halo_splitk(int Co, int C, int M) {
  int splitk, mps;
  wh_split(Co, C, M, Co % 128 == 0 ? 128 : 64, splitk, mps);
  return splitk;
}

bool conv_wgrad_halo(ConvTNParams p, int K, hipStream_t s) {
  if (!conv_wgrad_halo_supported(p)) return false;
  const int bm = wh_bm(p);
  wh_split(p.Co, p.C, p.M, bm, p.splitk, p.m_per_split);
  if (p.splitk > 1 && p.part == nullptr) return false;
  if (g_wh_mode == 2) {
    if (bm == 128) launch_wh_w<128, 2>(p, K, s);
    else launch_wh_w<64, 2>(p, K, s);
  } else {
    if (bm == 128) launch_wh_w<128, 1>(p, K, s);
    else launch_wh_w<64, 1>(p, K, s);
  }
  if (p.splitk > 1) tn_fold(p.part, p.dw, p.dw_cs, K, p.splitk, (long)p.Co * p.R, s);
  return true;
}
