// Large-tile implicit-GEMM convolution for gfx950 (MI355X), LDS fed by the LDS-DMA path.
//
//   Y[m][n] = Σ_tap Σ_c  X[pixel(m) + (dh_tap, dw_tap)][c] · Wb[n][boff_tap + c]
//
// One "tap" = one (kh, kw) filter position; the GEMM's K loop walks taps × 64-channel chunks,
// so every K tile is 64 contiguous channels of ONE input pixel per row (a 128-B line) — the
// A tile of 256 output pixels is a per-row gather of 128-B lines, which the LDS-DMA
// (`global_load_lds_dwordx4`: per-lane global address, lane-linear LDS destination) moves
// straight into LDS without touching VGPRs. Out-of-image taps read a zero page, so every lane
// of every DMA is active (the destination is lane-linear: a masked lane would leave a hole).
//
// The tap table makes one kernel serve
//   forward : Wb = W[Co][KH][KW][Ci], taps (kh, kw), boff = (kh·KW + kw)·Ci
//   dgrad   : Wb = flipped/transposed copy Wt[Ci][KH][KW][Co] (conv_weight_flip_t), A = dY;
//             stride 1 = one full-correlation launch, stride s = s² parity classes (only the
//             taps that reach a class; class rows remapped into dX by out_s/out_ph/out_pw).
//
// Tiling: 256 × BN (BN = 256 or 128) × 64, 512 threads = 8 waves (2×4 or 4×2), wave tile
// 128×64 or 64×64 of v_mfma_f32_32x32x16_bf16; 2 LDS stages (128 / 96 KB ⇒ 1 block per CU),
// the DMA of tile k+1 in flight during the MFMAs of tile k (guide §5.5 T3+T4, minimum
// 2-phase form); XOR swizzle chunk ^= (row>>1)&7 applied on the DMA SOURCE address (the LDS
// image stays lane-linear) and on the fragment read ⇒ the 16 rows of a ds_read_b128 lane
// group hit 16 distinct 16-B bank slots (conflict-free). XCD-aware tile order (T1).
//
// The narrower register-staged tiles in conv_nt.hip stay in use where this one does not pay:
// channel counts that are not multiples of 64 (stems, DenseNet, LeNet, d_model 100), N < 128,
// and launches too small to fill 256 CUs with 1-block-per-CU tiles.
#include <stdlib.h>

#include "dls.h"
#include "gemm_common.h"

namespace {

constexpr int GL_BK = 64;  // channels per K tile (one 128-B line per row)

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_dst) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

template <int BN, int WM, int WN>
__global__ void __launch_bounds__(512) conv_gl_kernel(ConvGLParams p) {
  constexpr int BM = 256;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  static_assert(WM * WN == 8 && TM >= 1 && TN >= 1, "8 waves");
  constexpr int A_TILE = BM * GL_BK * 2, B_TILE = BN * GL_BK * 2;  // bytes
  constexpr int STAGE = A_TILE + B_TILE;
  constexpr int AI = BM / 64, BI = BN / 64;  // DMA instructions per wave per tile (8 rows each)
  constexpr int SW = TN * 32 + 8;            // epilogue slab row (bf16), 16-B padded
  constexpr int EPI = 8 * 32 * SW * 2;
  constexpr int SMEM = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (SGPR)
  const int tilesM = (p.M + BM - 1) / BM, tilesN = (p.N + BN - 1) / BN;
  const int per_client = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int client = bid / per_client;
  const int t = bid - client * per_client;
  const int m0 = (t / tilesN) * BM, n0 = (t % tilesN) * BN;
  const bf16_t* __restrict__ x = p.x + (long)client * p.x_cs;
  const bf16_t* __restrict__ w = p.w + (long)(client / p.rep) * p.w_cs;

  // ---- DMA source state. Loader row of instruction i: i·64 + wid·8 + (lane>>3), 16-B chunk
  // position lane&7 in LDS; it fetches logical chunk (lane&7) ^ swz(row) from global.
  const int lrow = lane >> 3;
  const int swz_ld = ((wid & 1) * 4 + (lrow >> 1)) & 7;  // ((i·64 + wid·8 + lrow) >> 1) & 7
  const int coff = ((lane & 7) ^ swz_ld) * 8;            // element offset of the fetched chunk
  long a_base[AI];
  int a_ih[AI], a_iw[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + i * 64 + wid * 8 + lrow;
    if (m < p.M) {
      const uint32_t b = fdiv((uint32_t)m, p.fd_ohw);
      const uint32_t rem = (uint32_t)m - b * (uint32_t)(p.OH * p.OW);
      const uint32_t oh = fdiv(rem, p.fd_ow);
      const uint32_t ow = rem - oh * (uint32_t)p.OW;
      a_base[i] = (long)b * p.H * p.W * p.C + coff;
      a_ih[i] = (int)oh * p.stride - p.pad_h;
      a_iw[i] = (int)ow * p.stride - p.pad_w;
    } else {
      a_base[i] = 0;
      a_ih[i] = -(1 << 28);  // never inside the image
      a_iw[i] = 0;
    }
  }
  const bf16_t* b_src[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = n0 + i * 64 + wid * 8 + lrow;
    b_src[i] = n < p.N ? w + (long)n * p.ldb + coff : nullptr;
  }
  const bf16_t* zero = p.zero + (lane & 7) * 8;

  auto stage = [&](int buf, int kt) {
    const int tap = kt / p.cchunks;  // wave-uniform scalar math
    const int c0 = (kt - tap * p.cchunks) * GL_BK;
    const int dh = p.tap_dh[tap], dw = p.tap_dw[tap];
    const int boff = p.tap_boff[tap] + c0;
    unsigned char* As = smem + buf * STAGE;
    unsigned char* Bs = As + A_TILE;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
      const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const bf16_t* src = ok ? x + a_base[i] + ((long)ih * p.W + iw) * p.C + c0 : zero;
      glds16(src, As + (i * 64 + wid * 8) * (GL_BK * 2));
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const bf16_t* src = b_src[i] ? b_src[i] + boff : zero;
      glds16(src, Bs + (i * 64 + wid * 8) * (GL_BK * 2));
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  const int wm0 = (wid / WN) * (TM * 32), wn0 = (wid % WN) * (TN * 32);
  // fragment rows are (multiple of 32) + (lane & 31) ⇒ swz(row) = ((lane & 31) >> 1) & 7
  const int swz_rd = (lane >> 1) & 7;
  const int frow = lane & 31, fh = lane >> 5;
  auto compute = [&](int buf) {
    const unsigned char* As = smem + buf * STAGE;
    const unsigned char* Bs = As + A_TILE;
#pragma unroll
    for (int ks = 0; ks < GL_BK / 16; ++ks) {
      const int chunk = ((ks * 2 + fh) ^ swz_rd) * 16;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + (wm0 + i * 32 + frow) * (GL_BK * 2) + chunk);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn0 + j * 32 + frow) * (GL_BK * 2) + chunk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = p.ntaps * p.cchunks;
  if (nk > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
      compute(cur);
      // the DMA of tile kt+1 must have landed (issuing waves' vmcnt, then the barrier) before any
      // wave reads it; the barrier also retires every wave's reads of stage `cur` before the
      // next iteration's DMA overwrites it
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // ---- epilogue: bias (+ReLU) → bf16 → per-wave 32-row LDS slab → 16-B coalesced stores
  bf16_t* __restrict__ y = p.y + (long)client * p.y_cs;
  const bf16_t* accp = p.acc ? p.acc + (long)client * p.y_cs : nullptr;
  const bf16_t* bias = p.bias ? p.bias + (long)(client / p.rep) * p.b_cs : nullptr;
  float bvals[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + j * 32 + frow;
    bvals[j] = (bias && n < p.N) ? bf2f(bias[n]) : 0.f;
  }
  bf16_t* slab = reinterpret_cast<bf16_t*>(smem) + wid * 32 * SW;
  const bool vec_ok = (p.N % 8) == 0;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float v = acc[i][j][e] + bvals[j];
        if (p.relu) v = fmaxf(v, 0.f);
        slab[((e & 3) + 8 * (e >> 2) + 4 * fh) * SW + j * 32 + frow] = f2bf(v);
      }
    }
    __syncthreads();
    for (int qd = lane; qd < 32 * TN * 4; qd += 64) {
      const int r = qd / (TN * 4), cc = (qd % (TN * 4)) * 8;
      const int m = m0 + wm0 + i * 32 + r, n = n0 + wn0 + cc;
      if (m >= p.M || n >= p.N) continue;
      long row = m;
      if (p.out_s > 1) {
        const uint32_t b = fdiv((uint32_t)m, p.fd_ohw);
        const uint32_t rem = (uint32_t)m - b * (uint32_t)(p.OH * p.OW);
        const uint32_t oh = fdiv(rem, p.fd_ow);
        const uint32_t ow = rem - oh * (uint32_t)p.OW;
        row = ((long)b * p.out_H + oh * p.out_s + p.out_ph) * p.out_W + ow * p.out_s + p.out_pw;
      }
      bf16_t* dst = y + row * p.N + n;
      const bf16_t* acc_row = accp ? accp + row * p.N + n : nullptr;
      const bf16_t* src = slab + r * SW + cc;
      if (vec_ok && n + 8 <= p.N) {
        uint4 v = *reinterpret_cast<const uint4*>(src);
        if (acc_row) v = add_bf16x8(v, *reinterpret_cast<const uint4*>(acc_row));
        *reinterpret_cast<uint4*>(dst) = v;
      } else {
        for (int q = 0; q < 8 && n + q < p.N; ++q) dst[q] = acc_row ? f2bf(bf2f(src[q]) + bf2f(acc_row[q])) : src[q];
      }
    }
    __syncthreads();
  }
}

// Wt[kw-row][ci][kh'][kw'][co] = W[kw-row][co][KH-1-kh'][KW-1-kw'][ci]: 64×64 (co × ci) tiles
// through LDS, 16-B loads and stores on both sides.
__global__ void __launch_bounds__(256) flip_t_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt, long w_cs,
                                                     int Co, int KH, int KW, int Ci) {
  __shared__ bf16_t tile[64][64 + 8];
  const int tilesC = (Ci + 63) / 64, tilesO = (Co + 63) / 64;
  int b = blockIdx.x;
  const int tc = b % tilesC;
  b /= tilesC;
  const int to = b % tilesO;
  b /= tilesO;
  const int tap = b % (KH * KW);
  const int row = b / (KH * KW);
  const int kh = tap / KW, kw = tap % KW;
  const int tapf = (KH - 1 - kh) * KW + (KW - 1 - kw);
  const bf16_t* src = w + (long)row * w_cs;
  bf16_t* dst = wt + (long)row * Co * KH * KW * Ci;
  const int tid = threadIdx.x;
  const bool vec = (Ci % 8 == 0) && (Co % 8 == 0);
  // load W[co][kh][kw][ci0..ci0+63]
  for (int q = tid; q < 64 * 8; q += 256) {
    const int r = q >> 3, c8 = (q & 7) * 8;
    const int co = to * 64 + r, ci = tc * 64 + c8;
    const bf16_t* s = src + (((long)co * KH + kh) * KW + kw) * Ci + ci;
    if (vec && co < Co && ci + 8 <= Ci) {
      const uint4 v = *reinterpret_cast<const uint4*>(s);
      const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
#pragma unroll
      for (int u = 0; u < 8; ++u) tile[r][c8 + u] = e[u];
    } else {
      for (int u = 0; u < 8; ++u) tile[r][c8 + u] = (co < Co && ci + u < Ci) ? s[u] : (bf16_t)0;
    }
  }
  __syncthreads();
  // store Wt[ci][tapf][co0..co0+63]
  for (int q = tid; q < 64 * 8; q += 256) {
    const int r = q >> 3, o8 = (q & 7) * 8;
    const int ci = tc * 64 + r, co = to * 64 + o8;
    if (ci >= Ci) continue;
    bf16_t* d = dst + ((long)ci * KH * KW + tapf) * Co + co;
    if (vec && co + 8 <= Co) {
      uint4 v;
      bf16_t* e = reinterpret_cast<bf16_t*>(&v);
#pragma unroll
      for (int u = 0; u < 8; ++u) e[u] = tile[o8 + u][r];
      *reinterpret_cast<uint4*>(d) = v;
    } else {
      for (int u = 0; u < 8 && co + u < Co; ++u) d[u] = tile[o8 + u][r];
    }
  }
}

const bf16_t* zero_page() {
  static bf16_t* z = nullptr;
  if (!z) {
    CHECK_HIP(hipMalloc(&z, 4096));
    CHECK_HIP(hipMemset(z, 0, 4096));
    CHECK_HIP(hipDeviceSynchronize());
  }
  return z;
}

int gl_bn(int N) { return N >= 256 ? 256 : 128; }

void launch_gl(ConvGLParams& p, int K, hipStream_t s) {
  p.zero = zero_page();
  p.fd_ohw = make_fastdiv((uint32_t)(p.OH * p.OW));
  p.fd_ow = make_fastdiv((uint32_t)p.OW);
  if (p.out_s == 0) p.out_s = 1;
  const int bn = gl_bn(p.N);
  const int grid = K * cdiv(p.M, 256) * cdiv(p.N, bn);
  if (bn == 256)
    hipLaunchKernelGGL((conv_gl_kernel<256, 2, 4>), dim3(grid), dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((conv_gl_kernel<128, 4, 2>), dim3(grid), dim3(512), 0, s, p);
}

// -1: shape heuristic; 0: never; 1: whenever the shape is supported (tests, A/B benchmarks)
int gl_mode() {
  return native_option(g_opt_conv_gl, "DLS_CONV_GL", -1);
}

}  // namespace

bool conv_gl_supported(int C, int N, int ntaps) { return C % 64 == 0 && N % 8 == 0 && N >= 64 && ntaps <= 9; }

bool conv_gl_wanted(int K, int M, int N, int C, int ntaps, int mode) {
  if (mode < 0) mode = gl_mode();
  if (mode == 0 || !conv_gl_supported(C, N, ntaps)) return false;
  if (mode > 0) return true;
  // 1 block per CU. Measured on the ResNet-18 shapes (bench/kernel_bench.py --gl, K = 100 and 13):
  // wins from ≈200 blocks up (l3 at K = 13, 208 blocks: fwd 872 vs 566 TFLOP/s), loses below
  // (l4 at K = 13, 104 blocks: 515 vs 564); the narrow N = 64 layers lose (the A tile then
  // dominates the traffic; conv_nt's 64×64 single-buffer tile at 4 blocks/CU: 435 vs 299)
  const long blocks = (long)K * cdiv(M, 256) * cdiv(N, gl_bn(N));
  return N >= 128 && blocks >= 192;
}

void conv_gl_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, const bf16_t* bias, long x_cs, long y_cs, long w_cs,
                 long b_cs, int K, int rep, int B, int H, int W, int C, int OH, int OW, int KH, int KW, int stride,
                 int pad, int N, int relu, hipStream_t s) {
  ConvGLParams p{};
  p.x = x;
  p.w = w;
  p.y = y;
  p.bias = bias;
  p.x_cs = x_cs;
  p.y_cs = y_cs;
  p.w_cs = w_cs;
  p.b_cs = b_cs;
  p.B = B;
  p.H = H;
  p.W = W;
  p.C = C;
  p.OH = OH;
  p.OW = OW;
  p.stride = stride;
  p.pad_h = p.pad_w = pad;
  p.M = B * OH * OW;
  p.N = N;
  p.ldb = KH * KW * C;
  p.ntaps = KH * KW;
  p.cchunks = C / GL_BK;
  for (int kh = 0; kh < KH; ++kh)
    for (int kw = 0; kw < KW; ++kw) {
      const int tp = kh * KW + kw;
      p.tap_dh[tp] = kh;
      p.tap_dw[tp] = kw;
      p.tap_boff[tp] = tp * C;
    }
  p.rep = rep;
  p.relu = relu;
  p.out_s = 1;
  launch_gl(p, K, s);
}

void conv_weight_flip_t(const bf16_t* w, bf16_t* wt, long w_cs, int Kw, int Co, int KH, int KW, int Ci,
                        hipStream_t s) {
  const long grid = (long)Kw * KH * KW * cdiv(Co, 64) * cdiv(Ci, 64);
  hipLaunchKernelGGL(flip_t_kernel, dim3(grid), dim3(256), 0, s, w, wt, w_cs, Co, KH, KW, Ci);
}

void conv_gl_dgrad(const bf16_t* dy, const bf16_t* wt, bf16_t* dx, const bf16_t* acc, int K, int rep, int B, int OH, int OW, int Co,
                   int H, int W, int Ci, int KH, int KW, int stride, int pad, hipStream_t s) {
  ConvGLParams p{};
  p.x = dy;
  p.w = wt;
  p.y = dx;
  p.bias = nullptr;
  p.acc = acc;
  p.x_cs = (long)B * OH * OW * Co;
  p.y_cs = (long)B * H * W * Ci;
  p.w_cs = (long)Ci * KH * KW * Co;
  p.B = B;
  p.H = OH;  // the GEMM's A image is dY
  p.W = OW;
  p.C = Co;
  p.N = Ci;
  p.ldb = KH * KW * Co;
  p.cchunks = Co / GL_BK;
  p.rep = rep;
  p.stride = 1;
  // dx pixel ih of class ph (ih = s·oh' + ph) receives taps kh ≡ (ph + pad) (mod s):
  // kh = kh0 + s·j, dy row = oh' + (ph + pad - kh0)/s - j; walking j downwards makes it a
  // stride-1 correlation over the class subgrid (stride 1: a single class, the full flip)
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
      ConvGLParams q = p;
      q.OH = Hc;
      q.OW = Wc;
      q.M = B * Hc * Wc;
      q.out_s = stride;
      q.out_ph = ph;
      q.out_pw = pw;
      q.out_H = H;
      q.out_W = W;
      q.pad_h = nkh - 1 - dh;
      q.pad_w = nkw - 1 - dw;
      q.ntaps = nkh * nkw;
      for (int a = 0; a < nkh; ++a)
        for (int b = 0; b < nkw; ++b) {
          // loop tap (a, b) reads dy (oh' - pad_h + a, ow' - pad_w + b) against kernel tap
          // kh = kh0 + s·(nkh-1-a) — i.e. the flipped kernel's row KH-1-kh in Wt
          const int kh = kh0 + stride * (nkh - 1 - a), kw = kw0 + stride * (nkw - 1 - b);
          const int tp = a * nkw + b;
          q.tap_dh[tp] = a;
          q.tap_dw[tp] = b;
          q.tap_boff[tp] = ((KH - 1 - kh) * KW + (KW - 1 - kw)) * Co;
        }
      if (q.ntaps == 0) q.pad_h = q.pad_w = 0;  // no tap reaches this class: dx = 0
      launch_gl(q, K, s);
    }
  }
}
