// Launch API of the gfx950 kernels (host side). All launches are asynchronous on the given
// stream and never allocate or synchronise, so they can be captured into hipGraphs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;

// Host-side launch knobs (A/B measurements, tests), one object instead of import-time globals:
// each starts UNSET and then takes its environment variable (or the default) on first use;
// set_native_option() — the Python RuntimeOptions (distributed_learning_simulator_amd/options.py)
// — overrides it at any time between launches. Defined in elementwise.hip.
constexpr int kOptUnset = -1000000;
extern int g_opt_attn_mfma, g_opt_conv_gl, g_opt_pl_min_wg;
extern int g_opt_halo_wgrad_unroll;  // conv_halo_wgrad.hip k-step unroll (1 or 2)
// halo fwd / dgrad tiles past the valid samples skip their work (ConvNTParams::skip_valid; env
// DLS_SKIP_INVALID, Python OPTIONS.skip_invalid)
extern int g_opt_halo_skip;
extern int g_opt_conv_pix;  // conv_pl.hip pixel-major tap skipping on small images (1 on)
int native_option(int& slot, const char* env, int dflt);
bool set_native_option(const char* name, int value);  // false: unknown name

// Division by a runtime-constant divisor without the ~40-instruction integer divide:
// q = (umulhi(n, mul) + n) >> shift, exact for 0 <= n < 2^31 (host precomputes mul/shift).
struct FastDiv {
  uint32_t d, mul, shift;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1u << s) < d) ++s;
  f.shift = s;
  f.mul = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << s) - d)) / d + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.mul) + n) >> f.shift;
}

struct ConvNTParams {
  const bf16_t* x;  // A source image [K][B][H][W][C]
  const bf16_t* w;  // B rows [N][R] per weight row
  bf16_t* y;        // [K][M][N]
  const bf16_t* bias;
  const bf16_t* acc;   // optional [K][rows][N] (y layout) added to the result in the epilogue
  // acc_compact (stride-s dgrad parity class (0, 0) only): acc holds the class grid compactly —
  // GEMM row m reads acc row m (client stride acc_cs), not the dx pixel it writes. A 1x1 stride-s
  // downsample shortcut's input gradient lives only on that grid (ResNet blocks)
  long acc_cs;
  int acc_compact;
  // optional ReLU bits [K][rows][N/8] (contiguous rows, ldy == N) gating acc: y = gemm + acc·bit
  const uint8_t* acc_mask;
  const bf16_t* gate;  // optional, y layout: result zeroed where gate <= 0 (ReLU' of the next layer's input)
  long x_cs, y_cs, w_cs, b_cs;
  int B, H, W, C;
  int OH, OW, KH, KW, stride, pad, dil;
  int pad_w;  // horizontal padding (conv_nt() sets pad_w = pad for plain launches)
  int M, N, R;
  int rep;
  int relu;
  int b_kmajor;  // 1: B read from a forward conv weight [Co=C][wKH][wKW][Ci=N] (dgrad)
  // dgrad tap mapping (b_kmajor): loop tap kh2 ∈ [0,KH) reads weight row kh = kh_off - kh_step·kh2
  int wKH, wKW, kh_off, kh_step, kw_off, kw_step;
  // output row remap (sub-pixel dgrad): GEMM row (b, oh, ow) → dx pixel (oh·out_s+out_ph, ow·out_s+out_pw)
  int out_s, out_ph, out_pw, out_H, out_W;
  FastDiv fd_ohw, fd_ow, fd_kwc, fd_c;  // filled by conv_nt()
  // 1: every tensor pointer above is fp32 (reference precision); the GEMM runs as split-bf16
  // ("bf16x3") on the MFMA with fp32 accumulation (conv_f32.hip)
  int f32;
  // channel strides of channel-sliced views (DenseNet's preallocated block buffer): A pixel
  // stride ldx (0 = C), output / acc / gate row stride ldy (0 = N)
  int ldx, ldy;
  // optional BN statistics of the output (fp32 kernels): per 32-row group g and column n,
  // stats[client][g][0][n] = Σ y, stats[client][g][1][n] = Σ y² over the rows of valid samples
  // (row < stats_valid[client]·OH·OW) — the [K][parts][2N] partial layout bn_fwd consumes
  // (parts = cdiv(M, 32)), so BN skips its own statistics pass over y
  float* stats;
  const int* stats_valid;  // [K] valid samples per client (nullptr: all rows)
  // epilogue scale / dropout (Transformer training): v = out_scale·(acc·W + bias) (0 = 1); with
  // drop_p > 0, v = keep(k, m, n) ? v / (1 − drop_p) : 0 before the residual add, where
  // keep = mix32(m·N + n, drop_seeds[k]) ≥ drop_p·2³² (same rule as ops: dropout_apply)
  const uint32_t* drop_seeds;
  float drop_p;
  float out_scale;
  // optional pre-split weight planes (fp32 kernels): the B operand's bf16 hi plane in w's layout,
  // the lo plane ws_plane elements after it, client stride ws_cs (elements). Kept current by the
  // SGD kernel (sgd_step's `split`), so the GEMM skips splitting B in every workgroup.
  const bf16_t* wsplit;
  long ws_cs, ws_plane;
  // optional pre-split A operand (fp32 kernels, conv_pl.hip): x is then the bf16 hi plane of the
  // activation (same element layout as the fp32 tensor, client stride x_cs in bf16 elements)
  // and its lo plane starts x_lo elements after it (0 = A is an fp32 tensor). Written by the
  // producing BatchNorm (bn_fwd / bn_bwd planes outputs): with wsplit the GEMM moves both
  // operands HBM → LDS by LDS-DMA and spends no VALU on the split.
  long x_lo;
  // optional BN-backward partials (fp32 stride-1 dgrad whose dX is the dY of a BatchNorm with
  // input bnb_x [K][M][N] at row stride bnb_xld (0 = N; a channel prefix of DenseNet's block
  // buffer), statistics bnb_mean / bnb_rstd [K][N] and ReLU gate: the 1-bit mask bnb_mask
  // [K][M][N/8], else the fp32 output bnb_y (dX layout, > 0), else none): per 32-row group g and
  // column n, bnb[client][g][0][n] = Σ ĝ and bnb[client][g][1][n] = Σ ĝ·x̂ over rows <
  // bnb_valid[client] (ĝ = dX·relu', x̂ = (x − μ)·rstd) — the [K][parts][2N] layout
  // bn_bwd(pre_part) consumes, so BN skips its reduction pass over dY
  float* bnb;
  const float* bnb_x;
  long bnb_xld;
  const float* bnb_y;
  const uint8_t* bnb_mask;
  const float* bnb_mean;
  const float* bnb_rstd;
  const int* bnb_valid;
  // optional BatchNorm(+ReLU) applied to the A operand while it is staged (conv_halo.hip forward,
  // fp32): the layer input is then bn_x, the RAW output of the previous conv [K][B][H][W][C] fp32
  // (client stride bn_x_cs floats), and the GEMM reads relu?(bn_coef[k][c][0]·x + bn_coef[k][c][1])
  // — the BN's (scale, shift) pairs — zero outside the image and past bn_valid[k] rows; no
  // normalised activation is ever written
  const float* bn_x;
  long bn_x_cs;
  const float* bn_coef;
  int bn_relu;
  const int* bn_valid;
  // (training) the normalised activation's split planes [K][2][R][C] and ReLU bit mask [K][R][C/8],
  // written by the first N tile of each row block from the values it stages — what the BN apply
  // pass would have written for the conv's weight gradient and the BN's backward
  bf16_t* bn_yp;
  uint8_t* bn_mask;
  // (DenseNet channel prefix, bn_c > 0) bn_x rows at stride ldx inside the block buffer, only the
  // first bn_c ≤ C channels real (C: the 32-padded chunking of the weight rows; the rest stage as
  // zero); training writes the normalised activation in fp32 to bn_y (row stride bn_ldy, client
  // stride bn_y_cs) — the tensor the weight gradient and the BN backward read
  int bn_c;
  float* bn_y;
  long bn_y_cs;
  int bn_ldy;
  // optional (halo kernels): a row block whose first GEMM row is ≥ skip_valid[client]·skip_mul
  // holds only rows past the client's valid samples — no MFMA work: the workgroup writes zero
  // epilogue partials (stats / bnb) and leaves its output rows unwritten. Only for outputs whose
  // every reader stops at the valid rows (BatchNorm passes; ops.hip decides)
  const int* skip_valid;
  int skip_mul;
  // optional split planes of the fp32 output (NT epilogue, f32): hi plane at yp (y's element
  // layout, client stride yp_cs elements), lo plane yp_lo elements after it — the operand form of
  // the plane GEMMs that read this output (Transformer h, linear dgrads)
  bf16_t* yp;
  long yp_cs, yp_lo;
  // pixel-major GEMM rows (conv_pl.hip, set by conv_nt_pl for small images): GEMM row m is image
  // m % B at pixel m / B — a 32-row group then holds one pixel, so the K walk visits only the taps
  // that land inside the image for some row of the tile and a wave skips the MFMAs of groups
  // whose pixel the tap misses (4x4 images, 3x3 taps: 100 of 144 tap-pixels are inside)
  int pix;
  FastDiv fd_pb;
};

// BN-backward partial request handed to conv_dgrad (see ConvNTParams::bnb)
struct BNBwdPartials {
  float* part;
  const float* x;
  long xld;
  const float* y;
  const uint8_t* mask;
  const float* mean;
  const float* rstd;
  const int* valid;
};

// DenseNet growth-conv weight gradient with LDS halo reuse (conv_dense_wgrad.hip): dy [K][M][ldy]
// (the growth channels of the block gradient), y [K][M][C] (the normalised prefix), dw rows
// [N][3][3][C] at client stride dw_cs; part: nchunks·G per-workgroup slabs per client
struct DenseWgradParams {
  const float* dy;
  long dy_cs;
  int ldy;
  const float* y;
  long y_cs;
  float* dw;
  long dw_cs;
  float* part;
  int K, B, H, W, C, N, nchunks, G;
  // bn_sc set: y is recomputed while staged from the raw prefix (y = x at row stride ldy_x, client
  // stride y_cs) as relu(fmaf(x, scale, shift)) with the forward's BN [K][C][2] (scale, shift) —
  // bitwise the activation the forward would have stored; rows past valid_rows[k] are zeros
  const float* bn_sc;
  int ldy_x;
  const int* valid_rows;
};

// DenseNet growth-conv input gradient fused with its BatchNorm backward (conv_dense_dgrad.hip):
// dy [K][B·H·W][ldy] the growth channels of the block gradient, w [Kw][N][3][3][C] (client k reads
// w + (k / rep)·w_cs), x / dx the block buffer's prefix and its gradient ([K][B·H·W][ldx], client
// stride x_cs, dx += the BN input gradient), the ReLU gate (the forward's BN scale / shift applied to
// x, else mask [K][R][C/8] bits, else y [K][R][C] > 0), mean /
// rstd [K][C] the forward statistics. part / coef / G / nchunks are set by dense_dgrad_bn.
struct DenseDgradParams {
  const float* dy;
  long dy_cs;
  int ldy;
  const float* w;
  long w_cs;
  int rep;
  const float* x;
  float* dx;
  long x_cs;
  int ldx;
  const uint8_t* mask;
  const float* y;
  const float* bn_sc;  // [K][C][2] the forward's (scale, shift): gate fmaf(x, scale, shift) > 0 (else mask / y)
  const float* mean;
  const float* rstd;
  const int* valid_rows;
  const float* coef;
  float* part;
  int K, B, H, W, C, N, G, nchunks;
};

// 3x3 / stride-1 / pad-1 weight gradient with LDS halo reuse (conv_halo_wgrad.hip): dy [K][B·H·W][ldy]
// (N channels) and x [K][B][H][W][ldx] (C channels), each as bf16 planes (lo plane *_lo elements
// after the hi plane, client strides in bf16 elements) or fp32 (client strides in floats); dw rows
// [N][3][3][C] at client stride dw_cs (16-B aligned); part: halo_wgrad_part_floats slabs
// The optimiser step applied where a weight gradient is produced (the SGD "epilogue": the wgrad
// kernels' direct stores or their split folds), instead of storing dW for a separate sgd_step
// pass: per element of client k (when active[k]) the sgd_kernel arithmetic — g += wd·θ;
// m = first[k] ? g : μ·m + (1 − dampening)·g; g = nesterov ? g + μ·m : m; θ −= lr[k]·g — and
// the new θ's split planes. theta == nullptr: off (dW stored). Element e of client k lives at
// theta[k·th_cs + e], mom[k·th_cs + e], split[k·sp_cs + e] (hi) / + sp_lo (lo).
struct SgdEpi {
  float* theta;
  float* mom;
  bf16_t* split;
  long th_cs, sp_cs, sp_lo;
  const float* lr;
  const uint8_t* active;
  const uint8_t* first;
  float wd, momentum, dampening;
  int nesterov;
};
// (passed with each conv_tn / halo_wgrad launch: bindings.cpp sgd_arg)

struct HaloWgradParams {
  const void* dy;
  long dy_cs, dy_lo;
  int ldy;
  const void* x;
  long x_cs, x_lo;
  int ldx;
  // (x mode 2) BatchNorm(+ReLU) applied while staging: coef [K][C][2] (scale, shift); rows (pixels)
  // of samples past x_valid[k] (nullptr: none) read as zero, like the padding
  const float* coef;
  int relu;
  const int* x_valid;
  // optional [K] valid samples: tiles of later images (zero dY and X: the BN passes wrote zeros
  // there) are skipped — the pixel groups split the valid images' tiles only
  const int* valid_img;
  // (dy mode 2) dY is the input gradient of a BatchNorm(+ReLU) whose OUTPUT gradient dy holds
  // (fp32): dY = r < bb_valid[k] ? fmaf(a, relu' ? dy : 0, fmaf(e, bb_x, d)) : 0 — bn_bwd_apply's
  // arithmetic — with bb_coef [K][N][3] = (a, d, e), relu' from the bits bb_mask [K][rows][N / 8]
  // (nullptr: no gate) and bb_x the BN's raw input (rows at stride ldy). The c-block-0 workgroups
  // also store dY's split planes at bb_dxp ([K][2][rows][N]) for the dgrad — zeros for skipped images
  const float* bb_x;
  const uint8_t* bb_mask;
  const float* bb_coef;
  const int* bb_valid;
  bf16_t* bb_dxp;
  float* dw;
  long dw_cs;
  float* part;
  int K, B, H, W, C, N;
  int nblk, cblk, G;  // (filled by halo_wgrad)
  SgdEpi sgd;         // (theta != nullptr: step the weights instead of storing dW)
};
bool halo_wgrad_supported(int B, int H, int W, int C, int N);
long halo_wgrad_part_floats(int K, int B, int H, int W, int C, int N);
// xm: 0 x planes, 1 x fp32, 2 x fp32 + BN(+ReLU); dm: 0 dy planes, 1 dy fp32, 2 BN backward of an
// fp32 dy (bb_*). false: not served
bool halo_wgrad(HaloWgradParams p, int xm, int dm, hipStream_t s);

struct ConvTNParams {
  const bf16_t* dy;  // [K][M][Co]
  const bf16_t* x;   // [K][B][H][W][C]
  float* dw;         // [K] rows (stride dw_cs) of [Co][R]
  long dy_cs, x_cs, dw_cs;
  int B, H, W, C, OH, OW, KH, KW, stride, pad;
  int M, Co, R;
  int splitk, m_per_split;
  FastDiv fd_ohw, fd_ow;  // filled by conv_tn()
  int f32;                // 1: dy / x are fp32 (split-bf16 GEMM, conv_f32.hip)
  int ldy, ldx;           // dy row stride (0 = Co), x pixel stride (0 = C): channel-sliced views
  // deterministic split-K: with splitk > 1 and part != nullptr every split writes its own fp32
  // slab part[(split·K + client)·Co·R + co·R + r] (plain stores, no atomics, no pre-zeroed dw)
  // and a fold pass sums the slabs in split order into dw — bitwise-reproducible weight
  // gradients (the launchers run the fold; part holds splitk·K·Co·R floats)
  float* part;
  // pre-split operands (conv_pl.hip): dy / x are bf16 hi planes, lo planes dy_lo / x_lo
  // elements after them (0 = fp32 tensors); client strides dy_cs / x_cs in bf16 elements
  long dy_lo, x_lo;
  SgdEpi sgd;  // (pre-split launches only: step the weights instead of storing dW)
  // (conv_pl.hip, set by conv_tn_pl for small images) the pixel reduction walks (pixel, 32-image
  // chunk) pairs over only the pixels the workgroup's tap lands inside the image for
  int pix;
};

// Large-tile conv GEMM fed by the LDS-DMA (conv_gl.hip): K loop over a tap table × 64-channel
// chunks (C % 64 == 0); A pixel of GEMM row (b, oh, ow) and tap t is
// (oh·stride − pad_h + tap_dh[t], ow·stride − pad_w + tap_dw[t]); B row n starts at n·ldb, the
// tap's 64-channel chunk at tap_boff[t] + c0. Output rows remapped as in ConvNTParams.
struct ConvGLParams {
  const bf16_t* x;
  const bf16_t* w;
  bf16_t* y;
  const bf16_t* bias;
  const bf16_t* acc;   // optional, y layout: added to the result in the epilogue
  const bf16_t* zero;  // ≥ 128 B of zeros: the DMA source of out-of-image taps (filled by the launcher)
  long x_cs, y_cs, w_cs, b_cs;
  int B, H, W, C;  // A image
  int OH, OW;      // GEMM row grid
  int stride, pad_h, pad_w;
  int M, N, ldb, ntaps, cchunks;
  int tap_dh[9], tap_dw[9], tap_boff[9];
  int rep, relu;
  int out_s, out_ph, out_pw, out_H, out_W;
  FastDiv fd_ohw, fd_ow;
};
bool conv_gl_supported(int C, int N, int ntaps);
// mode: -1 heuristic (env DLS_CONV_GL overrides), 0 never, 1 whenever supported
bool conv_gl_wanted(int K, int M, int N, int C, int ntaps, int mode);
void conv_gl_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, const bf16_t* bias, long x_cs, long y_cs, long w_cs,
                 long b_cs, int K, int rep, int B, int H, int W, int C, int OH, int OW, int KH, int KW, int stride,
                 int pad, int N, int relu, hipStream_t s);
// Wt[row][ci][kh'][kw'][co] = W[row][co][KH-1-kh'][KW-1-kw'][ci] (dgrad B operand, k-contiguous)
void conv_weight_flip_t(const bf16_t* w, bf16_t* wt, long w_cs, int Kw, int Co, int KH, int KW, int Ci,
                        hipStream_t s);
void conv_gl_dgrad(const bf16_t* dy, const bf16_t* wt, bf16_t* dx, const bf16_t* acc, int K, int rep, int B, int OH, int OW, int Co,
                   int H, int W, int Ci, int KH, int KW, int stride, int pad, hipStream_t s);

// variant < 0: shape heuristic; 0..conv_nt_num_variants()-1: explicit tile config (benchmarks)
void conv_nt(ConvNTParams p, int K, int variant, hipStream_t s);
int conv_nt_num_variants();
int conv_nt_default_variant(int M, int N, int R, int b_kmajor);
// dX of a conv (any stride): stride-1 → one flipped-weight NT GEMM; stride s > 1 → s² parity
// classes, each a dense stride-1 GEMM over only the taps that reach it (no dilation zeros).
void conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const bf16_t* acc, long w_cs, int K, int rep, int B, int OH, int OW,
                int Co, int H, int W, int Ci, int KH, int KW, int stride, int pad, int variant, int f32, hipStream_t s,
                int ld_dy = 0, long dy_cs = 0, const bf16_t* wsplit = nullptr, long ws_cs = 0, long ws_plane = 0,
                long x_lo = 0, int acc_compact = 0,  // x_lo: dy is the hi plane of pre-split planes (ConvNTParams::x_lo)
                const BNBwdPartials* bnb = nullptr,  // (fp32, stride 1, Ci % 4 == 0)
                // wt_buf (fp32 planes, 3x3 stride-1 pad-1, 32-channel multiples): scratch of (K / rep)·2·9·Ci·Co
                // bf16 for the transposed flipped weight planes — the dgrad then runs the forward tiles
                bf16_t* wt_buf = nullptr,
                // acc_mask: bits [K][rows][Ci / 8] gating acc (acc · bit): the identity shortcut's
                // gradient dy·relu' from the block output's gradient and ReLU mask, never stored
                const uint8_t* acc_mask = nullptr,
                int wt_ready = 0);  // wt_buf already holds the transposed planes (wt_planes)
// the transposed flipped weight planes of a 3x3 dgrad (conv_dgrad wt_buf), built ahead of the dgrad
void wt_planes(const bf16_t* wsplit, long ws_cs, long ws_plane, bf16_t* wt, int Kw, int Co, int Ci, hipStream_t s);
void conv_tn(ConvTNParams p, int K, int variant, hipStream_t s);
int conv_tn_num_variants();
// split-K factor the launch will use (callers zero the gradient rows first when > 1)
int conv_tn_splitk(int K, int Co, int R, int M, int C, int variant, int f32, int ldy = 0, int ldx = 0,
                   int planes = 0);  // planes: the pre-split launch (conv_tn_pl_splitk, its own variant ids)
// fp32 (split-bf16 MFMA) GEMMs, conv_f32.hip; reached through conv_nt / conv_tn with p.f32 = 1
void conv_nt_f32(const ConvNTParams& p, int K, int variant, hipStream_t s);
int conv_nt_f32_num_variants();
void conv_tn_f32(ConvTNParams p, int K, int variant, hipStream_t s);
// pre-split operand planes (conv_pl.hip): false when the shape is outside the kernels' contract
bool conv_nt_pl_supported(const ConvNTParams& p);
bool conv_nt_pl(const ConvNTParams& p, int K, int variant, hipStream_t s);
int conv_nt_pl_num_variants();
int conv_nt_pl_variant();           // -1: shape heuristic (set by benchmarks)
void conv_nt_pl_set_variant(int v);
// 3x3 stride-1 split-plane conv with LDS halo reuse (conv_halo.hip): false = shape not covered
bool conv_halo(const ConvNTParams& p, int K, hipStream_t s);
// 3x3 / stride-1 / pad-1 fp32 forward whose input is a BatchNorm(+ReLU) of the raw tensor x,
// applied in the halo loader (ConvNTParams::bn_*); false: shape outside the halo kernels (the
// caller applies the BN and runs the plain conv)
bool conv_halo_bn_supported(int B, int H, int W, int C, int N);
// BN forward (scale, shift) coefficients of the first C channels from running fp64 sums
// [K][2][ldp] (client stride sums_cs), no pass over the input
void bn_coef_sums(const double* sums, long sums_cs, int ldp, const float* gamma, const float* beta,
                  const int* valid_rows, long g_cs, int K, int R, int C, float eps, int rep, float* mean, float* rstd,
                  float* coef, hipStream_t s);
// running fp64 channel sums of a DenseNet block: out[k·out_cs + j·ldo + c] = Σ_p part[k][p][j][c]
// (part [K][nparts][2][g] fp32 conv-epilogue partials; 2·g ≤ 1024)
void part_sum_f64(const float* part, int K, int nparts, int g, double* out, long out_cs, int ldo, hipStream_t s);
// fp64 Σx, Σx² of the C channels of x [K][R rows at stride ldx] over each client's first valid[k]
// rows → out[k·out_cs + j·ldo + c] (j = 0: Σx, 1: Σx²); ws: chan_sums_f64_ws(R, C) doubles per
// client; 2·C ≤ 1024
long chan_sums_f64_ws(int R, int C);
void chan_sums_f64(const float* x, long x_cs, int ldx, int K, int R, int C, const int* valid, double* ws, double* out,
                   long out_cs, int ldo, hipStream_t s);
// BN apply with precomputed (scale, shift) coefficients (bn_fwd coef_out) → split planes (+ ReLU bits)
// and / or the fp32 output y
void bn_apply_only(const float* x, const float* coef, const int* valid_rows, int K, int R, int C, int relu,
                   bf16_t* yp, uint8_t* rmask, hipStream_t s, float* y = nullptr);
bool conv_halo_bn_fwd(const float* x, long x_cs, const float* coef, int relu, const int* valid_rows,
                      const bf16_t* wsplit, long ws_cs, long ws_plane, int rep, float* y, long y_cs, int K, int B,
                      int H, int W, int C, int N, float* stats, const int* stats_valid, hipStream_t s,
                      bf16_t* yp = nullptr, uint8_t* mask = nullptr);
// DenseNet growth conv: BN(+ReLU) of the first creal channels of the block buffer x (row stride
// ldx) applied in the halo loader; coef [K][C][2] and the weight planes [N][3][3][C] padded to C =
// 32·⌈creal/32⌉ channels (zero); y rows at stride ldy (the block buffer's new channels); ny
// (optional, training): the normalised activation [K][B·H·W][ldny] fp32, mask (optional, with ny,
// creal % 8 == 0): its ReLU bits [K][B·H·W][ldny / 8]
bool conv_halo_bn_dense_supported(int B, int H, int W, int C, int N);
bool conv_halo_bn_dense_fwd(const float* x, long x_cs, int ldx, int creal, const float* coef, int relu,
                            const int* valid_rows, const bf16_t* wsplit, long ws_cs, long ws_plane, int rep, float* y,
                            long y_cs, int ldy, int K, int B, int H, int W, int C, int N, float* stats,
                            const int* stats_valid, float* ny, long ny_cs, int ldny, uint8_t* mask, hipStream_t s);
bool dense_dgrad_supported(int B, int H, int W, int C, int N);
long dense_dgrad_ws_floats(int K, int B, int H, int C);
bool dense_dgrad_bn(DenseDgradParams p, const float* gamma, long g_cs, float* dgamma, float* dbeta, long dg_cs,
                    float* ws, hipStream_t s);
// BN-backward coefficients (a, d, e per channel, [K][C][3]) + dγ / dβ from [K][nparts][2][C] partial
// sums Σĝ / Σĝx̂ (norm.hip)
void bn_bwd_coef_parts(const float* part, int nparts, const float* gamma, long g_cs, const int* valid_rows,
                       const float* mean, const float* rstd, int K, int R, int C, float* coef, float* dgamma,
                       float* dbeta, long dg_cs, hipStream_t s);
bool dense_wgrad_supported(int B, int H, int W, int C, int N);
long dense_wgrad_part_floats(int K, int B, int H, int W, int C);
bool dense_wgrad(const float* dy, long dy_cs, int ldy, const float* y, long y_cs, float* dw, long dw_cs, float* part,
                 int K, int B, int H, int W, int C, int N, hipStream_t s, const float* bn_sc = nullptr,
                 int ldy_x = 0, const int* valid_rows = nullptr);
void conv_halo_set_mode(int m);  // -1 shape rule, 0 never, 1 whenever supported
void conv_halo_set_variant(int v);  // -1 default, 0..2 pipeline / tile variant (benchmarks)
bool conv_tn_pl_supported(const ConvTNParams& p);
bool conv_tn_pl(ConvTNParams p, int K, int variant, hipStream_t s);
int conv_tn_pl_num_variants();
int conv_tn_pl_variant();
void conv_tn_pl_set_variant(int v);
// split-K factor of the pre-split wgrad launch (callers size ConvTNParams::part with it)
int conv_tn_pl_splitk(int K, int Co, int R, int M, int variant);
// dw[k][i] = Σ_s part[(s·K + k)·CoR + i] in split order (deterministic split-K fold)
void tn_fold(const float* part, float* dw, long dw_cs, int K, int splitk, long CoR, hipStream_t s,
             const SgdEpi* sgd = nullptr);
int conv_tn_f32_num_variants();
int conv_tn_f32_splitk(int K, int Co, int R, int M, int gco, int gc, int variant);

// ---------------------------------------------------------------- normalisation
// Activation / γ / β pointers are the compute dtype: bf16 (f32 = 0) or fp32 (f32 = 1, the
// reference precision); statistics, coefficients and parameter gradients are always fp32.
long bn_workspace_floats(int K, long R, int C);  // ws size for bn_fwd / bn_bwd
void bn_fwd(const void* x, const void* gamma, const void* beta, const void* res, void* y, float* mean, float* rstd,
            const int* valid_rows, long g_cs, int K, int R, int C, int relu, float eps, int rep, float* ws,
            uint8_t* relu_mask, int f32, hipStream_t s,
            int ldx = 0, const float* pre_part = nullptr,
            int pre_nparts = 0, bf16_t* yp = nullptr,
            int y_f32 = 1, float* coef_out = nullptr, int apply = 1,
            const float* res_coef = nullptr);  // res_coef [K][C][2]: res is a second BN's raw input, applied here; yp / y_f32: split planes of y (fp32 only) with or without y; relu_mask: optional [K][R][C/8] bits out; ldx: row stride of x / res (channel slice of a wider buffer), y
                                  // contiguous; pre_part: [K][pre_nparts][2C] Σx / Σx² partials from the
                                  // producing conv's epilogue (ConvNTParams::stats) — no statistics pass
void bn_bwd(const void* dy, const void* x, const void* y, const float* mean, const float* rstd, const void* gamma,
            const int* valid_rows, long g_cs, int K, int R, int C, int relu, void* dx, void* dpre, float* dgamma,
            float* dbeta, long dg_cs, float* ws, const uint8_t* relu_mask, int f32,
            hipStream_t s, int ldx = 0,
            int acc_dx = 0, bf16_t* dxp = nullptr,
            int dx_f32 = 1,  // dxp / dx_f32: split planes of dX (fp32, contiguous) with or without dX; relu_mask (from bn_fwd) replaces reading y for the ReLU gate; x / dx at row
                             // stride ldx, acc_dx: dx += (DenseNet block-buffer gradient)
            const float* pre_part = nullptr,  // [K][pre_nparts][2C] Σĝ / Σĝx̂ partials from the dgrad
            int pre_nparts = 0,               // epilogue that produced dy (ConvNTParams::bnb): no reduction pass
            float* coef_ext = nullptr,        // [K][C][3] (a, d, e) kept for a later stage instead of ws
            int stage = 0);                   // 0 coefficients + apply, 1 coefficients only, 2 apply only
void ln_fwd(const void* x, const void* gamma, const void* beta, void* y, float* mean, float* rstd, long g_cs, int K,
            long rows_per_client, int C, float eps, int rep, int f32, hipStream_t s,
            bf16_t* yp = nullptr);  // yp (fp32): y's split planes [K][2][rows][C] as well
void ln_bwd(const void* dy, const void* x, const float* mean, const float* rstd, const void* gamma, long g_cs, int K,
            long rows_per_client, int C, void* dx, float* dgamma, float* dbeta, long dg_cs, float* ws, int f32,
            hipStream_t s);
long col_sum_workspace_floats(int K, long rows, int C);
long ln_workspace_floats(int K, long rows_per_client, int C);
void col_sum(const void* x, float* out, long out_cs, int K, long rows, int C, int f32, hipStream_t s,
             float* ws = nullptr);

// ------------------------------------------------------------------- elementwise
void pool_fwd(const void* x, void* y, int* idx, int K, int B, int H, int W, int C, int OH, int OW, int k, int stride,
              int pad, int mode, int f32, hipStream_t s);
void pool_bwd(const void* dy, const int* idx, void* dx, int K, int B, int H, int W, int C, int OH, int OW, int k,
              int stride, int pad, int mode, int f32, hipStream_t s);
void gap_fwd(const void* x, void* y, int KB, int HW, int C, int f32, hipStream_t s);
void gap_bwd(const void* dy, void* dx, int KB, int HW, int C, int f32, hipStream_t s);
void ce_fwd_bwd(const void* logits, const int* labels, const int* valid, float* loss, float* correct, void* dlogits,
                int K, int B, int NC, int f32, hipStream_t s, float* rowbuf = nullptr);  // rowbuf [2][K][B]: deterministic row-order loss / correct sums
void relu_bwd(const void* dy, const void* y, void* dx, long n, int f32, hipStream_t s);

// ------------------------------------------------------------- FL / optimiser
// ---------------------------------------------------------------- compressed payloads (compress.hip)
// Pack per-(client, tensor) b-bit codes (bits[k][s] ∈ [0, 8], 0 = tensor not sent) of rows x
// [K][ld] into the ragged wire buffer out (client k at row_off[k], tensor s at seg_byte_off[k][s]);
// stochastic rounding (seeds[k]) or round-to-nearest. Unpack to dense rows, or fused into the
// fp64 server accumulator acc[i] += Σ_k w[k]·x̂_k[i]. P = padded flat size (multiple of 8).
void quant_pack(const float* x, long ld, const int* seg, const int64_t* seg_off, const int64_t* seg_numel,
                const uint8_t* bits, const float* lo, const float* scale, const int64_t* seg_byte_off,
                const int64_t* row_off, int K, int nseg, long P, int stochastic, const uint32_t* seeds, uint8_t* out,
                hipStream_t s);
void quant_unpack(const uint8_t* codes, const int* seg, const int64_t* seg_off, const int64_t* seg_numel,
                  const uint8_t* bits, const float* lo, const float* scale, const int64_t* seg_byte_off,
                  const int64_t* row_off, int K, int nseg, long P, float* out, long ld, hipStream_t s);
void quant_unpack_acc(const uint8_t* codes, const int* seg, const int64_t* seg_off, const int64_t* seg_numel,
                      const uint8_t* bits, const float* lo, const float* scale, const int64_t* seg_byte_off,
                      const int64_t* row_off, int K, int nseg, long P, const double* w, double* acc, hipStream_t s);

// out[k][r][c] = keep(k, r, c) ? x·scale : 0 over [K][rows][N] (row stride ld), the dropout rule of
// the GEMM epilogue; seeds [K]. f32: fp32 (else bf16) tensors.
void dropout_apply(const void* x, void* out, int K, long rows, int N, long ld, const uint32_t* seeds, float p,
                   float scale, int f32, hipStream_t s);
// dropout_apply on contiguous fp32 writing the split planes [K][2][rows][N] (+ fp32 unless out null);
// colsum (with ws, dropout_planes_ws_floats): also the column sums of the output [K][N] at client
// stride colsum_cs (the consuming linear's bias gradient), folded in a fixed order
long dropout_planes_ws_floats(int K, long rows, int N);
void dropout_planes(const float* x, float* out, bf16_t* yp, int K, long rows, int N, const uint32_t* seeds, float p,
                    float scale, hipStream_t s, float* colsum = nullptr, long colsum_cs = 0, float* ws = nullptr);
// out[k][c] (client stride out_cs) = Σ_i part[k][i][c] in order (part [K][nparts][C]; norm.hip)
void fold_col_partials(const float* part, int nparts, int C, float* out, long out_cs, int K, hipStream_t s);

// procedural synthetic images (data/datasets.py, bit-identical to the torch generator): out [n][npix/C·Cout]
void synth_images(const int64_t* idx, long n, long npix, int C, int Cout, const int* source, const float* proto,
                  unsigned long long salt, float sqrt6, float noise, float* out, hipStream_t s);

// ---------------------------------------------------------------- graph (graph.hip)
// Federated-GNN neighbour sampling: per frontier row (nodes[t] expanded for client clients[t])
// the `fanout` (<= 32) in-neighbours with the smallest hash keys; out_nbr [n][fanout] (-1 pad).
// seed_h = hmix(step seed) (data/graph.py). rowptr / col: int32 in-neighbour CSR, owner [N]
// client id of each training node (-1 otherwise), is_val [N].
void neighbor_sample(const int* rowptr, const int* col, const int* owner, const uint8_t* is_val, const int64_t* nodes,
                     const int64_t* clients, int n, int fanout, unsigned long long seed_h, int* out_nbr, int* out_cnt,
                     hipStream_t s);

void sgd_step(float* theta, const float* grad, float* mom, bf16_t* shadow, bf16_t* split, const float* lr,
              const uint8_t* active,
              const uint8_t* first, int K, long P, long ld, float wd, float momentum, float dampening, int nesterov,
              hipStream_t s);
// sgd_step over the float4 spans of a block table seg[b] = (first float4 of the row, count ≤ 2048):
// the parameters whose gradients stepped themselves in their wgrad kernels are left out
void sgd_step_seg(float* theta, const float* grad, float* mom, bf16_t* split, const float* lr, const uint8_t* active,
                  const uint8_t* first, int K, long ld, float wd, float momentum, float dampening, int nesterov,
                  const long2* seg, int nblocks, hipStream_t s);
void adam_step(float* theta, const float* grad, float* m, float* v, bf16_t* shadow, const float* lr,
               const uint8_t* active, const float* step, int K, long P, long ld, float b1, float b2, float eps,
               float wd, hipStream_t s);
void broadcast_rows(float* theta, bf16_t* shadow, const float* src, int K, long P, long ld, hipStream_t s);
// split[k] = (bf16 hi plane, bf16 lo plane) of theta[k] rows ([K][2][ld] bf16)
void split_rows(const float* theta, bf16_t* split, int K, long P, long ld, hipStream_t s);
// [K][2][rows][C32] split planes of rows of C fp32 values (client stride w_cs) zero-padded to C32
void split_rows_padded(const float* w, long w_cs, int K, int rows, int C, int C32, bf16_t* out, hipStream_t s);
void delta_rows(const float* theta, const float* base, float* out, int K, long P, long ld, hipStream_t s);
// out += Σ_k w_k x[k] / num += Σ w m x, den += Σ w m: fp64 accumulators (in place)
void weighted_sum(const float* x, const double* w, double* out, int K, long P, long ld, hipStream_t s);
void mix_rows(const float* x, const float* w, void* out, int K, int M, long P, long ld, long ld_out, int f32,
              hipStream_t s);
void masked_weighted_sum(const float* x, const uint8_t* mask, const double* w, double* num, double* den, int K,
                         long P, long ld, hipStream_t s);
void dropout_mask(uint8_t* mask, int K, long P, float p, const uint32_t* seeds, hipStream_t s);
void block_sq_norms(const float* x, const int* block_ids, float* out, int K, long P, long ld, int nblocks,
                    hipStream_t s);
void seg_minmax(const float* x, const int* seg, float* mn, float* mx, int K, long P, long ld, int nseg,
                hipStream_t s);
void stochastic_qdq(float* x, const int* seg, const float* mn, const float* mx, int K, long P, long ld, int nseg,
                    const uint32_t* seeds, int levels, hipStream_t s);
void nnadq_qdq(float* x, const int* seg, const float* lo, const float* scale, const float* levels, int K, long P,
               long ld, int nseg, hipStream_t s);
void sign_pack(const float* g, uint8_t* out, int K, long P, long ld, hipStream_t s);
void sign_vote(const uint8_t* packed, const uint8_t* active, int* votes, int K, long P, hipStream_t s);
// embedding lookup · scale (+ positional encoding pe [L][D] fp32, position = token index mod L)
void embedding_fwd(const int* tokens, const void* table, void* out, int K, long n_tok, int D, long t_cs, int rep,
                   int f32, hipStream_t s, float scale = 1.f, const float* pe = nullptr, int L = 0);
void embedding_bwd(const int* tokens, const void* dy, float* dtable, int K, long n_tok, int D, long t_cs, int f32,
                   hipStream_t s, float scale = 1.f);
// deterministic form: keys [n] = client·V + token sorted (stable), order [n] their row indices;
// dtable rows of absent tokens are left untouched (zero them first)
// part (optional, embedding_bwd_part_floats): the chunked two-pass form (skewed token counts)
void embedding_bwd_sorted(const int* keys, const int* order, const void* dy, float* dtable, long n, int D, int V,
                          long t_cs, int f32, hipStream_t s, float scale = 1.f, float* part = nullptr);
long embedding_bwd_part_floats(long n, int D);
// masked mean over the sequence axis of x [S][L][D] (valid length per sequence)
void seq_mean_fwd(const void* x, const int* len, void* y, long S, int L, int D, int f32, hipStream_t s);
void seq_mean_bwd(const void* dy, const int* len, void* dx, long S, int L, int D, int f32, hipStream_t s);
// --------------------------------------------------------------- attention / graph
bool attn_supported(int L, int DH);
// MFMA flash attention (attention_mfma.hip), head dim 32 / 64; attn_fwd / attn_bwd route to it
bool attn_mfma_supported(int L, int DH);
// ldqkv / ldo > 0: q/k/v (and dq/dk/dv) are column blocks of packed [KB][L][ldqkv] rows, o / do
// of [KB][L][ldo] rows (the QKV / out projections' own layouts; attention_mfma.hip)
// drop_p > 0: dropout on the attention probabilities, keep mask = mix32(((head % hpc)·L + q)·L +
// key, drop_seeds[head / hpc]) >= p·2³², hpc = heads per client (B·H); MFMA kernels only
bool attn_fwd_mfma(const void* q, const void* k, const void* v, const int* key_valid, void* o, float* lse, long KBH,
                   int H, int L, int DH, int f32, hipStream_t s, int ldqkv = 0, int ldo = 0,
                   const uint32_t* drop_seeds = nullptr, int heads_per_client = 1, float drop_p = 0.f);
bool attn_bwd_mfma(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                   const int* key_valid, void* dq, void* dk, void* dv, float* delta, long KBH, int H, int L, int DH,
                   int f32, hipStream_t s, int ldqkv = 0, int ldo = 0, const uint32_t* drop_seeds = nullptr,
                   int heads_per_client = 1, float drop_p = 0.f);
bool attn_packed_supported(int L, int DH);
bool attn_fwd(const void* q, const void* k, const void* v, const int* key_valid, void* o, float* lse, long KBH, int H,
              int L, int DH, int f32, hipStream_t s, int ldqkv = 0, int ldo = 0, const uint32_t* drop_seeds = nullptr,
              int heads_per_client = 1, float drop_p = 0.f);
bool attn_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
              const int* key_valid, void* dq, void* dk, void* dv, float* delta, long KBH, int H, int L, int DH, int f32,
              hipStream_t s, int ldqkv = 0, int ldo = 0, const uint32_t* drop_seeds = nullptr,
              int heads_per_client = 1, float drop_p = 0.f);
void spmm(const int* rowptr, const int* col, const float* val, const void* x, void* y, int K, int N, int Nx, int F,
          long x_cs, long y_cs, int f32, hipStream_t s);
void gather_rows(const void* src, const int* idx, void* dst, long n, long row_bytes, hipStream_t s);
