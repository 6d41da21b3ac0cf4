// Launch API of the gfx950 kernels (host side). All launches are asynchronous on the given
// stream and never allocate or synchronise, so they can be captured into hipGraphs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;

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
};

struct ConvTNParams {
  const bf16_t* dy;  // [K][M][Co]
  const bf16_t* x;   // [K][B][H][W][C]
  float* dw;         // [K] rows (stride dw_cs) of [Co][R]
  long dy_cs, x_cs, dw_cs;
  int B, H, W, C, OH, OW, KH, KW, stride, pad;
  int M, Co, R;
  int splitk, m_per_split;
  FastDiv fd_ohw, fd_ow;  // filled by conv_tn()
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
                int Co, int H, int W, int Ci, int KH, int KW, int stride, int pad, int variant, hipStream_t s);
void conv_tn(ConvTNParams p, int K, int variant, hipStream_t s);
int conv_tn_num_variants();
// split-K factor the launch will use (callers zero the gradient rows first when > 1)
int conv_tn_splitk(int K, int Co, int R, int M, int C, int variant);

// ---------------------------------------------------------------- normalisation
long bn_workspace_floats(int K, long R, int C);  // ws size for bn_fwd / bn_bwd
void bn_fwd(const bf16_t* x, const bf16_t* gamma, const bf16_t* beta, const bf16_t* res, bf16_t* y, float* mean,
            float* rstd, const int* valid_rows, long g_cs, int K, int R, int C, int relu, float eps, int rep,
            float* ws, uint8_t* relu_mask, unsigned* counters,
            hipStream_t s);  // relu_mask: optional [K][R][C/8] bits out; counters: optional [K] zeros (fused coefs)
void bn_bwd(const bf16_t* dy, const bf16_t* x, const bf16_t* y, const float* mean, const float* rstd,
            const bf16_t* gamma, const int* valid_rows, long g_cs, int K, int R, int C, int relu, bf16_t* dx,
            bf16_t* dpre, float* dgamma, float* dbeta, long dg_cs, float* ws, const uint8_t* relu_mask,
            unsigned* counters, hipStream_t s);  // relu_mask (from bn_fwd) replaces reading y for the ReLU gate
void ln_fwd(const bf16_t* x, const bf16_t* gamma, const bf16_t* beta, bf16_t* y, float* mean, float* rstd,
            long g_cs, int K, long rows_per_client, int C, float eps, int rep, hipStream_t s);
void ln_bwd(const bf16_t* dy, const bf16_t* x, const float* mean, const float* rstd, const bf16_t* gamma,
            long g_cs, int K, long rows_per_client, int C, bf16_t* dx, float* dgamma, float* dbeta, long dg_cs,
            float* ws, hipStream_t s);
void col_sum(const bf16_t* x, float* out, long out_cs, int K, long rows, int C, hipStream_t s);

// ------------------------------------------------------------------- elementwise
void pool_fwd(const bf16_t* x, bf16_t* y, int* idx, int K, int B, int H, int W, int C, int OH, int OW, int k,
              int stride, int pad, int mode, hipStream_t s);
void pool_bwd(const bf16_t* dy, const int* idx, bf16_t* dx, int K, int B, int H, int W, int C, int OH, int OW,
              int k, int stride, int pad, int mode, hipStream_t s);
void gap_fwd(const bf16_t* x, bf16_t* y, int KB, int HW, int C, hipStream_t s);
void gap_bwd(const bf16_t* dy, bf16_t* dx, int KB, int HW, int C, hipStream_t s);
void ce_fwd_bwd(const bf16_t* logits, const int* labels, const int* valid, float* loss, float* correct,
                bf16_t* dlogits, int K, int B, int NC, hipStream_t s);
void relu_bwd(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long n, hipStream_t s);

// ------------------------------------------------------------- FL / optimiser
void sgd_step(float* theta, const float* grad, float* mom, bf16_t* shadow, const float* lr, const uint8_t* active,
              const uint8_t* first, int K, long P, long ld, float wd, float momentum, float dampening, int nesterov,
              hipStream_t s);
void adam_step(float* theta, const float* grad, float* m, float* v, bf16_t* shadow, const float* lr,
               const uint8_t* active, const float* step, int K, long P, long ld, float b1, float b2, float eps,
               float wd, hipStream_t s);
void broadcast_rows(float* theta, bf16_t* shadow, const float* src, int K, long P, long ld, hipStream_t s);
void delta_rows(const float* theta, const float* base, float* out, int K, long P, long ld, hipStream_t s);
void weighted_sum(const float* x, const float* w, float* out, int K, long P, long ld, hipStream_t s);
void mix_rows(const float* x, const float* w, bf16_t* out, int K, int M, long P, long ld, long ld_out,
              hipStream_t s);
void masked_weighted_sum(const float* x, const uint8_t* mask, const float* w, float* num, float* den, int K, long P,
                         long ld, hipStream_t s);
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
void embedding_fwd(const int* tokens, const bf16_t* table, bf16_t* out, int K, long n_tok, int D, long t_cs,
                   int rep, hipStream_t s);
void embedding_bwd(const int* tokens, const bf16_t* dy, float* dtable, int K, long n_tok, int D, long t_cs,
                   hipStream_t s);
// --------------------------------------------------------------- attention / graph
bool attn_supported(int L, int DH);
bool attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const int* key_valid, bf16_t* o, float* lse, long KBH,
              int H, int L, int DH, hipStream_t s);
bool attn_bwd(const bf16_t* dout, const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const float* lse,
              const int* key_valid, bf16_t* dq, bf16_t* dk, bf16_t* dv, float* delta, long KBH, int H, int L, int DH,
              hipStream_t s);
void spmm(const int* rowptr, const int* col, const float* val, const bf16_t* x, bf16_t* y, int K, int N, int Nx, int F,
          long x_cs, long y_cs, hipStream_t s);
void gather_rows(const bf16_t* src, const int* idx, bf16_t* dst, long n, long row_elems, hipStream_t s);
