// Normalisation kernels (gfx950): client-batched BatchNorm with per-client batch statistics
// over the *valid* rows only (ragged cohorts), fused residual-add + ReLU, and LayerNorm.
//
// BN forward = stats pass (per-(client,channel) Σx, Σx² with 16-B vector loads, LDS tree,
// one fp32 atomic per channel per block) + apply pass (normalise, γ/β, +residual, ReLU,
// zero padded rows). BN backward = reduction pass (Σg, Σg·x̂ with g = dy·relu'(y)) + apply
// pass (dx, and dpre for the residual branch); dγ/dβ land directly in the flat fp32
// gradient buffer (row stride P).
#include "common.h"
#include <algorithm>
#include <numeric>

#include "dls.h"

namespace {

constexpr int ROWS_PER_BLOCK = 512;  // upper bound; launches pick rows per block for >= ~2048 blocks

// Rows per workgroup for a (clients × rows) channel pass: enough workgroups to fill 256 CUs
// even when few clients are resident (K = 13 per GPU at 100 clients / 8 GPUs) and late layers
// are short (ResNet l4: 1,024 rows per client), but ≥ 64 rows so per-channel atomics stay few.
static int rows_per_block(long R, int K) {
  const long want = std::min<long>(64, (2048 + K - 1) / K);  // ≤ 64 partials per client
  const long bpc = std::max(1L, std::min(want, std::max(1L, R / 64)));
  return (int)std::min<long>(ROWS_PER_BLOCK, (R + bpc - 1) / bpc);
}

// Arguments of the per-(client, channel) coefficient stage (see bn_coef_kernel for the math).
struct BNCoefArgs {
  const void* gamma;  // T (bf16 or fp32, the compute dtype)
  const void* beta;
  const float* mean_in;
  const float* rstd_in;
  float* mean_out;
  float* rstd_out;
  float* coef;
  float* dgamma;
  float* dbeta;
  long dg_cs, g_cs;
  float eps;
  int rep, bwd;
};

template <typename T>
__device__ __forceinline__ void bn_coef_math(float s0, float s1, int k, int c, int C, float n, const BNCoefArgs& a) {
  const long i = (long)k * C + c;
  const float g = ldf(static_cast<const T*>(a.gamma) + (long)(k / a.rep) * a.g_cs + c);
  if (!a.bwd) {
    const float mu = s0 / n;
    const float var = fmaxf(s1 / n - mu * mu, 0.f);
    const float rs = rsqrtf(var + a.eps);
    const float sc = g * rs;
    a.mean_out[i] = mu;
    a.rstd_out[i] = rs;
    a.coef[2 * i] = sc;
    a.coef[2 * i + 1] = ldf(static_cast<const T*>(a.beta) + (long)(k / a.rep) * a.g_cs + c) - mu * sc;
  } else {
    const float mu = a.mean_in[i], rs = a.rstd_in[i];
    const float aa = g * rs;
    const float e = -aa * rs * s1 / n;
    const float d = -aa * s0 / n - e * mu;
    a.coef[3 * i] = aa;
    a.coef[3 * i + 1] = d;
    a.coef[3 * i + 2] = e;
    if (a.dgamma) {
      a.dbeta[(long)k * a.dg_cs + c] = s0;
      a.dgamma[(long)k * a.dg_cs + c] = s1;
    }
  }
}

// Generic per-(client, channel) double reduction over rows [0, nrows_valid):
//   mode 0: s0 += x, s1 += x²                       (BN fwd stats)
//   mode 1: g = dy*relu'(y); s0 += g, s1 += g*x̂      (BN bwd)
//   mode 2: s0 += x                                  (column sums, bias grads)
template <typename T, int V, int MODE>
__global__ void __launch_bounds__(256) chan_reduce_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                          const T* __restrict__ yv, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          const int* __restrict__ valid_rows, int R, int C, int relu,
                                                          float* __restrict__ ws, long ws_cs, int rpb,
                                                          const uint8_t* __restrict__ rmask, BNCoefArgs ca, int lda,
                                                          int ldb) {
  // lda / ldb: row strides of a and of b (channel-sliced views of a wider buffer, DenseNet);
  // yv is contiguous (row stride C)
  __shared__ float red[2][256 * V];
  const int k = blockIdx.y;
  const int CT = C / V;
  const int tid = threadIdx.x;
  const int nvalid = valid_rows ? min(valid_rows[k], R) : R;
  const int r0 = blockIdx.x * rpb;
  const int r1 = min(nvalid, r0 + rpb);
  const long base = (long)k * R * C, base_a = (long)k * R * lda, base_b = (long)k * R * ldb;
  for (int cg = 0; cg < CT; cg += 256) {
    const int ctn = min(256, CT - cg);
    const int RT = 256 / ctn;
    const int cc = tid % ctn, rl = tid / ctn;
    const bool active = rl < RT && (cg + cc) < CT;
    float s0[V], s1[V];
#pragma unroll
    for (int i = 0; i < V; ++i) s0[i] = s1[i] = 0.f;
    const int c0 = (cg + cc) * V;
    float mu[V], rs[V];
    if (MODE == 1 && active) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        mu[i] = mean[(long)k * C + c0 + i];
        rs[i] = rstd[(long)k * C + c0 + i];
      }
    }
    if (active) {
      for (int r = r0 + rl; r < r1; r += RT) {
        const long off = base + (long)r * C + c0;
        float va[V];
        load_vec<V>(a + base_a + (long)r * lda + c0, va);
        if (MODE == 0) {
#pragma unroll
          for (int i = 0; i < V; ++i) {
            s0[i] += va[i];
            s1[i] += va[i] * va[i];
          }
        } else if (MODE >= 2) {
#pragma unroll
          for (int i = 0; i < V; ++i) s0[i] += va[i];
        } else {
          float vx[V], vy[V];
          load_vec<V>(b + base_b + (long)r * ldb + c0, vx);
          uint32_t mbits = 0xFFu;
          if (rmask) {  // 1-bit ReLU mask written by the forward (V == 8): 1/16 of reading y
            mbits = rmask[((long)k * R + r) * (C / 8) + c0 / 8];
          } else if (relu) {
            load_vec<V>(yv + off, vy);
          }
#pragma unroll
          for (int i = 0; i < V; ++i) {
            const bool dead = rmask ? !((mbits >> i) & 1u) : (relu && vy[i] <= 0.f);
            const float g = dead ? 0.f : va[i];
            s0[i] += g;
            s1[i] += g * (vx[i] - mu[i]) * rs[i];
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < V; ++i) {
      red[0][tid * V + i] = s0[i];
      red[1][tid * V + i] = s1[i];
    }
    __syncthreads();
    if (active && rl == 0) {
      for (int j = 1; j < RT; ++j) {
        const int t2 = j * ctn + cc;
#pragma unroll
        for (int i = 0; i < V; ++i) {
          s0[i] += red[0][t2 * V + i];
          s1[i] += red[1][t2 * V + i];
        }
      }
      if (MODE == 2) {  // column sums straight into a (pre-zeroed) strided output
#pragma unroll
        for (int i = 0; i < V; ++i) atomicAdd(&ws[(long)k * ws_cs + c0 + i], s0[i]);
      } else if (MODE == 3) {  // column-sum partials [K][gridDim.x][C], folded in order
        float* part = ws + ((long)k * gridDim.x + blockIdx.x) * C;
#pragma unroll
        for (int i = 0; i < V; ++i) part[c0 + i] = s0[i];
      } else {  // per-workgroup partials [K][gridDim.x][2C]: deterministic, no memset, no atomics
        float* part = ws + ((long)k * gridDim.x + blockIdx.x) * 2 * C;
#pragma unroll
        for (int i = 0; i < V; ++i) {
          part[c0 + i] = s0[i];
          part[C + c0 + i] = s1[i];
        }
      }
    }
    __syncthreads();
  }
}

// Per-(client, channel) coefficients from the reduced sums (one tiny launch), so the apply
// passes are a pure fused multiply-add stream with no per-element division or rsqrt.
//  fwd:  coef = {scale = γ·rstd, shift = β − mean·scale};  also publishes mean / rstd
//  bwd:  dx = a·g + d + e·x  with a = γ·rstd, e = −a·rstd·Σgx̂/n, d = −a·Σg/n − e·mean;
//        dγ = Σgx̂, dβ = Σg written straight into the flat gradient buffer
// grid (cdiv(C, 32), K), 1024 threads = 32 channels × 32 part-groups: the per-workgroup partial
// sums of a client are reduced in a fixed order (deterministic) by 8 lanes per channel.
// partial-sum rows reduced in parallel per channel: G = 8 (256-thread workgroups). The coefficient
// kernel is tiny and sits on the stream's critical path; a 1024-thread form (G = 32) has to wait
// for a whole CU's wave slots while the other sub-cohort stream's GEMM workgroups occupy them
// (measured slower, profiles/r2_ab_bn_coef_groups.txt: removed)

// DenseNet running channel sums: out[k·out_cs + j·ldo + c] = Σ_p part[k][p][j][c] in fp64 (j = Σx, Σx²;
// c < g new channels) — the epilogue partials of one growth conv summed into the block's running
// sums in one launch (one 1024-thread workgroup per client, four independent fp64 chains per
// thread so the loads pipeline, all combined in a fixed order: deterministic). Replaces a PyTorch
// fp64 reduction over the middle dimension plus a strided copy (≈ 170 µs per layer).
template <typename T>
__global__ void __launch_bounds__(1024) part_sum_f64_kernel(const T* __restrict__ part, int nparts, int g,
                                                            double* __restrict__ out, long out_cs, int ldo) {
  __shared__ double red[1024];
  const int k = blockIdx.x, ncol = 2 * g, t = threadIdx.x;
  const int groups = 1024 / ncol;  // (host: ncol <= 1024)
  const int col = t % ncol, grp = t / ncol;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (grp < groups) {
    const T* pk = part + (long)k * nparts * ncol + col;
    const long st = (long)groups * ncol;
    int p = grp;
    for (; p + 3 * groups < nparts; p += 4 * groups) {
      const T* q = pk + (long)p * ncol;
      a0 += (double)q[0];
      a1 += (double)q[st];
      a2 += (double)q[2 * st];
      a3 += (double)q[3 * st];
    }
    for (; p < nparts; p += groups) a0 += (double)pk[(long)p * ncol];
  }
  red[t] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (t < ncol) {
    double a = 0.0;
    for (int q = 0; q < groups; ++q) a += red[q * ncol + t];
    out[(long)k * out_cs + (long)(t / g) * ldo + (t % g)] = a;
  }
}


// DenseNet block input: fp64 Σx, Σx² of every channel over a chunk of `rb` rows (rows at stride
// ldx, rows past the client's valid count excluded) → part[k][chunk][2][C]; part_sum_f64_kernel<double>
// then folds the chunks in order into the running sums (replaces PyTorch casts + reductions)
__global__ void __launch_bounds__(256) chan_sums_f64_kernel(const float* __restrict__ x, long x_cs, int ldx, int R,
                                                            int C, const int* __restrict__ valid, int rb,
                                                            double* __restrict__ part, int nch) {
  __shared__ double r0[256], r1[256];
  const int k = blockIdx.y, ch = blockIdx.x, t = threadIdx.x;
  const int nv = valid ? min(valid[k], R) : R;
  const int rbeg = ch * rb, rend = min(nv, rbeg + rb);
  const float* xk = x + (long)k * x_cs;
  for (int c0 = 0; c0 < C; c0 += 256) {
    const int ctn = min(256, C - c0), S = 256 / ctn;
    const int cc = t % ctn, sg = t / ctn;
    double s0 = 0.0, s1 = 0.0;
    if (sg < S) {
#pragma unroll 4
      for (int r = rbeg + sg; r < rend; r += S) {
        const double v = (double)xk[(long)r * ldx + c0 + cc];
        s0 += v;
        s1 = fma(v, v, s1);
      }
    }
    r0[t] = s0;
    r1[t] = s1;
    __syncthreads();
    if (sg == 0) {
      for (int j = 1; j < S; ++j) {
        s0 += r0[j * ctn + cc];
        s1 += r1[j * ctn + cc];
      }
      double* pp = part + ((long)k * nch + ch) * 2 * C + c0 + cc;
      pp[0] = s0;
      pp[C] = s1;
    }
    __syncthreads();
  }
}

// First stage for the conv-epilogue statistics, which arrive as one partial per 32 GEMM rows
// (2,048 per client on a 32x32x64 layer): a single (32-channel, client) workgroup reading them
// one after another took ~0.4 ms per BN layer (latency-bound: 2 x 33 workgroups on 256 CUs).
// This stage folds FOLD consecutive partials of every (client, 2C column) into one fp64 value
// with grid (cdiv(nparts, FOLD), K) — thousands of workgroups, plain coalesced row reads, a
// fixed summation order (deterministic) — and bn_coef then reduces the few fp64 folds.
constexpr int FOLD = 64;
__global__ void __launch_bounds__(256) part_fold_kernel(const float* __restrict__ part, int nparts, int C2,
                                                        double* __restrict__ out, int nfold) {
  __shared__ double red[256];
  const int k = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
  const int b0 = g * FOLD, nb = min(FOLD, nparts - b0);
  const float* src = part + ((long)k * nparts + b0) * C2;
  double* dst = out + ((long)k * nfold + g) * C2;
  // ctn lanes across columns, S = 256 / ctn sub-groups across the partial rows
  for (int c0 = 0; c0 < C2; c0 += 256) {
    const int ctn = min(256, C2 - c0);
    const int S = 256 / ctn;
    const int cc = tid % ctn, sg = tid / ctn;
    double a = 0.0;
    if (sg < S) {
#pragma unroll 8
      for (int b = sg; b < nb; b += S) a += (double)src[(long)b * C2 + c0 + cc];
    }
    red[tid] = a;
    __syncthreads();
    if (sg == 0) {
      for (int j = 1; j < S; ++j) a += red[j * ctn + cc];
      dst[c0 + cc] = a;
    }
    __syncthreads();
  }
}

template <typename T, typename PT, int G>
__global__ void __launch_bounds__(32 * G) bn_coef_kernel(const PT* __restrict__ ws, int nparts,
                                                      const T* __restrict__ gamma,
                                                      const T* __restrict__ beta, const int* __restrict__ valid_rows,
                                                      const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      float* __restrict__ coef, float* __restrict__ dgamma,
                                                      float* __restrict__ dbeta, long dg_cs, long g_cs, int K, int R, int C,
                                                      float eps, int rep, int bwd, int ldp, long pcs) {
  // partials are summed in fp64 (the conv-epilogue statistics arrive as thousands of 32-row
  // partials per channel; Σx² − n·μ² then keeps its precision), in a fixed order
  __shared__ double red[2][G][33];
  const int k = blockIdx.y;
  const int cl = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double d0 = 0.0, d1 = 0.0;
  if (c < C) {
    // (ldp / pcs: row length / client stride of the partial rows when they cover more channels
    // than C — a DenseNet block's running sums, read for a channel prefix; 0 = C / nparts·2C)
    const int lp = ldp ? ldp : C;
    const PT* part = ws + (long)k * (pcs ? pcs : (long)nparts * 2 * lp);
    for (int b = grp; b < nparts; b += G) {
      d0 += part[(long)b * 2 * lp + c];
      d1 += part[(long)b * 2 * lp + lp + c];
    }
  }
  red[0][grp][cl] = d0;
  red[1][grp][cl] = d1;
  __syncthreads();
  if (grp != 0 || c >= C) return;
#pragma unroll
  for (int g2 = 1; g2 < G; ++g2) {
    d0 += red[0][g2][cl];
    d1 += red[1][g2][cl];
  }
  const float s0 = (float)d0, s1 = (float)d1;
  const long i = (long)k * C + c;
  const int nvalid = valid_rows ? min(valid_rows[k], R) : R;
  const float n = (float)max(nvalid, 1);
  const float g = ldf(gamma + (long)(k / rep) * g_cs + c);
  if (!bwd) {
    const double mud = d0 / n;
    const float mu = (float)mud;
    const float var = (float)fmax(d1 / n - mud * mud, 0.0);
    const float rs = rsqrtf(var + eps);
    const float sc = g * rs;
    mean_out[i] = mu;
    rstd_out[i] = rs;
    coef[2 * i] = sc;
    coef[2 * i + 1] = ldf(beta + (long)(k / rep) * g_cs + c) - mu * sc;
  } else {
    const float mu = mean_in[i], rs = rstd_in[i];
    const float a = g * rs;
    const float e = -a * rs * s1 / n;
    const float d = -a * s0 / n - e * mu;
    coef[3 * i] = a;
    coef[3 * i + 1] = d;
    coef[3 * i + 2] = e;
    if (dgamma) {
      dbeta[(long)k * dg_cs + c] = s0;
      dgamma[(long)k * dg_cs + c] = s1;
    }
  }
}

template <typename TT, typename PT, typename... A>
void launch_coef(dim3 grid, hipStream_t s, A... args) {
  hipLaunchKernelGGL((bn_coef_kernel<TT, PT, 8>), grid, dim3(32 * 8), 0, s, args...);
}

// V fp32 values → their split-bf16 planes (hi = bf16(v), lo = bf16(v − hi), RNE): the operand form
// of the pre-split GEMMs (conv_pl.hip), bit-identical to the split those GEMMs would do themselves
template <int V>
__device__ __forceinline__ void store_planes(bf16_t* hi, bf16_t* lo, const float* f) {
  if constexpr (V % 2 == 0) {
    uint32_t h[V / 2], l[V / 2];
#pragma unroll
    for (int i = 0; i < V / 2; ++i) split_pair(f[2 * i], f[2 * i + 1], h[i], l[i]);
    if constexpr (V == 8) {
      *reinterpret_cast<uint4*>(hi) = make_uint4(h[0], h[1], h[2], h[3]);
      *reinterpret_cast<uint4*>(lo) = make_uint4(l[0], l[1], l[2], l[3]);
    } else if constexpr (V == 4) {
      *reinterpret_cast<uint2*>(hi) = make_uint2(h[0], h[1]);
      *reinterpret_cast<uint2*>(lo) = make_uint2(l[0], l[1]);
    } else {
#pragma unroll
      for (int i = 0; i < V / 2; ++i) {
        reinterpret_cast<uint32_t*>(hi)[i] = h[i];
        reinterpret_cast<uint32_t*>(lo)[i] = l[i];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) split2(f[i], hi[i], lo[i]);
  }
}

// thread owns one V-channel chunk and strides over rows; grid (row-blocks, K)
// yp (fp32 only): also / instead (y_f32 = 0) write the output's split planes, client k's hi plane
// at yp + 2·k·R·C, its lo plane R·C elements later (the [K][2][R][C] layout of ops split_planes)
template <typename T, int V>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                       T* __restrict__ y, const int* __restrict__ valid_rows,
                                                       const float* __restrict__ coef, int R, int C, int relu,
                                                       int rpb, uint8_t* __restrict__ rmask, int ldx,
                                                       bf16_t* __restrict__ yp, int y_f32,
                                                       const float* __restrict__ res_coef) {
  // x / res rows at stride ldx (channel slice of a wider buffer), y contiguous. res_coef [K][C][2]:
  // res is the RAW input of a second BatchNorm (no ReLU, same valid rows) whose apply is folded
  // in here — out += res_scale·res + res_shift, the bits of applying it first (ResNet downsample)
  const int k = blockIdx.y;
  const int CT = C / V;
  const int nvalid = valid_rows ? min(valid_rows[k], R) : R;
  const int r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  const long base = (long)k * R * C, base_x = (long)k * R * ldx;
  for (int cg = 0; cg < CT; cg += 256) {
    const int ctn = min(256, CT - cg);
    const int RT = 256 / ctn;
    const int cc = threadIdx.x % ctn, rl = threadIdx.x / ctn;
    if (rl >= RT) continue;
    const int c0 = (cg + cc) * V;
    float sc[V], sh[V], rsc[V], rsh[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sc[j] = coef[2 * ((long)k * C + c0 + j)];
      sh[j] = coef[2 * ((long)k * C + c0 + j) + 1];
      rsc[j] = res_coef ? res_coef[2 * ((long)k * C + c0 + j)] : 0.f;
      rsh[j] = res_coef ? res_coef[2 * ((long)k * C + c0 + j) + 1] : 0.f;
    }
    for (int r = r0 + rl; r < r1; r += RT) {
      const long off = base + (long)r * C + c0;
      float out[V];
      if (r < nvalid) {
        float v[V];
        const long offx = base_x + (long)r * ldx + c0;
        load_vec<V>(x + offx, v);
#pragma unroll
        for (int j = 0; j < V; ++j) out[j] = fmaf(v[j], sc[j], sh[j]);
        if (res) {
          float rv[V];
          load_vec<V>(res + offx, rv);
          if (res_coef) {
#pragma unroll
            for (int j = 0; j < V; ++j) out[j] += fmaf(rv[j], rsc[j], rsh[j]);
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j) out[j] += rv[j];
          }
        }
        if (relu) {
#pragma unroll
          for (int j = 0; j < V; ++j) out[j] = fmaxf(out[j], 0.f);
        }
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) out[j] = 0.f;
      }
      if (rmask) {  // bit j = (stored out_j > 0): exactly the mask the backward would read from y
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < V; ++j) m |= (rt<T>(out[j]) > 0.f ? 1u : 0u) << j;
        rmask[((long)k * R + r) * (C / 8) + c0 / 8] = (uint8_t)m;
      }
      if (y_f32) store_vec<V>(y + off, out);
      if (yp) {
        bf16_t* hp = yp + (long)k * R * C + off;  // (off includes k·R·C: hi at 2·k·R·C + r·C + c)
        store_planes<V>(hp, hp + (long)R * C, out);
      }
    }
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                           const T* __restrict__ y,
                                                           const int* __restrict__ valid_rows,
                                                           const float* __restrict__ coef, int R, int C, int relu,
                                                           T* __restrict__ dx, T* __restrict__ dpre,
                                                           int rpb, const uint8_t* __restrict__ rmask, int ldx,
                                                           int acc_dx, bf16_t* __restrict__ dxp, int dx_f32) {
  // dxp (fp32, contiguous dx, no acc_dx): dX's split planes ([K][2][R][C]), with or without
  // (dx_f32 = 0) the fp32 dX
  // x and dx rows at stride ldx (channel slice of a wider buffer); acc_dx: dx += (DenseNet: the
  // block buffer's gradient collects every later layer's contribution); dy / y / dpre contiguous
  const int k = blockIdx.y;
  const int CT = C / V;
  const int nvalid = valid_rows ? min(valid_rows[k], R) : R;
  const int r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  const long base = (long)k * R * C, base_x = (long)k * R * ldx;
  for (int cg = 0; cg < CT; cg += 256) {
    const int ctn = min(256, CT - cg);
    const int RT = 256 / ctn;
    const int cc = threadIdx.x % ctn, rl = threadIdx.x / ctn;
    if (rl >= RT) continue;
    const int c0 = (cg + cc) * V;
    float ca[V], cd[V], ce[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const long q = 3 * ((long)k * C + c0 + j);
      ca[j] = coef[q];
      cd[j] = coef[q + 1];
      ce[j] = coef[q + 2];
    }
    for (int r = r0 + rl; r < r1; r += RT) {
      const long off = base + (long)r * C + c0;
      const long offx = base_x + (long)r * ldx + c0;
      float o[V], gp[V];
      if (r < nvalid) {
        float vdy[V], vx[V];
        load_vec<V>(dy + off, vdy);
        load_vec<V>(x + offx, vx);
        if (rmask) {
          const uint32_t mbits = rmask[((long)k * R + r) * (C / 8) + c0 / 8];
#pragma unroll
          for (int j = 0; j < V; ++j) vdy[j] = ((mbits >> j) & 1u) ? vdy[j] : 0.f;
        } else if (relu) {
          float vy[V];
          load_vec<V>(y + off, vy);
#pragma unroll
          for (int j = 0; j < V; ++j) vdy[j] = vy[j] > 0.f ? vdy[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
          gp[j] = vdy[j];
          o[j] = fmaf(ca[j], vdy[j], fmaf(ce[j], vx[j], cd[j]));
        }
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = gp[j] = 0.f;
      }
      if (acc_dx) {
        float prev[V];
        load_vec<V>(dx + offx, prev);
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] += prev[j];
      }
      if (dx_f32) store_vec<V>(dx + offx, o);
      if (dxp) {
        bf16_t* hp = dxp + (long)k * R * C + off;
        store_planes<V>(hp, hp + (long)R * C, o);
      }
      if (dpre) store_vec<V>(dpre + off, gp);
    }
  }
}

int vw(int C) { return (C % 8 == 0) ? 8 : (C % 4 == 0) ? 4 : 1; }

// ------------------------------------------------------------------ LayerNorm
// yp (fp32 only): also write y's split planes ([K][2][rpc][C]: hi, then lo rpc·C later) for the
// split-plane linears that read it (ops.functional planes)
template <typename T>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ gamma,
                                                     const T* __restrict__ beta, T* __restrict__ y,
                                                     float* __restrict__ mean, float* __restrict__ rstd, long g_cs,
                                                     long nrows, long rpc, int C, float eps, int rep,
                                                     bf16_t* __restrict__ yp) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const int k = (int)(row / rpc);
  const T* xr = x + row * C;
  float s = 0.f, sq = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float v = ldf(xr + c);
    s += v;
    sq += v * v;
  }
  s = wave_sum(s);
  sq = wave_sum(sq);
  const float mu = s / C;
  const float rs = rsqrtf(fmaxf(sq / C - mu * mu, 0.f) + eps);
  const T* g = gamma + (long)(k / rep) * g_cs;
  const T* b = beta + (long)(k / rep) * g_cs;
  bf16_t* hp = yp ? yp + (row + (long)k * rpc) * C : nullptr;  // (row = k·rpc + r: hi at (2k·rpc + r)·C)
  for (int c = lane; c < C; c += 64) {
    const float o = (ldf(xr + c) - mu) * rs * ldf(g + c) + ldf(b + c);
    stf(y + row * C + c, o);
    if (hp) {
      bf16_t h, l;
      split2(rt<T>(o), h, l);
      hp[c] = h;
      hp[rpc * C + c] = l;
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// fp32, C % 128 == 0: each lane owns column pairs (2·lane + 128·i): one 8-B load per pair (the
// row held in registers, read once), 8-B y stores and 4-B packed (hi, lo) plane stores — the
// generic kernel above re-reads x and writes the planes 2 B per lane
template <int NC2>
__global__ void __launch_bounds__(256) ln_fwd_pairs_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* __restrict__ y,
                                                           float* __restrict__ mean, float* __restrict__ rstd,
                                                           long g_cs, long nrows, long rpc, int C, float eps, int rep,
                                                           bf16_t* __restrict__ yp) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const int k = (int)(row / rpc);
  const float2* xr = reinterpret_cast<const float2*>(x + row * C);
  float2 v[NC2];
  float s = 0.f, sq = 0.f;
#pragma unroll
  for (int i = 0; i < NC2; ++i) {
    v[i] = xr[lane + 64 * i];
    s += v[i].x;
    s += v[i].y;
    sq += v[i].x * v[i].x;
    sq += v[i].y * v[i].y;
  }
  s = wave_sum(s);
  sq = wave_sum(sq);
  const float mu = s / C;
  const float rs = rsqrtf(fmaxf(sq / C - mu * mu, 0.f) + eps);
  const float2* g = reinterpret_cast<const float2*>(gamma + (long)(k / rep) * g_cs);
  const float2* b = reinterpret_cast<const float2*>(beta + (long)(k / rep) * g_cs);
  float2* yr = reinterpret_cast<float2*>(y + row * C);
  uint32_t* hp = yp ? reinterpret_cast<uint32_t*>(yp + (row + (long)k * rpc) * C) : nullptr;
#pragma unroll
  for (int i = 0; i < NC2; ++i) {
    const int c2 = lane + 64 * i;
    const float2 gg = g[c2], bb = b[c2];
    const float2 o = make_float2((v[i].x - mu) * rs * gg.x + bb.x, (v[i].y - mu) * rs * gg.y + bb.y);
    yr[c2] = o;
    if (hp) {
      uint32_t h, l;
      split_pair(o.x, o.y, h, l);
      hp[c2] = h;
      hp[rpc * C / 2 + c2] = l;
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

constexpr int LN_MAXC = 16;  // C <= 1024
// NC = ceil(C / 64) column slots per lane. Each wave walks rows_per_wave rows of one client with the
// row in registers (read once) and the next row's dy / x / μ / rstd loads issued before this row's
// reductions, so a row's HBM round trip overlaps the previous row's math and stores.
template <typename T, int NC>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const T* __restrict__ gamma, long g_cs, long rpc, int C,
                                                     T* __restrict__ dx, float* __restrict__ dgamma,
                                                     float* __restrict__ dbeta, long dg_cs, int rows_per_wave,
                                                     float* __restrict__ part) {
  // grid: (row-groups, K); each wave handles rows_per_wave rows of client k
  const int k = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long rbeg = wave * rows_per_wave;
  const long rend = min(rpc, rbeg + rows_per_wave);
  const T* g = gamma + (long)k * g_cs;
  float dg[NC], db[NC], gv[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    dg[i] = db[i] = 0.f;
    const int c = lane + 64 * i;
    gv[i] = c < C ? ldf(g + c) : 0.f;
  }
  float cy[NC], cx[NC], cmu = 0.f, crs = 0.f;
  auto load_row = [&](long r, float* ly, float* lx, float& lmu, float& lrs) {
    const long row = (long)k * rpc + r;
    lmu = mean[row];
    lrs = rstd[row];
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + 64 * i;
      ly[i] = c < C ? ldf(dy + row * C + c) : 0.f;
      lx[i] = c < C ? ldf(x + row * C + c) : 0.f;
    }
  };
  if (rbeg < rend) load_row(rbeg, cy, cx, cmu, crs);
  for (long r = rbeg; r < rend; ++r) {
    float ny[NC], nx[NC], nmu = 0.f, nrs = 0.f;
    if (r + 1 < rend) load_row(r + 1, ny, nx, nmu, nrs);
    const long row = (long)k * rpc + r;
    float a = 0.f, b = 0.f, xh[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      xh[i] = (cx[i] - cmu) * crs;
      const float gg = cy[i] * gv[i];
      a += gg;
      b += gg * xh[i];
      dg[i] += cy[i] * xh[i];
      db[i] += cy[i];
    }
    a = wave_sum(a) / C;
    b = wave_sum(b) / C;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + 64 * i;
      if (c < C) stf(dx + row * C + c, crs * (cy[i] * gv[i] - a - xh[i] * b));
    }
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      cy[i] = ny[i];
      cx[i] = nx[i];
    }
    cmu = nmu;
    crs = nrs;
  }
  if (rend > rbeg || part) {  // (partials: every wave writes its row, zeros included)
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + 64 * i;
      if (c < C) {
        if (part) {  // this wave's partial row [2C], folded in wave order (deterministic)
          float* pw = part + ((long)k * gridDim.x * 4 + wave) * 2 * C;
          pw[c] = dg[i];
          pw[C + c] = db[i];
        } else {
          atomicAdd(&dgamma[(long)k * dg_cs + c], dg[i]);
          atomicAdd(&dbeta[(long)k * dg_cs + c], db[i]);
        }
      }
    }
  }
}

// out0[k·out_cs + c] = Σ_b part[(k·nparts + b)·W + c] (b ascending), out1 likewise at column C + c
__global__ void __launch_bounds__(256) part_sum_kernel(const float* __restrict__ part, int nparts, int W, int C,
                                                       float* __restrict__ out0, float* __restrict__ out1, long out_cs) {
  const int k = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float* p = part + (long)k * nparts * W;
  float a = 0.f, b = 0.f;
  for (int i = 0; i < nparts; ++i) {
    a += p[(long)i * W + c];
    if (out1) b += p[(long)i * W + C + c];
  }
  out0[(long)k * out_cs + c] = a;
  if (out1) out1[(long)k * out_cs + c] = b;
}

}  // namespace

#define DISPATCH_V(V, ...)          \
  if (V == 8) {                     \
    constexpr int VV = 8;           \
    __VA_ARGS__;                    \
  } else if (V == 4) {              \
    constexpr int VV = 4;           \
    __VA_ARGS__;                    \
  } else {                          \
    constexpr int VV = 1;           \
    __VA_ARGS__;                    \
  }
// element type of the activations / γ β: bf16 (f32 = 0) or fp32 (f32 = 1)
#define DISPATCH_T(F32, ...)        \
  if (F32) {                        \
    typedef float TT;               \
    __VA_ARGS__;                    \
  } else {                          \
    typedef bf16_t TT;              \
    __VA_ARGS__;                    \
  }
#define CP(p) static_cast<const TT*>(p)
#define MP(p) static_cast<TT*>(p)

// fp32 offset of the fp64 fold area (even: 8-B aligned in the 256-B aligned workspace)
static long bn_fold_offset(int K, long R, int C) {
  const long parts = (R + rows_per_block(R, K) - 1) / rows_per_block(R, K);
  return ((long)K * 3 * C + (long)K * parts * 2 * C + 1) & ~1L;
}

long bn_workspace_floats(int K, long R, int C) {
  // + the fp64 folds of conv-epilogue partials (at most one per 32 rows, FOLD per fold)
  const long nfold = cdiv((int)cdiv((int)R, 32), FOLD);
  return bn_fold_offset(K, R, C) + (long)K * nfold * 2 * C * 2;
}

void bn_fwd(const void* x, const void* gamma, const void* beta, const void* res, void* y, float* mean, float* rstd,
            const int* valid_rows, long g_cs, int K, int R, int C, int relu, float eps, int rep, float* ws,
            uint8_t* rmask, int f32, hipStream_t s, int ldx, const float* pre_part,
            int pre_nparts, bf16_t* yp, int y_f32, float* coef_out, int apply, const float* res_coef) {
  if (ldx == 0) ldx = C;
  // ws layout: [K][3C] coefficients, then [K][parts][2C] per-workgroup partial sums. coef_out: the
  // (scale, shift) pairs go there instead and outlive this call (apply = 0: the consumer conv
  // applies them while staging its input, conv_halo_bn_fwd)
  float* coef = coef_out ? coef_out : ws;
  const float* part = pre_part ? pre_part : ws + (long)3 * C * K;
  const int rpb = rows_per_block(R, K);
  dim3 grid(cdiv(R, rpb), K);
  const int nparts = pre_part ? pre_nparts : (int)grid.x;
  const int V = vw(std::gcd(C, ldx));
  BNCoefArgs ca{gamma, beta, nullptr, nullptr, mean, rstd, coef, nullptr, nullptr, 0L, g_cs, eps, rep, 0};
  if (V != 8) rmask = nullptr;  // bit masks need 8-channel vectors
  DISPATCH_T(f32, {
    if (!pre_part) {  // (else the producing conv's epilogue already wrote the partial sums)
      DISPATCH_V(V, hipLaunchKernelGGL((chan_reduce_kernel<TT, VV, 0>), grid, dim3(256), 0, s, CP(x), nullptr, nullptr,
                                       nullptr, nullptr, valid_rows, R, C, 0, ws + (long)3 * C * K, (long)2 * C, rpb,
                                       nullptr, ca, ldx, ldx));
    }
    if (pre_part && nparts > FOLD && nparts <= cdiv(R, 32)) {
      // thousands of epilogue partials per client: fold them wide first (part_fold_kernel)
      const int nfold = cdiv(nparts, FOLD);
      double* folds = reinterpret_cast<double*>(ws + bn_fold_offset(K, R, C));
      hipLaunchKernelGGL(part_fold_kernel, dim3(nfold, K), dim3(256), 0, s, pre_part, nparts, 2 * C, folds, nfold);
      launch_coef<TT, double>(dim3(cdiv(C, 32), K), s, (const double*)folds, nfold, CP(gamma), CP(beta), valid_rows,
                              (const float*)nullptr, (const float*)nullptr, mean, rstd, coef, (float*)nullptr,
                              (float*)nullptr, 0L, g_cs, K, R, C, eps, rep, 0, 0, 0L);
    } else {
      launch_coef<TT, float>(dim3(cdiv(C, 32), K), s, part, nparts, CP(gamma), CP(beta), valid_rows,
                             (const float*)nullptr, (const float*)nullptr, mean, rstd, coef, (float*)nullptr,
                             (float*)nullptr, 0L, g_cs, K, R, C, eps, rep, 0, 0, 0L);
    }
    if (apply) {
      DISPATCH_V(V, hipLaunchKernelGGL((bn_apply_kernel<TT, VV>), grid, dim3(256), 0, s, CP(x), CP(res), MP(y),
                                       valid_rows, coef, R, C, relu, rpb, rmask, ldx, f32 ? yp : nullptr,
                                       f32 ? y_f32 : 1, res_coef));
    }
  });
}

void bn_apply_only(const float* x, const float* coef, const int* valid_rows, int K, int R, int C, int relu,
                   bf16_t* yp, uint8_t* rmask, hipStream_t s, float* y) {
  // the apply pass of bn_fwd with coefficients computed earlier (bn_coef): planes (+ ReLU bits)
  // and / or the fp32 output y — what a deferred BN materialises when its consumer cannot apply it
  const int rpb = rows_per_block(R, K);
  dim3 grid(cdiv(R, rpb), K);
  if (C % 8 == 0) {
    hipLaunchKernelGGL((bn_apply_kernel<float, 8>), grid, dim3(256), 0, s, x, (const float*)nullptr, y,
                       valid_rows, coef, R, C, relu, rpb, rmask, C, yp, y ? 1 : 0, (const float*)nullptr);
  } else {
    hipLaunchKernelGGL((bn_apply_kernel<float, 1>), grid, dim3(256), 0, s, x, (const float*)nullptr, y,
                       valid_rows, coef, R, C, relu, rpb, (uint8_t*)nullptr, C, yp, y ? 1 : 0, (const float*)nullptr);
  }
}

void bn_bwd(const void* dy, const void* x, const void* y, const float* mean, const float* rstd, const void* gamma,
            const int* valid_rows, long g_cs, int K, int R, int C, int relu, void* dx, void* dpre, float* dgamma,
            float* dbeta, long dg_cs, float* ws, const uint8_t* rmask, int f32, hipStream_t s,
            int ldx, int acc_dx, bf16_t* dxp, int dx_f32, const float* pre_part, int pre_nparts, float* coef_ext,
            int stage) {
  // stage 0: coefficients + apply; 1: coefficients (and dγ, dβ) only, into coef_ext — a consumer
  // applies them in its loader (conv_halo_wgrad.hip dy mode 2); 2: the apply alone from coef_ext
  if (!f32 || acc_dx || (ldx != 0 && ldx != C)) {  // planes: fp32, contiguous dX only
    dxp = nullptr;
    dx_f32 = 1;
  }
  if (ldx == 0) ldx = C;
  float* coef = coef_ext ? coef_ext : ws;
  float* part = ws + (long)3 * C * K;
  const int rpb = rows_per_block(R, K);
  dim3 grid(cdiv(R, rpb), K);
  const int V = vw(std::gcd(C, ldx));
  if (V != 8) rmask = nullptr;
  BNCoefArgs ca{gamma, nullptr, mean, rstd, nullptr, nullptr, coef, dgamma, dbeta, dg_cs, g_cs, 0.f, 1, 1};
  DISPATCH_T(f32, {
    if (stage == 2) {
    } else if (pre_part) {  // Σĝ / Σĝx̂ from the dgrad epilogue that produced dy: coefficients only
      if (pre_nparts > FOLD && pre_nparts <= cdiv(R, 32)) {
        const int nfold = cdiv(pre_nparts, FOLD);
        double* folds = reinterpret_cast<double*>(ws + bn_fold_offset(K, R, C));
        hipLaunchKernelGGL(part_fold_kernel, dim3(nfold, K), dim3(256), 0, s, pre_part, pre_nparts, 2 * C, folds,
                           nfold);
        launch_coef<TT, double>(dim3(cdiv(C, 32), K), s, (const double*)folds, nfold, CP(gamma), (const TT*)nullptr,
                                valid_rows, mean, rstd, (float*)nullptr, (float*)nullptr, coef, dgamma, dbeta, dg_cs,
                                g_cs, K, R, C, 0.f, 1, 1, 0, 0L);
      } else {
        launch_coef<TT, float>(dim3(cdiv(C, 32), K), s, pre_part, pre_nparts, CP(gamma), (const TT*)nullptr,
                               valid_rows, mean, rstd, (float*)nullptr, (float*)nullptr, coef, dgamma, dbeta, dg_cs,
                               g_cs, K, R, C, 0.f, 1, 1, 0, 0L);
      }
    } else {
      DISPATCH_V(V, hipLaunchKernelGGL((chan_reduce_kernel<TT, VV, 1>), grid, dim3(256), 0, s, CP(dy), CP(x), CP(y),
                                       mean, rstd, valid_rows, R, C, relu, part, (long)2 * C, rpb, rmask, ca, C, ldx));
    }
    if (!pre_part && stage != 2)
      launch_coef<TT, float>(dim3(cdiv(C, 32), K), s, (const float*)part, (int)grid.x, CP(gamma), (const TT*)nullptr,
                             valid_rows, mean, rstd, (float*)nullptr, (float*)nullptr, coef, dgamma, dbeta, dg_cs, g_cs, K,
                             R, C, 0.f, 1, 1, 0, 0L);
    if (stage != 1)
      DISPATCH_V(V, hipLaunchKernelGGL((bn_bwd_apply_kernel<TT, VV>), grid, dim3(256), 0, s, CP(dy), CP(x), CP(y),
                                       valid_rows, coef, R, C, relu, MP(dx), MP(dpre), rpb, rmask, ldx, acc_dx, dxp,
                                       dx_f32));
  });
}

void fold_col_partials(const float* part, int nparts, int C, float* out, long out_cs, int K, hipStream_t s) {
  hipLaunchKernelGGL(part_sum_kernel, dim3(cdiv(C, 256), K), dim3(256), 0, s, part, nparts, C, C, out, (float*)nullptr,
                     out_cs);
}

void bn_bwd_coef_parts(const float* part, int nparts, const float* gamma, long g_cs, const int* valid_rows,
                       const float* mean, const float* rstd, int K, int R, int C, float* coef, float* dgamma,
                       float* dbeta, long dg_cs, hipStream_t s) {
  launch_coef<float, float>(dim3(cdiv(C, 32), K), s, part, nparts, gamma, (const float*)nullptr, valid_rows, mean, rstd,
                            (float*)nullptr, (float*)nullptr, coef, dgamma, dbeta, dg_cs, g_cs, K, R, C, 0.f, 1, 1, 0,
                            0L);
}

void part_sum_f64(const float* part, int K, int nparts, int g, double* out, long out_cs, int ldo, hipStream_t s) {
  if (K == 0) return;
  hipLaunchKernelGGL(part_sum_f64_kernel<float>, dim3(K), dim3(1024), 0, s, part, nparts, g, out, out_cs, ldo);
}

long chan_sums_f64_ws(int R, int C) { return (long)cdiv(R, 256) * 2 * C; }  // doubles per client

void chan_sums_f64(const float* x, long x_cs, int ldx, int K, int R, int C, const int* valid, double* ws, double* out,
                   long out_cs, int ldo, hipStream_t s) {
  if (K == 0 || R == 0) return;
  const int rb = 256, nch = cdiv(R, rb);
  hipLaunchKernelGGL(chan_sums_f64_kernel, dim3(nch, K), dim3(256), 0, s, x, x_cs, ldx, R, C, valid, rb, ws, nch);
  hipLaunchKernelGGL(part_sum_f64_kernel<double>, dim3(K), dim3(1024), 0, s, (const double*)ws, nch, C, out, out_cs,
                     ldo);
}

void bn_coef_sums(const double* sums, long sums_cs, int ldp, const float* gamma, const float* beta,
                  const int* valid_rows, long g_cs, int K, int R, int C, float eps, int rep, float* mean, float* rstd,
                  float* coef, hipStream_t s) {
  // BN forward coefficients from running fp64 sums [K][2][ldp] (Σx, Σx² of each channel), read for
  // the first C channels: no pass over x (DenseNet: a channel's statistics are the same for every
  // later layer that normalises it, so they are summed once, from the producing conv's epilogue)
  using TT = float;
  launch_coef<TT, double>(dim3(cdiv(C, 32), K), s, sums, 1, gamma, beta, valid_rows, (const float*)nullptr,
                          (const float*)nullptr, mean, rstd, coef, (float*)nullptr, (float*)nullptr, 0L, g_cs, K, R, C,
                          eps, rep, 0, ldp, sums_cs);
}

long col_sum_workspace_floats(int K, long rows, int C) {
  const int rpb = rows_per_block(rows, K);
  return (long)K * cdiv(rows, rpb) * C;
}

void col_sum(const void* x, float* out, long out_cs, int K, long rows, int C, int f32, hipStream_t s, float* ws) {
  // ws (col_sum_workspace_floats): per-workgroup partials folded in order into out (any prior
  // contents overwritten, deterministic); without ws, atomics into out (zeroed by the caller)
  const int rpb = rows_per_block(rows, K);
  dim3 grid(cdiv(rows, rpb), K);
  const int V = vw(C);
  if (ws) {
    DISPATCH_T(f32, DISPATCH_V(V, hipLaunchKernelGGL((chan_reduce_kernel<TT, VV, 3>), grid, dim3(256), 0, s, CP(x),
                                                     nullptr, nullptr, nullptr, nullptr, nullptr, (int)rows, C, 0, ws,
                                                     0L, rpb, nullptr, BNCoefArgs{}, C, C)));
    hipLaunchKernelGGL(part_sum_kernel, dim3(cdiv(C, 256), K), dim3(256), 0, s, ws, (int)grid.x, C, C, out,
                       (float*)nullptr, out_cs);
    return;
  }
  DISPATCH_T(f32, DISPATCH_V(V, hipLaunchKernelGGL((chan_reduce_kernel<TT, VV, 2>), grid, dim3(256), 0, s, CP(x),
                                                   nullptr, nullptr, nullptr, nullptr, nullptr, (int)rows, C, 0, out,
                                                   out_cs, rpb, nullptr, BNCoefArgs{}, C, C)));
}

void ln_fwd(const void* x, const void* gamma, const void* beta, void* y, float* mean, float* rstd, long g_cs, int K,
            long rpc, int C, float eps, int rep, int f32, hipStream_t s, bf16_t* yp) {
  const long nrows = (long)K * rpc;
  // (column pairs per lane: 0.39 → 0.24 ms at 25 × 8192 × 512, profiles/r5_c25_ab_layernorm.txt)
  const bool pairs = f32 && (C == 512 || C == 1024) && (rep == 1 || g_cs % 2 == 0);
  if (pairs) {
    const float* xf = static_cast<const float*>(x);
    if (C == 512)
      hipLaunchKernelGGL((ln_fwd_pairs_kernel<4>), dim3(cdiv(nrows, 4)), dim3(256), 0, s, xf,
                         static_cast<const float*>(gamma), static_cast<const float*>(beta), static_cast<float*>(y),
                         mean, rstd, g_cs, nrows, rpc, C, eps, rep, yp);
    else
      hipLaunchKernelGGL((ln_fwd_pairs_kernel<8>), dim3(cdiv(nrows, 4)), dim3(256), 0, s, xf,
                         static_cast<const float*>(gamma), static_cast<const float*>(beta), static_cast<float*>(y),
                         mean, rstd, g_cs, nrows, rpc, C, eps, rep, yp);
    return;
  }
  DISPATCH_T(f32, hipLaunchKernelGGL(ln_fwd_kernel<TT>, dim3(cdiv(nrows, 4)), dim3(256), 0, s, CP(x), CP(gamma),
                                     CP(beta), MP(y), mean, rstd, g_cs, nrows, rpc, C, eps, rep, f32 ? yp : nullptr));
}

static int ln_rows_per_wave(long rpc) {
  return rpc >= 4096 ? 128 : 16;  // (128: bench/ln_bench.py 0.33 -> 0.28 ms vs 64)
}

long ln_workspace_floats(int K, long rpc, int C) {
  const long waves = (rpc + ln_rows_per_wave(rpc) - 1) / ln_rows_per_wave(rpc);
  return (long)K * cdiv(waves, 4) * 4 * 2 * C;
}

void ln_bwd(const void* dy, const void* x, const float* mean, const float* rstd, const void* gamma, long g_cs, int K,
            long rpc, int C, void* dx, float* dgamma, float* dbeta, long dg_cs, float* ws, int f32, hipStream_t s) {
  // ws (ln_workspace_floats): per-wave dγ / dβ partials folded in wave order (deterministic,
  // overwrites dgamma / dbeta); without ws, atomics into zeroed dgamma / dbeta
  const int rows_per_wave = ln_rows_per_wave(rpc);
  const long waves = (rpc + rows_per_wave - 1) / rows_per_wave;
  dim3 grid(cdiv(waves, 4), K);
  if (C <= 512) {
    DISPATCH_T(f32, hipLaunchKernelGGL((ln_bwd_kernel<TT, 8>), grid, dim3(256), 0, s, CP(dy), CP(x), mean, rstd,
                                       CP(gamma), g_cs, rpc, C, MP(dx), dgamma, dbeta, dg_cs, rows_per_wave, ws));
  } else {
    DISPATCH_T(f32, hipLaunchKernelGGL((ln_bwd_kernel<TT, LN_MAXC>), grid, dim3(256), 0, s, CP(dy), CP(x), mean,
                                       rstd, CP(gamma), g_cs, rpc, C, MP(dx), dgamma, dbeta, dg_cs, rows_per_wave, ws));
  }
  if (ws)
    hipLaunchKernelGGL(part_sum_kernel, dim3(cdiv(C, 256), K), dim3(256), 0, s, ws, (int)grid.x * 4, 2 * C, C, dgamma,
                       dbeta, dg_cs);
}
