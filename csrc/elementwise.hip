// Memory-bound kernels (gfx950): pooling, global-average-pool, fused softmax-CE fwd+bwd,
// the fused optimiser steps over flat [K, P] client buffers, FedAvg weighted row reductions,
// and the transport-compression kernels (dropout masks, stochastic quantisation, 1-bit sign
// pack / majority vote). All vectorised to 16-B accesses where the layout allows.
#include <algorithm>

#include "common.h"
#include "sgd_epi.h"
#include "dls.h"
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace {

// ------------------------------------------------------------------ pooling (NHWC)
// mode 0 = max (records argmax as flat input spatial index), 1 = average
template <typename T>
__global__ void pool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int* __restrict__ idx,
                                long total, int H, int W, int C, int OH, int OW, int k, int stride, int pad,
                                int mode) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % C;
  long t = i / C;
  const int ow = t % OW;
  t /= OW;
  const int oh = t % OH;
  const long img = t / OH;
  const T* xi = x + img * H * W * C;
  float best = -INFINITY, acc = 0.f;
  int bi = -1;
  for (int a = 0; a < k; ++a) {
    const int ih = oh * stride - pad + a;
    if (ih < 0 || ih >= H) continue;
    for (int b = 0; b < k; ++b) {
      const int iw = ow * stride - pad + b;
      if (iw < 0 || iw >= W) continue;
      const float v = ldf(xi + ((long)ih * W + iw) * C + c);
      if (mode == 0) {
        if (v > best) {
          best = v;
          bi = ih * W + iw;
        }
      } else {
        acc += v;
      }
    }
  }
  if (mode == 0) {
    stf(y + i, best);
    idx[i] = bi;
  } else {
    stf(y + i, acc / (float)(k * k));
  }
}

// gather-form backward (no atomics): each input element sums the windows that cover it
template <typename T>
__global__ void pool_bwd_kernel(const T* __restrict__ dy, const int* __restrict__ idx, T* __restrict__ dx,
                                long total, int H, int W, int C, int OH, int OW, int k, int stride, int pad,
                                int mode) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % C;
  long t = i / C;
  const int iw = t % W;
  t /= W;
  const int ih = t % H;
  const long img = t / H;
  const long obase = img * OH * OW * C;
  float acc = 0.f;
  const int oh_lo = max(0, (ih + pad - k + stride) / stride), oh_hi = min(OH - 1, (ih + pad) / stride);
  const int ow_lo = max(0, (iw + pad - k + stride) / stride), ow_hi = min(OW - 1, (iw + pad) / stride);
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    if (ih + pad - oh * stride < 0 || ih + pad - oh * stride >= k) continue;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      if (iw + pad - ow * stride < 0 || iw + pad - ow * stride >= k) continue;
      const long o = obase + ((long)oh * OW + ow) * C + c;
      if (mode == 0) {
        if (idx[o] == ih * W + iw) acc += ldf(dy + o);
      } else {
        acc += ldf(dy + o) / (float)(k * k);
      }
    }
  }
  stf(dx + i, acc);
}

// 8-channel form (C % 8 == 0): one thread per (input pixel, 8 channels) — 16-B dy loads and dx
// stores, 2 × 16-B index loads per window, one window-range computation per 8 channels (the
// scalar form is integer-divide and 2-B-access bound: ResNet-50's 112² stem pool, 12 ms/call)
template <typename T>
__global__ void __launch_bounds__(256) pool_bwd8_kernel(const T* __restrict__ dy, const int* __restrict__ idx,
                                                        T* __restrict__ dx, long total8, int H, int W, int C,
                                                        int OH, int OW, int k, int stride, int pad, int mode) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total8) return;
  const int C8 = C >> 3;
  const int c0 = (int)(i % C8) * 8;
  const long pix = i / C8;  // (img, ih, iw)
  const int iw = (int)(pix % W);
  const long t = pix / W;
  const int ih = (int)(t % H);
  const long img = t / H;
  const long obase = img * OH * OW * C + c0;
  const int me = ih * W + iw;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const int oh_lo = max(0, (ih + pad - k + stride) / stride), oh_hi = min(OH - 1, (ih + pad) / stride);
  const int ow_lo = max(0, (iw + pad - k + stride) / stride), ow_hi = min(OW - 1, (iw + pad) / stride);
  const float inv = 1.f / (float)(k * k);
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    if (ih + pad - oh * stride < 0 || ih + pad - oh * stride >= k) continue;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      if (iw + pad - ow * stride < 0 || iw + pad - ow * stride >= k) continue;
      const long o = obase + ((long)oh * OW + ow) * C;
      float g[8];
      load_vec<8>(dy + o, g);
      if (mode == 0) {
        const int4 a = *reinterpret_cast<const int4*>(idx + o);
        const int4 b = *reinterpret_cast<const int4*>(idx + o + 4);
        const int id[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += id[j] == me ? g[j] : 0.f;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += g[j] * inv;
      }
    }
  }
  store_vec<8>(dx + pix * C + c0, acc);
}

// global average pool: [KB][HW][C] -> [KB][C]
template <typename T>
__global__ void gap_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int HW, int C, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long img = i / C;
  const int c = i % C;
  const T* p = x + img * HW * C + c;
  float s = 0.f;
  for (int j = 0; j < HW; ++j) s += ldf(p + (long)j * C);
  stf(y + i, s / HW);
}

template <typename T>
__global__ void gap_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int HW, int C, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % C;
  const long img = i / ((long)HW * C);
  stf(dx + i, ldf(dy + img * C + c) / HW);
}

// fused softmax cross-entropy: one wave per sample row; per-client mean over valid rows.
// Writes loss[K] (mean), correct[K] and dlogits = (softmax - onehot)/n_k (0 on padded rows).
template <typename T>
__global__ void __launch_bounds__(256) ce_kernel(const T* __restrict__ logits, const int* __restrict__ labels,
                                                 const int* __restrict__ valid, float* __restrict__ loss,
                                                 float* __restrict__ correct, T* __restrict__ dlogits, int B,
                                                 int NC, float* __restrict__ rowbuf) {
  const int k = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const int nv = valid ? valid[k] : B;
  const long off = ((long)k * B + row) * NC;
  if (row >= nv) {
    for (int c = lane; c < NC; c += 64) stf(dlogits + off + c, 0.f);
    if (rowbuf && lane == 0) rowbuf[(long)k * B + row] = rowbuf[((long)gridDim.y + k) * B + row] = 0.f;
    return;
  }
  const float inv_n = 1.f / (float)max(nv, 1);
  float mx = -INFINITY;
  int amax = 0;
  for (int c = lane; c < NC; c += 64) {
    const float v = ldf(logits + off + c);
    if (v > mx) {
      mx = v;
      amax = c;
    }
  }
  // wave argmax (first max index on ties)
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oi = __shfl_xor(amax, o, 64);
    if (om > mx || (om == mx && oi < amax)) {
      mx = om;
      amax = oi;
    }
  }
  float se = 0.f;
  for (int c = lane; c < NC; c += 64) se += expf(ldf(logits + off + c) - mx);
  se = wave_sum(se);
  const float lse = mx + logf(se);
  const int lab = labels[(long)k * B + row];
  for (int c = lane; c < NC; c += 64) {
    const float pr = expf(ldf(logits + off + c) - lse);
    stf(dlogits + off + c, (pr - (c == lab ? 1.f : 0.f)) * inv_n);
  }
  if (lane == 0) {
    const float nll = lse - ldf(logits + off + lab);
    if (rowbuf) {  // per-row terms, summed in row order by ce_fold_kernel (deterministic)
      rowbuf[(long)k * B + row] = nll * inv_n;
      rowbuf[((long)gridDim.y + k) * B + row] = amax == lab ? 1.f : 0.f;
    } else {
      atomicAdd(&loss[k], nll * inv_n);
      if (amax == lab) atomicAdd(&correct[k], 1.f);
    }
  }
}

// loss[k] = Σ_row rowbuf[0][k][row], correct[k] = Σ_row rowbuf[1][k][row], rows in order
__global__ void ce_fold_kernel(const float* __restrict__ rowbuf, float* __restrict__ loss, float* __restrict__ correct,
                               int K, int B) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float a = 0.f, c = 0.f;
  for (int r = 0; r < B; ++r) {
    a += rowbuf[(long)k * B + r];
    c += rowbuf[((long)K + k) * B + r];
  }
  loss[k] = a;
  correct[k] = c;
}

template <typename T>
__global__ void relu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = ldf(y + i) > 0.f ? dy[i] : (T)0;
}

// ------------------------------------------------------------- optimiser steps
// grid: (chunks of P/4, K). float4 over the row; per-client lr / active / first-step flags.
// split[k] row = [hi plane (ld)][lo plane (ld)] bf16 of theta[k] (the fp32 GEMMs' pre-split
// weight operand, ConvNTParams::wsplit): 4 consecutive values → 8 B of hi + 8 B of lo
__device__ __forceinline__ void store_split4(bf16_t* __restrict__ split, long k, long ld, long i, const float* v) {
  uint32_t h0, l0, h1, l1;
  split_pair(v[0], v[1], h0, l0);
  split_pair(v[2], v[3], h1, l1);
  bf16_t* sp = split + k * 2 * ld;
  reinterpret_cast<uint2*>(sp)[i] = make_uint2(h0, h1);
  reinterpret_cast<uint2*>(sp + ld)[i] = make_uint2(l0, l1);
}

__global__ void __launch_bounds__(256) split_rows_kernel(const float* __restrict__ theta, bf16_t* __restrict__ split,
                                                         long P4, long ld) {
  const int k = blockIdx.y;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P4; i += (long)gridDim.x * blockDim.x) {
    const float4 t = reinterpret_cast<const float4*>(theta + (long)k * ld)[i];
    const float v[4] = {t.x, t.y, t.z, t.w};
    store_split4(split, k, ld, i, v);
  }
}

// split planes of rows of C values zero-padded to C32 (DenseNet growth-conv weights for the halo
// kernel, which stages whole 32-channel chunks): out[k][p][r][c] = split_p(c < C ? w[k][r][c] : 0),
// one launch instead of a zero fill, a strided copy and the split pass
__global__ void __launch_bounds__(256) split_rows_padded_kernel(const float* __restrict__ w, long w_cs, int rows, int C,
                                                                int C32, bf16_t* __restrict__ out) {
  const int k = blockIdx.y;
  const long n = (long)rows * C32;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int r = (int)(i / C32), c = (int)(i - (long)r * C32);
  const float v = c < C ? w[(long)k * w_cs + (long)r * C + c] : 0.f;
  bf16_t hi, lo;
  split2(v, hi, lo);
  out[(long)k * 2 * n + i] = hi;
  out[(long)k * 2 * n + n + i] = lo;
}

// SEG: the flat step over the spans of a block table (seg[blockIdx.x] = (first float4, count)):
// the parameters whose gradients did not already step themselves (SgdEpi, sgd_epi.h)
template <bool SEG>
__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ theta, const float* __restrict__ grad,
                                                  float* __restrict__ mom, bf16_t* __restrict__ shadow,
                                                  bf16_t* __restrict__ split,
                                                  const float* __restrict__ lr, const uint8_t* __restrict__ active,
                                                  const uint8_t* __restrict__ first, long P4, long ld, float wd,
                                                  float momentum, float dampening, int nesterov,
                                                  const long2* __restrict__ seg) {
  const int k = blockIdx.y;
  if (!active[k]) return;
  const float a = lr[k];
  const bool fs = first[k] != 0;
  const long base = (long)k * ld;
  SgdEpi e{};
  e.wd = wd;
  e.momentum = momentum;
  e.dampening = dampening;
  e.nesterov = nesterov;
  long beg, end, stride;
  if constexpr (SEG) {
    const long2 b = seg[blockIdx.x];
    beg = b.x + threadIdx.x;
    end = b.x + b.y;
    stride = blockDim.x;
  } else {
    beg = (long)blockIdx.x * blockDim.x + threadIdx.x;
    end = P4;
    stride = (long)gridDim.x * blockDim.x;
  }
  // two float4 per thread per trip, both loaded before either is stored: the stores of one trip
  // would otherwise order the next trip's loads behind them (one HBM round trip per float4)
  for (long i0 = beg; i0 < end; i0 += 2 * stride) {
    float4 t[2], g[2], m[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long i = i0 + u * stride;
      if (i < end) {
        t[u] = reinterpret_cast<float4*>(theta + base)[i];
        g[u] = reinterpret_cast<const float4*>(grad + base)[i];
        if (momentum != 0.f) m[u] = reinterpret_cast<float4*>(mom + base)[i];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long i = i0 + u * stride;
      if (i >= end) break;
      float tv[4] = {t[u].x, t[u].y, t[u].z, t[u].w}, gv[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
      float mv[4] = {0.f, 0.f, 0.f, 0.f};
      if (momentum != 0.f) {
        mv[0] = m[u].x;
        mv[1] = m[u].y;
        mv[2] = m[u].z;
        mv[3] = m[u].w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) tv[j] = sgd_epi_core(e, fs, a, tv[j], gv[j], mv[j]);
      reinterpret_cast<float4*>(theta + base)[i] = make_float4(tv[0], tv[1], tv[2], tv[3]);
      if (momentum != 0.f) reinterpret_cast<float4*>(mom + base)[i] = make_float4(mv[0], mv[1], mv[2], mv[3]);
      if (shadow) {
        uint2 uu;
        uu.x = (uint32_t)f2bf(tv[0]) | ((uint32_t)f2bf(tv[1]) << 16);
        uu.y = (uint32_t)f2bf(tv[2]) | ((uint32_t)f2bf(tv[3]) << 16);
        reinterpret_cast<uint2*>(shadow + base)[i] = uu;
      }
      if (split) store_split4(split, k, ld, i, tv);
    }
  }
}

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ theta, const float* __restrict__ grad,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ shadow, const float* __restrict__ lr,
                                                   const uint8_t* __restrict__ active, const float* __restrict__ step,
                                                   long P, long ld, float b1, float b2, float eps, float wd) {
  const int k = blockIdx.y;
  if (!active[k]) return;
  const float a = lr[k];
  const float t = step[k];
  const float c1 = 1.f - __powf(b1, t), c2 = 1.f - __powf(b2, t);
  const long base = (long)k * ld;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    const float th = theta[base + i];
    const float g = grad[base + i] + wd * th;
    const float mm = b1 * m[base + i] + (1.f - b1) * g;
    const float vv = b2 * v[base + i] + (1.f - b2) * g * g;
    m[base + i] = mm;
    v[base + i] = vv;
    const float nt = th - a * (mm / c1) / (sqrtf(vv / c2) + eps);
    theta[base + i] = nt;
    if (shadow) shadow[base + i] = f2bf(nt);
  }
}

__global__ void broadcast_kernel(float* __restrict__ theta, bf16_t* __restrict__ shadow,
                                 const float* __restrict__ src, long P4, long ld) {
  const int k = blockIdx.y;
  const long base = (long)k * ld;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P4; i += (long)gridDim.x * blockDim.x) {
    const float4 s = reinterpret_cast<const float4*>(src)[i];
    reinterpret_cast<float4*>(theta + base)[i] = s;
    if (shadow) {
      uint2 u;
      u.x = (uint32_t)f2bf(s.x) | ((uint32_t)f2bf(s.y) << 16);
      u.y = (uint32_t)f2bf(s.z) | ((uint32_t)f2bf(s.w) << 16);
      reinterpret_cast<uint2*>(shadow + base)[i] = u;
    }
  }
}

__global__ void delta_kernel(const float* __restrict__ theta, const float* __restrict__ base_p,
                             float* __restrict__ out, long P4, long ld) {
  const int k = blockIdx.y;
  const long base = (long)k * ld;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P4; i += (long)gridDim.x * blockDim.x) {
    const float4 t = reinterpret_cast<const float4*>(theta + base)[i];
    const float4 b = reinterpret_cast<const float4*>(base_p)[i];
    reinterpret_cast<float4*>(out + base)[i] = make_float4(t.x - b.x, t.y - b.y, t.z - b.z, t.w - b.w);
  }
}

// out[:] += Σ_k w_k x[k, :] in fp64 (reference FedAvg accumulates float64(θ)·n, fed_avg_algorithm.py:
// 39-52): the fp64 accumulator stays fp64 across cohorts and the RCCL all-reduce; fixed k order
__global__ void __launch_bounds__(256) weighted_sum_kernel(const float* __restrict__ x, const double* __restrict__ w,
                                                           double* __restrict__ out, int K, long P4, long ld) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P4; i += (long)gridDim.x * blockDim.x) {
    double4 a = reinterpret_cast<double4*>(out)[i];
    for (int k = 0; k < K; ++k) {
      const float4 v = reinterpret_cast<const float4*>(x + (long)k * ld)[i];
      const double wk = w[k];
      a.x += wk * v.x;
      a.y += wk * v.y;
      a.z += wk * v.z;
      a.w += wk * v.w;
    }
    reinterpret_cast<double4*>(out)[i] = a;
  }
}

// Subset-model mixing for Shapley utilities: out[m, :] = Σ_k W[m, k]·x[k, :] for a
// slice of ≤ 32 subset models per blockIdx.y, written straight in the bf16 compute dtype the
// batched evaluation consumes. Each x row is read once per 32 models (a per-subset weighted
// sum re-reads all K rows for every model); fp32 accumulation, W staged in LDS.
constexpr int MIX_M = 32;
constexpr int MIX_KMAX = 256;
template <typename T>
__global__ void __launch_bounds__(256) mix_rows_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                       T* __restrict__ out, int K, int M, long P4, long ld,
                                                       long ld_out) {
  __shared__ float wl[MIX_M * MIX_KMAX];
  const int m0 = blockIdx.y * MIX_M;
  const int mn = min(MIX_M, M - m0);
  for (int t = threadIdx.x; t < MIX_M * K; t += blockDim.x) wl[t] = t < mn * K ? w[(long)m0 * K + t] : 0.f;
  __syncthreads();
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P4; i += (long)gridDim.x * blockDim.x) {
    float acc[MIX_M][4];
#pragma unroll
    for (int m = 0; m < MIX_M; ++m) acc[m][0] = acc[m][1] = acc[m][2] = acc[m][3] = 0.f;
    for (int k = 0; k < K; ++k) {
      const float4 v = reinterpret_cast<const float4*>(x + (long)k * ld)[i];
#pragma unroll
      for (int m = 0; m < MIX_M; ++m) {
        const float c = wl[m * K + k];  // wave-uniform address: LDS broadcast
        acc[m][0] = fmaf(c, v.x, acc[m][0]);
        acc[m][1] = fmaf(c, v.y, acc[m][1]);
        acc[m][2] = fmaf(c, v.z, acc[m][2]);
        acc[m][3] = fmaf(c, v.w, acc[m][3]);
      }
    }
#pragma unroll
    for (int m = 0; m < MIX_M; ++m) {
      if (m < mn) store_vec<4>(out + (long)(m0 + m) * ld_out + 4 * i, acc[m]);
    }
  }
}

// FedDropoutAvg: num[:] += Σ_k w_k m_k x_k, den[:] += Σ_k w_k m_k (fp64, accumulated in place)
__global__ void masked_weighted_sum_kernel(const float* __restrict__ x, const uint8_t* __restrict__ mask,
                                           const double* __restrict__ w, double* __restrict__ num,
                                           double* __restrict__ den, int K, long P, long ld) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    double a = num[i], d = den[i];
    for (int k = 0; k < K; ++k) {
      if (mask[(long)k * ld + i]) {
        a += w[k] * x[(long)k * ld + i];
        d += w[k];
      }
    }
    num[i] = a;
    den[i] = d;
  }
}

// Per-row seeds are derived from the CLIENT id (not its row position), so masks / rounding
// noise are identical whatever rank or wave hosts the client (matches ops.fl.uniform_rows).
__global__ void dropout_mask_kernel(uint8_t* __restrict__ mask, long P, float p, const uint32_t* __restrict__ seeds,
                                    long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long k = i / P, e = i - k * P;
  const uint32_t h = mix32((uint32_t)(e & 0xffffffffu), seeds[k]);
  mask[i] = ((float)h * (1.f / 4294967296.f)) >= p;
}

// Σ x² per (client, block). Every tensor starts 16-element aligned in the flat layout and
// inter-tensor padding is zero, so a lane's 16-element chunk belongs to the block of its first
// element. Lanes hold consecutive chunks → segmented wave reduction → one atomic per run.
__global__ void __launch_bounds__(256) block_sq_kernel(const float* __restrict__ x, const int* __restrict__ ids,
                                                       float* __restrict__ out, long P, long ld, int nb) {
  const int k = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const long nchunk = P / 16;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long c0 = (long)blockIdx.x * blockDim.x; c0 < nchunk; c0 += stride) {
    const long c = c0 + threadIdx.x;
    int b = -1;
    float s = 0.f;
    if (c < nchunk) {
      b = ids[c * 16];
      const float4* p = reinterpret_cast<const float4*>(x + (long)k * ld + c * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 v = p[j];
        s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      }
    }
    for (int o = 1; o < 64; o <<= 1) {
      const int bo = __shfl_down(b, o, 64);
      const float so = __shfl_down(s, o, 64);
      if (lane + o < 64 && bo == b) s += so;
    }
    const int bprev = __shfl_up(b, 1, 64);
    if (b >= 0 && (lane == 0 || bprev != b)) atomicAdd(&out[(long)k * nb + b], s);
  }
}

__global__ void seg_minmax_kernel(const float* __restrict__ x, const int* __restrict__ seg, float* __restrict__ mn,
                                  float* __restrict__ mx, long P, long ld, int nseg) {
  // per block: a contiguous range; reduce runs of equal segment id within each wave
  const int k = blockIdx.y;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int s = (i < P) ? seg[i] : -1;
  float lo = (i < P) ? x[(long)k * ld + i] : INFINITY;
  float hi = (i < P) ? x[(long)k * ld + i] : -INFINITY;
  // segmented wave reduction (segments are contiguous, so equal ids are adjacent)
  for (int o = 1; o < 64; o <<= 1) {
    const int so = __shfl_down(s, o, 64);
    const float lo2 = __shfl_down(lo, o, 64), hi2 = __shfl_down(hi, o, 64);
    if (lane + o < 64 && so == s) {
      lo = fminf(lo, lo2);
      hi = fmaxf(hi, hi2);
    }
  }
  const int sprev = __shfl_up(s, 1, 64);
  if (s >= 0 && (lane == 0 || sprev != s)) {
    // float atomics on min/max via int ordering trick
    float* pmn = &mn[(long)k * nseg + s];
    float* pmx = &mx[(long)k * nseg + s];
    int* imn = reinterpret_cast<int*>(pmn);
    int* imx = reinterpret_cast<int*>(pmx);
    if (lo >= 0)
      atomicMin(imn, __float_as_int(lo));
    else
      atomicMax(reinterpret_cast<unsigned*>(imn), __float_as_uint(lo)), (void)0;
    if (hi >= 0)
      atomicMax(imx, __float_as_int(hi));
    else
      atomicMin(reinterpret_cast<unsigned*>(imx), __float_as_uint(hi));
  }
}

__global__ void stochastic_qdq_kernel(float* __restrict__ x, const int* __restrict__ seg,
                                      const float* __restrict__ mn, const float* __restrict__ mx, long P, long ld,
                                      int nseg, const uint32_t* __restrict__ seeds, int levels) {
  const int k = blockIdx.y;
  const uint32_t seed = seeds[k];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    const int s = seg[i];
    const float lo = mn[(long)k * nseg + s];
    const float sc = fmaxf((mx[(long)k * nseg + s] - lo) / levels, 1e-30f);
    const long gi = (long)k * ld + i;
    const float u = (float)mix32((uint32_t)(i & 0xffffffffu), seed) * (1.f / 4294967296.f);
    float q = floorf((x[gi] - lo) / sc + u);
    q = fminf(fmaxf(q, 0.f), (float)levels);
    x[gi] = lo + q * sc;
  }
}

// NNADQ (FedOBD): deterministic per-(client, tensor) quantisation with an adaptive level count;
// lo / scale / levels are per (row, segment). Writes the dequantised value in place.
__global__ void nnadq_qdq_kernel(float* __restrict__ x, const int* __restrict__ seg, const float* __restrict__ lo,
                                 const float* __restrict__ scale, const float* __restrict__ levels, long P, long ld,
                                 int nseg) {
  const int k = blockIdx.y;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    const long q0 = (long)k * nseg + seg[i];
    const float l = lo[q0], sc = scale[q0];
    const long gi = (long)k * ld + i;
    float q = rintf((x[gi] - l) / sc);
    q = fminf(fmaxf(q, 0.f), levels[q0]);
    x[gi] = l + q * sc;
  }
}

// dropout on [K][rows][N] (row stride ld): the GEMM epilogue's mask rule (common.h drop_keep)
template <typename T>
__global__ void dropout_apply_kernel(const T* __restrict__ x, T* __restrict__ out, long rows, int N, long ld,
                                     const uint32_t* __restrict__ seeds, float p, float scale) {
  const int k = blockIdx.y;
  const uint32_t seed = seeds[k];
  const long total = rows * (long)N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long m = i / N;
    const int n = (int)(i - m * N);
    const long o = ((long)k * rows + m) * ld + n;
    const float v = ldf(x + o);
    stf(out + o, drop_keep(seed, m, N, n, p) ? v * scale : 0.f);
  }
}

// the same mask on fp32 [K][rows][N] (contiguous), writing the result's split planes
// [K][2][rows][N] (hi, lo) and, when out != nullptr, the fp32 values too; two columns a lane
// grid (row blocks of DP_RB rows, K): thread t owns column pairs t, t + 256, ... and walks the
// block's rows (no per-element division); with `part` it also sums its columns over those rows
// (the consuming linear's bias gradient: [K][row blocks][N] partials, folded in order)
constexpr int DP_RB = 64;
__global__ void __launch_bounds__(256) dropout_planes_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                             bf16_t* __restrict__ yp, long rows, int N,
                                                             const uint32_t* __restrict__ seeds, float p, float scale,
                                                             float* __restrict__ part) {
  const int k = blockIdx.y;
  const uint32_t seed = seeds[k];
  const int N2 = N / 2;
  const long r0 = (long)blockIdx.x * DP_RB, r1 = min(rows, r0 + DP_RB);
  const float2* xk = reinterpret_cast<const float2*>(x + (long)k * rows * N);
  float2* ok = out ? reinterpret_cast<float2*>(out + (long)k * rows * N) : nullptr;
  uint32_t* hk = reinterpret_cast<uint32_t*>(yp + (long)k * 2 * rows * N);
  uint32_t* lk = hk + rows * (long)N / 2;
  for (int c2 = threadIdx.x; c2 < N2; c2 += 256) {
    const int n = 2 * c2;
    float sx = 0.f, sy = 0.f;
    for (long m = r0; m < r1; ++m) {
      const long i = m * N2 + c2;
      float2 v = xk[i];
      v.x = drop_keep(seed, m, N, n, p) ? v.x * scale : 0.f;
      v.y = drop_keep(seed, m, N, n + 1, p) ? v.y * scale : 0.f;
      if (ok) ok[i] = v;
      uint32_t h, l;
      split_pair(v.x, v.y, h, l);
      hk[i] = h;
      lk[i] = l;
      sx += v.x;
      sy += v.y;
    }
    if (part) {
      float* pr = part + ((long)k * gridDim.x + blockIdx.x) * N;
      pr[n] = sx;
      pr[n + 1] = sy;
    }
  }
}

// procedural synthetic images (data/datasets.py SyntheticImages._generate, bit-identical):
// h = lowbias32(idx·0x9E3779B1 + p·0x85EBCA77 + salt), h2 = lowbias32(h + 0x68E31DA4),
// x = proto[class][p] + ((h + h2)·2^-32 − 1)·√6·noise, channels zero-padded C → Cout
__device__ __forceinline__ uint64_t lowbias32(uint64_t x) {
  x &= 0xFFFFFFFFull;
  x ^= x >> 16;
  x = (x * 0x7FEB352Dull) & 0xFFFFFFFFull;
  x ^= x >> 15;
  x = (x * 0x846CA68Bull) & 0xFFFFFFFFull;
  return x ^ (x >> 16);
}

__global__ void synth_images_kernel(const int64_t* __restrict__ idx, long n, long npix, int C, int Cout,
                                    const int* __restrict__ source, const float* __restrict__ proto,
                                    unsigned long long salt, float sqrt6, float noise, float* __restrict__ out) {
#pragma clang fp contract(off)
  const long per = npix / C * Cout;
  const long total = n * per;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long i = t / per, q = t - i * per;
    const long px = q / Cout;
    const int c = (int)(q - px * Cout);
    if (c >= C) {
      out[t] = 0.f;
      continue;
    }
    const long p = px * C + c;
    const uint64_t id = (uint64_t)idx[i];
    const uint64_t h = lowbias32(id * 0x9E3779B1ull + (uint64_t)p * 0x85EBCA77ull + salt);
    const uint64_t h2 = lowbias32(h + 0x68E31DA4ull);
    const float u = ((float)h + (float)h2) * (1.f / 4294967296.f) - 1.f;
    const float nz = (u * sqrt6) * noise;
    out[t] = proto[(long)source[id] * npix + p] + nz;
  }
}

__global__ void sign_pack_kernel(const float* __restrict__ g, uint8_t* __restrict__ out, long P, long ld,
                                 long nbytes) {
  const int k = blockIdx.y;
  for (long j = (long)blockIdx.x * blockDim.x + threadIdx.x; j < nbytes; j += (long)gridDim.x * blockDim.x) {
    uint32_t b = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const long i = j * 8 + t;
      if (i < P && g[(long)k * ld + i] >= 0.f) b |= 1u << t;
    }
    out[(long)k * nbytes + j] = (uint8_t)b;
  }
}

__global__ void sign_vote_kernel(const uint8_t* __restrict__ packed, const uint8_t* __restrict__ active,
                                 int* __restrict__ votes, int K, long P, long nbytes) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    int v = 0;
    for (int k = 0; k < K; ++k) {
      if (active && !active[k]) continue;
      v += ((packed[(long)k * nbytes + (i >> 3)] >> (i & 7)) & 1) ? 1 : -1;
    }
    votes[i] = v;
  }
}

// out[k, t, :] = table[k / rep][tok[k, t], :] · scale (+ pe[t mod L, :]): the Transformer's
// embedding lookup, √d scaling and positional-encoding add in one pass
template <typename T>
__global__ void embedding_fwd_kernel(const int* __restrict__ tok, const T* __restrict__ table,
                                     T* __restrict__ out, long n_tok, int D, long t_cs, int rep, long total, float scale,
                                     const float* __restrict__ pe, int L) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long row = i / D;
  const int d = i % D;
  const int k = (int)(row / n_tok);
  float v = ldf(table + (long)(k / rep) * t_cs + (long)tok[row] * D + d) * scale;
  if (pe) v += pe[(long)((row % n_tok) % L) * D + d];
  stf(out + i, v);
}

template <typename T>
__global__ void embedding_bwd_kernel(const int* __restrict__ tok, const T* __restrict__ dy,
                                     float* __restrict__ dtable, long n_tok, int D, long t_cs, long total, float scale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long row = i / D;
  const int d = i % D;
  const int k = (int)(row / n_tok);
  atomicAdd(&dtable[(long)k * t_cs + (long)tok[row] * D + d], ldf(dy + i) * scale);
}

// Deterministic embedding backward: rows sorted by key = client·V + token (stable, so equal keys
// keep their sequence order); the wave of a segment's first row sums the segment's dY rows in
// that order and writes the table row once — no atomics, bitwise-reproducible
template <typename T>
__global__ void __launch_bounds__(256) embedding_bwd_sorted_kernel(const int* __restrict__ keys,
                                                                   const int* __restrict__ order,
                                                                   const T* __restrict__ dy, float* __restrict__ dtable,
                                                                   long n, int D, int V, long t_cs, float scale) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const int key = keys[r];
  if (r > 0 && keys[r - 1] == key) return;
  const int k = key / V, tok = key - k * V;
  float* out = dtable + (long)k * t_cs + (long)tok * D;
  for (int d0 = 0; d0 < D; d0 += 64 * 4) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (long i = r; i < n && keys[i] == key; ++i) {
      const T* row = dy + (long)order[i] * D;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = d0 + j * 64 + lane;
        if (d < D) acc[j] += ldf(row + d);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = d0 + j * 64 + lane;
      if (d < D) out[d] = acc[j] * scale;
    }
  }
}

// Chunked form for skewed token counts (padding tokens: thousands of rows of one key per client,
// which the per-segment wave above sums serially). The sorted rows are cut into fixed chunks of
// EMB_CH rows, one wave each (A): a key run that starts and ends inside the chunk writes its
// table row; a run that started in an earlier chunk leaves its in-chunk sum in part[c][0], one
// that starts here and continues leaves it in part[c][1]. Then (B) the chunk where a continuing
// run starts adds the following chunks' part[·][0] in chunk order and writes the row. Fixed
// chunking and order: bitwise-reproducible, no atomics, no host sync.
constexpr int EMB_CH = 64;

__device__ __forceinline__ bool emb_run_starts(const int* keys, long rs, long cs, int key) {
  return rs > cs || rs == 0 || keys[rs - 1] != key;
}
__device__ __forceinline__ bool emb_run_ends(const int* keys, long re, long ce, long n, int key) {
  return re < ce || re >= n || keys[re] != key;
}

template <typename T>
__global__ void __launch_bounds__(256) embedding_bwd_chunk_kernel(const int* __restrict__ keys,
                                                                  const int* __restrict__ order,
                                                                  const T* __restrict__ dy,
                                                                  float* __restrict__ dtable,
                                                                  float* __restrict__ part, long n, int D, int V,
                                                                  long t_cs, float scale) {
  const long c = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long cs = c * EMB_CH;
  if (cs >= n) return;
  const long ce = min(n, cs + EMB_CH);
  for (int d0 = 0; d0 < D; d0 += 64 * 4) {
    long rs = cs;
    while (rs < ce) {
      const int key = keys[rs];
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      long re = rs;
      for (; re < ce && keys[re] == key; ++re) {
        const T* row = dy + (long)order[re] * D;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int d = d0 + j * 64 + lane;
          if (d < D) acc[j] += ldf(row + d);
        }
      }
      const bool st = emb_run_starts(keys, rs, cs, key), en = emb_run_ends(keys, re, ce, n, key);
      float* out;
      float sc = 1.f;
      if (st && en) {
        const int k = key / V, tok = key - k * V;
        out = dtable + (long)k * t_cs + (long)tok * D;
        sc = scale;
      } else {
        out = part + (c * 2 + (st ? 1 : 0)) * (long)D;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = d0 + j * 64 + lane;
        if (d < D) out[d] = acc[j] * sc;
      }
      rs = re;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) embedding_bwd_join_kernel(const int* __restrict__ keys,
                                                                 const float* __restrict__ part,
                                                                 float* __restrict__ dtable, long n, int D, int V,
                                                                 long t_cs, float scale) {
  const long c = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long cs = c * EMB_CH;
  if (cs >= n) return;
  const long ce = min(n, cs + EMB_CH);
  const int key = keys[ce - 1];  // the chunk's last run
  long rs = ce - 1;
  while (rs > cs && keys[rs - 1] == key) --rs;
  if (!emb_run_starts(keys, rs, cs, key) || emb_run_ends(keys, ce, ce, n, key)) return;
  const int k = key / V, tok = key - k * V;
  float* out = dtable + (long)k * t_cs + (long)tok * D;
  for (int d0 = 0; d0 < D; d0 += 64 * 4) {
    float acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = d0 + j * 64 + lane;
      acc[j] = d < D ? part[(c * 2 + 1) * (long)D + d] : 0.f;
    }
    for (long c2 = c + 1;; ++c2) {  // chunks the run continues into, in order
      const long cs2 = c2 * EMB_CH, ce2 = min(n, cs2 + EMB_CH);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = d0 + j * 64 + lane;
        if (d < D) acc[j] += part[(c2 * 2) * (long)D + d];
      }
      if (ce2 >= n || keys[ce2] != key || keys[ce2 - 1] != key) break;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = d0 + j * 64 + lane;
      if (d < D) out[d] = acc[j] * scale;
    }
  }
}

// masked mean over the sequence: y[s, :] = Σ_{t < len[s]} x[s, t, :] / max(len[s], 1)
template <typename T>
__global__ void seq_mean_fwd_kernel(const T* __restrict__ x, const int* __restrict__ len, T* __restrict__ y, int L,
                                    int D, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long s = i / D;
  const int d = i % D;
  const int n = min(len[s], L);
  float acc = 0.f;
  for (int t = 0; t < n; ++t) acc += ldf(x + (s * L + t) * D + d);
  stf(y + i, acc / (float)max(n, 1));
}

template <typename T>
__global__ void seq_mean_bwd_kernel(const T* __restrict__ dy, const int* __restrict__ len, T* __restrict__ dx, int L,
                                    int D, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int d = i % D;
  const long st = i / D;
  const int t = st % L;
  const long s = st / L;
  const int n = min(len[s], L);
  stf(dx + i, t < n ? ldf(dy + s * D + d) / (float)max(n, 1) : 0.f);
}

__global__ void gather_rows_kernel(const uint4* __restrict__ src, const int* __restrict__ idx,
                                   uint4* __restrict__ dst, long n, long row_vec8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * row_vec8) return;
  const long r = i / row_vec8, c = i % row_vec8;
  dst[i] = src[(long)idx[r] * row_vec8 + c];
}

int grid_for(long n, int per_block = 256, int cap = 4096) { return (int)max(1L, min((long)cap, (n + per_block - 1) / per_block)); }

}  // namespace

#define DISPATCH_T(F32, ...) \
  if (F32) {                 \
    typedef float TT;        \
    __VA_ARGS__;             \
  } else {                   \
    typedef bf16_t TT;       \
    __VA_ARGS__;             \
  }
#define CP(p) static_cast<const TT*>(p)
#define MP(p) static_cast<TT*>(p)

void pool_fwd(const void* x, void* y, int* idx, int K, int B, int H, int W, int C, int OH, int OW, int k, int stride,
              int pad, int mode, int f32, hipStream_t s) {
  const long total = (long)K * B * OH * OW * C;
  DISPATCH_T(f32, hipLaunchKernelGGL(pool_fwd_kernel<TT>, dim3(cdiv(total, 256)), dim3(256), 0, s, CP(x), MP(y), idx,
                                     total, H, W, C, OH, OW, k, stride, pad, mode));
}

void pool_bwd(const void* dy, const int* idx, void* dx, int K, int B, int H, int W, int C, int OH, int OW, int k,
              int stride, int pad, int mode, int f32, hipStream_t s) {
  const long total = (long)K * B * H * W * C;
  if (C % 8 == 0) {
    DISPATCH_T(f32, hipLaunchKernelGGL(pool_bwd8_kernel<TT>, dim3(cdiv(total / 8, 256)), dim3(256), 0, s, CP(dy), idx,
                                       MP(dx), total / 8, H, W, C, OH, OW, k, stride, pad, mode));
    return;
  }
  DISPATCH_T(f32, hipLaunchKernelGGL(pool_bwd_kernel<TT>, dim3(cdiv(total, 256)), dim3(256), 0, s, CP(dy), idx, MP(dx),
                                     total, H, W, C, OH, OW, k, stride, pad, mode));
}

void gap_fwd(const void* x, void* y, int KB, int HW, int C, int f32, hipStream_t s) {
  const long total = (long)KB * C;
  DISPATCH_T(f32, hipLaunchKernelGGL(gap_fwd_kernel<TT>, dim3(cdiv(total, 256)), dim3(256), 0, s, CP(x), MP(y), HW, C,
                                     total));
}

void gap_bwd(const void* dy, void* dx, int KB, int HW, int C, int f32, hipStream_t s) {
  const long total = (long)KB * HW * C;
  DISPATCH_T(f32, hipLaunchKernelGGL(gap_bwd_kernel<TT>, dim3(cdiv(total, 256)), dim3(256), 0, s, CP(dy), MP(dx), HW,
                                     C, total));
}

void ce_fwd_bwd(const void* logits, const int* labels, const int* valid, float* loss, float* correct, void* dlogits,
                int K, int B, int NC, int f32, hipStream_t s, float* rowbuf) {
  if (!rowbuf) {
    CHECK_HIP(hipMemsetAsync(loss, 0, sizeof(float) * K, s));
    CHECK_HIP(hipMemsetAsync(correct, 0, sizeof(float) * K, s));
  }
  DISPATCH_T(f32, hipLaunchKernelGGL(ce_kernel<TT>, dim3(cdiv(B, 4), K), dim3(256), 0, s, CP(logits), labels, valid,
                                     loss, correct, MP(dlogits), B, NC, rowbuf));
  if (rowbuf) hipLaunchKernelGGL(ce_fold_kernel, dim3(cdiv(K, 64)), dim3(64), 0, s, rowbuf, loss, correct, K, B);
}

void relu_bwd(const void* dy, const void* y, void* dx, long n, int f32, hipStream_t s) {
  DISPATCH_T(f32, hipLaunchKernelGGL(relu_bwd_kernel<TT>, dim3(cdiv(n, 256)), dim3(256), 0, s, CP(dy), CP(y), MP(dx),
                                     n));
}

void sgd_step(float* theta, const float* grad, float* mom, bf16_t* shadow, bf16_t* split, const float* lr,
              const uint8_t* active, const uint8_t* first, int K, long P, long ld, float wd, float momentum,
              float dampening, int nesterov, hipStream_t s) {
  const long P4 = P / 4;  // P is a multiple of 16 (layout alignment)
  dim3 grid(grid_for(P4, 256, 1024), K);
  hipLaunchKernelGGL(sgd_kernel<false>, grid, dim3(256), 0, s, theta, grad, mom, shadow, split, lr, active, first, P4,
                     ld, wd, momentum, dampening, nesterov, (const long2*)nullptr);
}

void sgd_step_seg(float* theta, const float* grad, float* mom, bf16_t* split, const float* lr, const uint8_t* active,
                  const uint8_t* first, int K, long ld, float wd, float momentum, float dampening, int nesterov,
                  const long2* seg, int nblocks, hipStream_t s) {
  if (K == 0 || nblocks == 0) return;
  hipLaunchKernelGGL(sgd_kernel<true>, dim3(nblocks, K), dim3(256), 0, s, theta, grad, mom, (bf16_t*)nullptr, split, lr,
                     active, first, 0L, ld, wd, momentum, dampening, nesterov, seg);
}

void split_rows_padded(const float* w, long w_cs, int K, int rows, int C, int C32, bf16_t* out, hipStream_t s) {
  const long n = (long)rows * C32;
  if (K == 0 || n == 0) return;
  hipLaunchKernelGGL(split_rows_padded_kernel, dim3((unsigned)cdiv(n, 256), K), dim3(256), 0, s, w, w_cs, rows, C, C32,
                     out);
}

void split_rows(const float* theta, bf16_t* split, int K, long P, long ld, hipStream_t s) {
  dim3 grid(grid_for(P / 4, 256, 1024), K);
  hipLaunchKernelGGL(split_rows_kernel, grid, dim3(256), 0, s, theta, split, P / 4, ld);
}

void adam_step(float* theta, const float* grad, float* m, float* v, bf16_t* shadow, const float* lr,
               const uint8_t* active, const float* step, int K, long P, long ld, float b1, float b2, float eps,
               float wd, hipStream_t s) {
  dim3 grid(grid_for(P, 256, 1024), K);
  hipLaunchKernelGGL(adam_kernel, grid, dim3(256), 0, s, theta, grad, m, v, shadow, lr, active, step, P, ld, b1, b2,
                     eps, wd);
}

void broadcast_rows(float* theta, bf16_t* shadow, const float* src, int K, long P, long ld, hipStream_t s) {
  dim3 grid(grid_for(P / 4, 256, 1024), K);
  hipLaunchKernelGGL(broadcast_kernel, grid, dim3(256), 0, s, theta, shadow, src, P / 4, ld);
}

void delta_rows(const float* theta, const float* base, float* out, int K, long P, long ld, hipStream_t s) {
  dim3 grid(grid_for(P / 4, 256, 1024), K);
  hipLaunchKernelGGL(delta_kernel, grid, dim3(256), 0, s, theta, base, out, P / 4, ld);
}

void weighted_sum(const float* x, const double* w, double* out, int K, long P, long ld, hipStream_t s) {
  hipLaunchKernelGGL(weighted_sum_kernel, dim3(grid_for(P / 4, 256, 8192)), dim3(256), 0, s, x, w, out, K, P / 4, ld);
}

void mix_rows(const float* x, const float* w, void* out, int K, int M, long P, long ld, long ld_out, int f32,
              hipStream_t s) {
  if (K > MIX_KMAX || M <= 0) {  // the wrapper (ops/hip.py) routes larger K elsewhere
    CHECK_HIP(hipErrorInvalidValue);
    return;
  }
  dim3 grid(grid_for(P / 4, 256, 2048), cdiv(M, MIX_M));
  DISPATCH_T(f32, hipLaunchKernelGGL(mix_rows_kernel<TT>, grid, dim3(256), 0, s, x, w, MP(out), K, M, P / 4, ld,
                                     ld_out));
}

void masked_weighted_sum(const float* x, const uint8_t* mask, const double* w, double* num, double* den, int K, long P,
                         long ld, hipStream_t s) {
  hipLaunchKernelGGL(masked_weighted_sum_kernel, dim3(grid_for(P, 256, 8192)), dim3(256), 0, s, x, mask, w, num, den,
                     K, P, ld);
}

void dropout_mask(uint8_t* mask, int K, long P, float p, const uint32_t* seeds, hipStream_t s) {
  const long n = (long)K * P;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, mask, P, p, seeds, n);
}

void block_sq_norms(const float* x, const int* block_ids, float* out, int K, long P, long ld, int nblocks,
                    hipStream_t s) {
  CHECK_HIP(hipMemsetAsync(out, 0, sizeof(float) * K * nblocks, s));
  dim3 grid(grid_for(P / 16, 256, 1024), K);
  hipLaunchKernelGGL(block_sq_kernel, grid, dim3(256), 0, s, x, block_ids, out, P, ld, nblocks);
}

void seg_minmax(const float* x, const int* seg, float* mn, float* mx, int K, long P, long ld, int nseg,
                hipStream_t s) {
  dim3 grid(cdiv(P, 256), K);
  hipLaunchKernelGGL(seg_minmax_kernel, grid, dim3(256), 0, s, x, seg, mn, mx, P, ld, nseg);
}

void stochastic_qdq(float* x, const int* seg, const float* mn, const float* mx, int K, long P, long ld, int nseg,
                    const uint32_t* seed, int levels, hipStream_t s) {
  dim3 grid(grid_for(P, 256, 2048), K);
  hipLaunchKernelGGL(stochastic_qdq_kernel, grid, dim3(256), 0, s, x, seg, mn, mx, P, ld, nseg, seed, levels);
}

void nnadq_qdq(float* x, const int* seg, const float* lo, const float* scale, const float* levels, int K, long P,
               long ld, int nseg, hipStream_t s) {
  dim3 grid(grid_for(P, 256, 2048), K);
  hipLaunchKernelGGL(nnadq_qdq_kernel, grid, dim3(256), 0, s, x, seg, lo, scale, levels, P, ld, nseg);
}

void sign_pack(const float* g, uint8_t* out, int K, long P, long ld, hipStream_t s) {
  const long nbytes = (P + 7) / 8;
  dim3 grid(grid_for(nbytes, 256, 2048), K);
  hipLaunchKernelGGL(sign_pack_kernel, grid, dim3(256), 0, s, g, out, P, ld, nbytes);
}

void sign_vote(const uint8_t* packed, const uint8_t* active, int* votes, int K, long P, hipStream_t s) {
  hipLaunchKernelGGL(sign_vote_kernel, dim3(grid_for(P, 256, 8192)), dim3(256), 0, s, packed, active, votes, K, P,
                     (P + 7) / 8);
}

void embedding_fwd(const int* tokens, const void* table, void* out, int K, long n_tok, int D, long t_cs, int rep,
                   int f32, hipStream_t s, float scale, const float* pe, int L) {
  const long total = (long)K * n_tok * D;
  DISPATCH_T(f32, hipLaunchKernelGGL(embedding_fwd_kernel<TT>, dim3(cdiv(total, 256)), dim3(256), 0, s, tokens,
                                     CP(table), MP(out), n_tok, D, t_cs, rep, total, scale, pe, L > 0 ? L : 1));
}

void embedding_bwd(const int* tokens, const void* dy, float* dtable, int K, long n_tok, int D, long t_cs, int f32,
                   hipStream_t s, float scale) {
  const long total = (long)K * n_tok * D;
  DISPATCH_T(f32, hipLaunchKernelGGL(embedding_bwd_kernel<TT>, dim3(cdiv(total, 256)), dim3(256), 0, s, tokens, CP(dy),
                                     dtable, n_tok, D, t_cs, total, scale));
}

void embedding_bwd_sorted(const int* keys, const int* order, const void* dy, float* dtable, long n, int D, int V,
                          long t_cs, int f32, hipStream_t s, float scale, float* part) {
  if (part) {  // chunked (part: [cdiv(n, EMB_CH)][2][D] fp32 scratch)
    const long nch = cdiv(n, (long)EMB_CH);
    DISPATCH_T(f32, hipLaunchKernelGGL(embedding_bwd_chunk_kernel<TT>, dim3(cdiv(nch, 4L)), dim3(256), 0, s, keys,
                                       order, CP(dy), dtable, part, n, D, V, t_cs, scale));
    DISPATCH_T(f32, hipLaunchKernelGGL(embedding_bwd_join_kernel<TT>, dim3(cdiv(nch, 4L)), dim3(256), 0, s, keys,
                                       part, dtable, n, D, V, t_cs, scale));
    return;
  }
  DISPATCH_T(f32, hipLaunchKernelGGL(embedding_bwd_sorted_kernel<TT>, dim3(cdiv(n, 4)), dim3(256), 0, s, keys, order,
                                     CP(dy), dtable, n, D, V, t_cs, scale));
}
long embedding_bwd_part_floats(long n, int D) { return cdiv(n, (long)EMB_CH) * 2 * D; }

void seq_mean_fwd(const void* x, const int* len, void* y, long S, int L, int D, int f32, hipStream_t s) {
  const long total = S * D;
  DISPATCH_T(f32, hipLaunchKernelGGL(seq_mean_fwd_kernel<TT>, dim3(cdiv(total, 256)), dim3(256), 0, s, CP(x), len,
                                     MP(y), L, D, total));
}

void seq_mean_bwd(const void* dy, const int* len, void* dx, long S, int L, int D, int f32, hipStream_t s) {
  const long total = S * L * D;
  DISPATCH_T(f32, hipLaunchKernelGGL(seq_mean_bwd_kernel<TT>, dim3(cdiv(total, 256)), dim3(256), 0, s, CP(dy), len,
                                     MP(dx), L, D, total));
}

void gather_rows(const void* src, const int* idx, void* dst, long n, long row_bytes, hipStream_t s) {
  const long v16 = row_bytes / 16;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(cdiv(n * v16, 256)), dim3(256), 0, s, static_cast<const uint4*>(src), idx,
                     static_cast<uint4*>(dst), n, v16);
}

void dropout_apply(const void* x, void* out, int K, long rows, int N, long ld, const uint32_t* seeds, float p,
                   float scale, int f32, hipStream_t s) {
  const long total = rows * (long)N;
  if (total == 0 || K == 0) return;
  const dim3 grid((unsigned)std::min<long>(cdiv(total, 256), 4096), K);
  if (f32)
    hipLaunchKernelGGL(dropout_apply_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(x),
                       static_cast<float*>(out), rows, N, ld, seeds, p, scale);
  else
    hipLaunchKernelGGL(dropout_apply_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(x),
                       static_cast<bf16_t*>(out), rows, N, ld, seeds, p, scale);
}

long dropout_planes_ws_floats(int K, long rows, int N) { return (long)K * cdiv(rows, DP_RB) * N; }

void dropout_planes(const float* x, float* out, bf16_t* yp, int K, long rows, int N, const uint32_t* seeds, float p,
                    float scale, hipStream_t s, float* colsum, long colsum_cs, float* ws) {
  if (rows == 0 || K == 0) return;
  if (N % 2) throw std::runtime_error("dropout_planes: N must be even");
  const dim3 grid((unsigned)cdiv(rows, DP_RB), K);
  hipLaunchKernelGGL(dropout_planes_kernel, grid, dim3(256), 0, s, x, out, yp, rows, N, seeds, p, scale,
                     colsum ? ws : nullptr);
  if (colsum) fold_col_partials(ws, (int)grid.x, N, colsum, colsum_cs, K, s);
}

void synth_images(const int64_t* idx, long n, long npix, int C, int Cout, const int* source, const float* proto,
                  unsigned long long salt, float sqrt6, float noise, float* out, hipStream_t s) {
  const long total = n * (npix / C) * Cout;
  if (total == 0) return;
  hipLaunchKernelGGL(synth_images_kernel, dim3((unsigned)std::min<long>(cdiv(total, 256), 65536)), dim3(256), 0, s,
                     idx, n, npix, C, Cout, source, proto, salt, sqrt6, noise, out);
}

// ------------------------------------------------------------------ host launch knobs (dls.h)
int g_opt_attn_mfma = kOptUnset, g_opt_conv_gl = kOptUnset;
int g_opt_pl_min_wg = kOptUnset;
int g_opt_halo_wgrad_unroll = kOptUnset, g_opt_halo_skip = kOptUnset;
int g_opt_conv_pix = kOptUnset;

int native_option(int& slot, const char* env, int dflt) {
  if (slot == kOptUnset) {
    const char* e = getenv(env);
    slot = e ? atoi(e) : dflt;
  }
  return slot;
}

bool set_native_option(const char* name, int value) {
  struct Entry {
    const char* name;
    int* slot;
  };
  const Entry table[] = {{"attn_mfma", &g_opt_attn_mfma},
                         {"conv_gl", &g_opt_conv_gl},       {"pl_min_wg", &g_opt_pl_min_wg},
                         {"halo_wgrad_unroll", &g_opt_halo_wgrad_unroll}, {"halo_skip", &g_opt_halo_skip},
                         {"conv_pix", &g_opt_conv_pix}};
  for (const Entry& t : table)
    if (strcmp(t.name, name) == 0) {
      *t.slot = value;
      return true;
    }
  return false;
}
