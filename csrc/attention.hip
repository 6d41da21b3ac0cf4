// Client-batched multi-head attention (fwd + bwd) for short sequences and small heads, gfx950.
//
//   q, k, v, o, do, dq, dk, dv : [KBH][L][DH] bf16   (KBH = clients × batch × heads, contiguous)
//   lse, delta                 : [KBH][L] fp32
//   key_valid                  : [KB] int32 (valid keys of each sequence; null = all L)
//
// Flash-style, never materialising the L×L score matrix (at L=300, 5 heads, 100 clients × 64
// sequences it would be 23 GB per layer): one workgroup per (sequence·head, 256-query block),
// the head's K and V (and for the backward Q / dO / lse / δ) staged ONCE in LDS as fp32, one
// query (or key) row per lane, online softmax over 16-key chunks (one rescale per chunk).
// The inner products are DH ≤ 64 wide — below one MFMA tile at the model's DH = 20 — so the
// math runs on the VALU with LDS-broadcast reads (every lane reads the same key row:
// conflict-free); the kernels are bound by the L² exp/FMA work, not by HBM.
//   fwd : o_i = Σ_j softmax_j(s_ij) v_j,  s_ij = (q_i·k_j)/√DH over valid keys;  lse_i
//   dq  : δ_i = do_i·o_i;  dq_i = Σ_j p_ij (do_i·v_j − δ_i) k_j / √DH       (writes δ)
//   dkv : dv_j = Σ_i p_ij do_i;  dk_j = Σ_i p_ij (do_i·v_j − δ_i) q_i / √DH
#include "common.h"

#include <stdlib.h>
#include "dls.h"

namespace {

constexpr int MAX_ROWS = 512;  // query / key rows per workgroup (one per lane): see attn_rows()
constexpr int CHUNK = 16;   // keys per online-softmax rescale

template <int DH, typename T>
__device__ __forceinline__ void load_row(const T* __restrict__ src, float* r) {
#pragma unroll
  for (int d = 0; d < DH; ++d) r[d] = ldf(src + d);
}

// one LDS row (broadcast: every lane reads the same address) as 16-B ds_read_b128s — rows are
// DH·4 B, 16-B aligned for every supported DH; half the LDS read instructions of the b64 form
template <int DH>
__device__ __forceinline__ void lds_row(const float* __restrict__ p, float* r) {
  static_assert(DH % 4 == 0, "rows are read as float4");
#pragma unroll
  for (int d = 0; d < DH; d += 4) {
    const float4 v = *reinterpret_cast<const float4*>(p + d);
    r[d] = v.x;
    r[d + 1] = v.y;
    r[d + 2] = v.z;
    r[d + 3] = v.w;
  }
}

// stage rows [0, L) of a [L][DH] bf16 matrix into LDS fp32 [L][DH]
template <int DH, typename T>
__device__ __forceinline__ void stage(const T* __restrict__ src, float* dst, int L) {
  for (int e = threadIdx.x; e < L * DH; e += blockDim.x) dst[e] = ldf(src + e);
}

template <int DH, typename T>
__global__ void __launch_bounds__(MAX_ROWS) attn_fwd_kernel(const T* __restrict__ q, const T* __restrict__ k,
                                                         const T* __restrict__ v, const int* __restrict__ key_valid,
                                                         T* __restrict__ o, float* __restrict__ lse, int L, int H,
                                                         float scale) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ks = smem;
  float* Vs = smem + L * DH;
  const long head = blockIdx.x;
  const long base = head * L * DH;
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  stage<DH>(k + base, Ks, nk);
  stage<DH>(v + base, Vs, nk);
  __syncthreads();
  const int i = blockIdx.y * blockDim.x + threadIdx.x;
  if (i >= L) return;
  float qi[DH], acc[DH];
  load_row<DH>(q + base + (long)i * DH, qi);
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    qi[d] *= scale;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j0 = 0; j0 < nk; j0 += CHUNK) {
    const int jn = min(CHUNK, nk - j0);
    float s[CHUNK];
    float cm = -INFINITY;
#pragma unroll
    for (int t = 0; t < CHUNK; ++t) {
      float a = -INFINITY;
      if (t < jn) {
        float kr[DH];
        lds_row<DH>(Ks + (j0 + t) * DH, kr);
        a = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) a = fmaf(qi[d], kr[d], a);
      }
      s[t] = a;
      cm = fmaxf(cm, a);
    }
    const float mn = fmaxf(m, cm);
    const float corr = __expf(m - mn);
    l *= corr;
#pragma unroll
    for (int d = 0; d < DH; ++d) acc[d] *= corr;
#pragma unroll
    for (int t = 0; t < CHUNK; ++t) {
      if (t < jn) {
        const float p = __expf(s[t] - mn);
        l += p;
        float vr[DH];
        lds_row<DH>(Vs + (j0 + t) * DH, vr);
#pragma unroll
        for (int d = 0; d < DH; ++d) acc[d] = fmaf(p, vr[d], acc[d]);
      }
    }
    m = mn;
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  T* orow = o + base + (long)i * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) stf(orow + d, acc[d] * inv);
  lse[head * L + i] = l > 0.f ? m + __logf(l) : 0.f;
}

template <int DH, typename T>
__global__ void __launch_bounds__(MAX_ROWS) attn_bwd_dq_kernel(const T* __restrict__ dout, const T* __restrict__ q,
                                                            const T* __restrict__ k, const T* __restrict__ v,
                                                            const T* __restrict__ o, const float* __restrict__ lse,
                                                            const int* __restrict__ key_valid, T* __restrict__ dq,
                                                            float* __restrict__ delta, int L, int H, float scale) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ks = smem;
  float* Vs = smem + L * DH;
  const long head = blockIdx.x;
  const long base = head * L * DH;
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  stage<DH>(k + base, Ks, nk);
  stage<DH>(v + base, Vs, nk);
  __syncthreads();
  const int i = blockIdx.y * blockDim.x + threadIdx.x;
  if (i >= L) return;
  float qi[DH], di[DH], g[DH];
  load_row<DH>(q + base + (long)i * DH, qi);
  load_row<DH>(dout + base + (long)i * DH, di);
  float dl = 0.f;
  {
    float oi[DH];
    load_row<DH>(o + base + (long)i * DH, oi);
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      dl = fmaf(di[d], oi[d], dl);
      qi[d] *= scale;
      g[d] = 0.f;
    }
  }
  delta[head * L + i] = dl;
  const float li = lse[head * L + i];
  for (int j = 0; j < nk; ++j) {
    float kr[DH], vr[DH];
    lds_row<DH>(Ks + j * DH, kr);
    lds_row<DH>(Vs + j * DH, vr);
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      s = fmaf(qi[d], kr[d], s);
      dp = fmaf(di[d], vr[d], dp);
    }
    const float ds = __expf(s - li) * (dp - dl);
#pragma unroll
    for (int d = 0; d < DH; ++d) g[d] = fmaf(ds, kr[d], g[d]);
  }
  T* out = dq + base + (long)i * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) stf(out + d, g[d] * scale);
}

template <int DH, typename T>
__global__ void __launch_bounds__(MAX_ROWS) attn_bwd_dkv_kernel(const T* __restrict__ dout, const T* __restrict__ q,
                                                             const T* __restrict__ k, const T* __restrict__ v,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ delta,
                                                             const int* __restrict__ key_valid, T* __restrict__ dk,
                                                             T* __restrict__ dv, int L, int H, float scale) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Qs = smem;
  float* Ds = smem + L * DH;
  float* Ls = smem + 2 * L * DH;
  float* Es = Ls + L;
  const long head = blockIdx.x;
  const long base = head * L * DH;
  const int nk = key_valid ? min(key_valid[head / H], L) : L;
  stage<DH>(q + base, Qs, L);
  stage<DH>(dout + base, Ds, L);
  for (int e = threadIdx.x; e < L; e += blockDim.x) {
    Ls[e] = lse[head * L + e];
    Es[e] = delta[head * L + e];
  }
  __syncthreads();
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= L) return;
  T* dkr = dk + base + (long)j * DH;
  T* dvr = dv + base + (long)j * DH;
  if (j >= nk) {  // padded key: no probability mass, no gradient
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      stf(dkr + d, 0.f);
      stf(dvr + d, 0.f);
    }
    return;
  }
  float kj[DH], vj[DH], gk[DH], gv[DH];
  load_row<DH>(k + base + (long)j * DH, kj);
  load_row<DH>(v + base + (long)j * DH, vj);
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    kj[d] *= scale;
    gk[d] = gv[d] = 0.f;
  }
  for (int i = 0; i < L; ++i) {
    float qr[DH], dr[DH];
    lds_row<DH>(Qs + i * DH, qr);
    lds_row<DH>(Ds + i * DH, dr);
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      s = fmaf(qr[d], kj[d], s);
      dp = fmaf(dr[d], vj[d], dp);
    }
    const float p = __expf(s - Ls[i]);
    const float ds = p * (dp - Es[i]);
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      gv[d] = fmaf(p, dr[d], gv[d]);
      gk[d] = fmaf(ds, qr[d], gk[d]);
    }
  }
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    stf(dkr + d, gk[d] * scale);
    stf(dvr + d, gv[d]);
  }
}

#define ATTN_DISPATCH(DHV, CALL) \
  switch (DHV) {                 \
    case 8: { constexpr int D = 8; CALL; } break;   \
    case 16: { constexpr int D = 16; CALL; } break; \
    case 20: { constexpr int D = 20; CALL; } break; \
    case 32: { constexpr int D = 32; CALL; } break; \
    case 64: { constexpr int D = 64; CALL; } break; \
    default: return false;                          \
  }

// dynamic LDS beyond 64 KiB must be opted into per kernel
void big_lds(const void* fn, size_t bytes) {
  if (bytes > 64 * 1024) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

// Rows per workgroup: the fewest workgroups per head (≤ 512 rows each), each rounded up to whole
// waves. At the model's L = 300 that is one 320-thread workgroup per head (94 % of lanes busy)
// instead of 256 + 256 threads (59 %): the kernels are VALU-bound, so idle lanes are lost time.
static int attn_rows(int L) {
  const int nblk = cdiv(L, MAX_ROWS);
  return ((cdiv(L, nblk) + 63) / 64) * 64;
}

// every head dim the MFMA kernels cover (attention_mfma.hip: 8 / 16 / 20 padded to 32, 32, 48
// padded to 64, 64) runs there unless DLS_ATTN_MFMA=0; the VALU kernels below are the fallback
// (no dropout, no packed layouts)
static bool use_mfma(int L, int DH) {
  return native_option(g_opt_attn_mfma, "DLS_ATTN_MFMA", 1) != 0 && attn_mfma_supported(L, DH);
}

bool attn_packed_supported(int L, int DH) { return use_mfma(L, DH); }

bool attn_supported(int L, int DH) {
  if (attn_mfma_supported(L, DH)) return true;
  if (!(DH == 8 || DH == 16 || DH == 20 || DH == 32 || DH == 64)) return false;
  return (2L * L * DH + 2L * L) * 4 <= 160L * 1024;
}

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

bool attn_fwd(const void* q, const void* k, const void* v, const int* key_valid, void* o, float* lse, long KBH, int H,
              int L, int DH, int f32, hipStream_t s, int ldqkv, int ldo, const uint32_t* drop_seeds,
              int heads_per_client, float drop_p) {
  if (use_mfma(L, DH))
    return attn_fwd_mfma(q, k, v, key_valid, o, lse, KBH, H, L, DH, f32, s, ldqkv, ldo, drop_seeds, heads_per_client,
                         drop_p);
  if (ldqkv || ldo || drop_p > 0.f) return false;  // packed layouts / dropout: MFMA kernels only
  if (!attn_supported(L, DH) || (2L * L * DH + 2L * L) * 4 > 160L * 1024) return false;
  const int rows = attn_rows(L);
  const dim3 grid((unsigned)KBH, cdiv(L, rows));
  const size_t sh = (size_t)2 * L * DH * sizeof(float);
  const float scale = 1.0f / sqrtf((float)DH);
  DISPATCH_T(f32, ATTN_DISPATCH(DH, big_lds((const void*)attn_fwd_kernel<D, TT>, sh);
                                hipLaunchKernelGGL((attn_fwd_kernel<D, TT>), grid, dim3(rows), sh, s, CP(q), CP(k),
                                                   CP(v), key_valid, MP(o), lse, L, H, scale)));
  return true;
}

bool attn_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
              const int* key_valid, void* dq, void* dk, void* dv, float* delta, long KBH, int H, int L, int DH, int f32,
              hipStream_t s, int ldqkv, int ldo, const uint32_t* drop_seeds, int heads_per_client, float drop_p) {
  if (use_mfma(L, DH))
    return attn_bwd_mfma(dout, q, k, v, o, lse, key_valid, dq, dk, dv, delta, KBH, H, L, DH, f32, s, ldqkv, ldo,
                         drop_seeds, heads_per_client, drop_p);
  if (ldqkv || ldo || drop_p > 0.f) return false;
  if (!attn_supported(L, DH) || (2L * L * DH + 2L * L) * 4 > 160L * 1024) return false;
  const int rows = attn_rows(L);
  const dim3 grid((unsigned)KBH, cdiv(L, rows));
  const float scale = 1.0f / sqrtf((float)DH);
  const size_t sh1 = (size_t)2 * L * DH * sizeof(float);
  const size_t sh2 = ((size_t)2 * L * DH + 2 * L) * sizeof(float);
  DISPATCH_T(f32, ATTN_DISPATCH(DH, big_lds((const void*)attn_bwd_dq_kernel<D, TT>, sh1);
                                hipLaunchKernelGGL((attn_bwd_dq_kernel<D, TT>), grid, dim3(rows), sh1, s, CP(dout),
                                                   CP(q), CP(k), CP(v), CP(o), lse, key_valid, MP(dq), delta, L, H,
                                                   scale)));
  DISPATCH_T(f32, ATTN_DISPATCH(DH, big_lds((const void*)attn_bwd_dkv_kernel<D, TT>, sh2);
                                hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, TT>), grid, dim3(rows), sh2, s, CP(dout),
                                                   CP(q), CP(k), CP(v), lse, delta, key_valid, MP(dk), MP(dv), L, H,
                                                   scale)));
  return true;
}

// ------------------------------------------------------------------------ SpMM (GCN)
// y[k][i][:] = Σ_{e ∈ row i} val[e] · x[k][col[e]][:]   (CSR graph shared by all K clients)
// One wave per (row, client); lanes own 8-feature chunks (16-B loads), fp32 accumulation.
template <typename T>
__global__ void __launch_bounds__(256) spmm_kernel(const int* __restrict__ rowptr, const int* __restrict__ col,
                                                   const float* __restrict__ val, const T* __restrict__ x,
                                                   T* __restrict__ y, int N, int Nx, int F, long x_cs, long y_cs) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + wave;
  if (i >= N) return;
  const int kc = blockIdx.y;
  const T* xk = x + (long)kc * x_cs;
  T* yk = y + (long)kc * y_cs + (long)i * F;
  const int e0 = rowptr[i], e1 = rowptr[i + 1];
  for (int f0 = lane * 8; f0 < F; f0 += 64 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bool vec = f0 + 8 <= F && (F % 8 == 0);
    for (int e = e0; e < e1; ++e) {
      const float a = val[e];
      const T* xr = xk + (long)col[e] * F + f0;
      if (vec) {
        float t[8];
        load_vec<8>(xr, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(a, t[j], acc[j]);
      } else {
        for (int j = 0; j < 8 && f0 + j < F; ++j) acc[j] = fmaf(a, ldf(xr + j), acc[j]);
      }
    }
    if (vec) {
      store_vec<8>(yk + f0, acc);
    } else {
      for (int j = 0; j < 8 && f0 + j < F; ++j) stf(yk + f0 + j, acc[j]);
    }
  }
}

void spmm(const int* rowptr, const int* col, const float* val, const void* x, void* y, int K, int N, int Nx, int F,
          long x_cs, long y_cs, int f32, hipStream_t s) {
  DISPATCH_T(f32, hipLaunchKernelGGL(spmm_kernel<TT>, dim3(cdiv(N, 4), K), dim3(256), 0, s, rowptr, col, val, CP(x),
                                     MP(y), N, Nx, F, x_cs, y_cs));
}
