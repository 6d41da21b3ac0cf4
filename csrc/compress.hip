// Compressed upload / broadcast payloads (gfx950): pack quantised codes into the actual wire
// buffer, unpack on the receiver — either to dense rows or fused into the server's fp64
// weighted accumulation (reference topology/quantized_endpoint.py).
//
// Payload of client k: for every sent tensor (segment) s, b = bits[k][s] ∈ [1, 8] bits per
// element, packed LSB-first. Layout tensors start at 16-element aligned flat offsets, so the flat
// groups [8t, 8t+8) never straddle two tensors. The 8 codes of a group fill exactly b bytes, at
//   row_off[k] + seg_byte_off[k][s] + (j0 / 8)·b      (j0 = element index within s)
// A tensor's tail group writes only ceil(n·b / 8) bytes. One thread per (client, group): no two
// threads touch the same byte. Codes:
//   stochastic (FedPAQ, QSGD with 255 signed levels: lo = −‖x‖, scale = ‖x‖/127, ops/quant.py):
//                                    q = clamp(floor((x − lo) / scale + u), 0, 2^b − 2),
//                                    u = mix32(flat index, seed_k)
//   deterministic (NNADQ):           q = clamp(rint((x − lo) / scale), 0, 2^b − 1)
// and x̂ = lo + q·scale (contraction disabled in the decoders: bit-identical to the CPU oracle;
// written as plain operators there — HIP's __fmul_rn / __fadd_rn are header functions compiled
// under -ffp-contract=fast, which the backend fuses after inlining).
#include "common.h"
#include "dls.h"

namespace {

__global__ void quant_pack_kernel(const float* __restrict__ x, long ld, const int* __restrict__ seg,
                                  const int64_t* __restrict__ seg_off, const int64_t* __restrict__ seg_numel,
                                  const uint8_t* __restrict__ bits, const float* __restrict__ lo,
                                  const float* __restrict__ scale, const int64_t* __restrict__ seg_byte_off,
                                  const int64_t* __restrict__ row_off, int nseg, long ngroups, int stochastic,
                                  const uint32_t* __restrict__ seeds, uint8_t* __restrict__ out) {
  const int k = blockIdx.y;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ngroups) return;
  const long e0 = t * 8;
  const int s = seg[e0];
  if (s >= nseg) return;  // inter-tensor padding
  const long q0 = (long)k * nseg + s;
  const int b = bits[q0];
  if (b == 0) return;  // tensor not sent by this client
  const long j0 = e0 - seg_off[s];
  const int n = (int)min(8L, seg_numel[s] - j0);
  const float l = lo[q0], sc = scale[q0];
  const float top = (float)((1 << b) - (stochastic ? 2 : 1));  // QSGD: codes 0..2s, s = 2^(b-1) − 1
  const float* xr = x + (long)k * ld + e0;
  unsigned long long word = 0;
  for (int e = 0; e < n; ++e) {
    const float r = __fdiv_rn(__fsub_rn(xr[e], l), sc);
    float q;
    if (stochastic) {
      const float u = (float)mix32((uint32_t)((e0 + e) & 0xffffffffu), seeds[k]) * (1.f / 4294967296.f);
      q = floorf(__fadd_rn(r, u));
    } else {
      q = rintf(r);
    }
    q = fminf(fmaxf(q, 0.f), top);
    word |= (unsigned long long)(unsigned)q << (e * b);
  }
  uint8_t* dst = out + row_off[k] + seg_byte_off[q0] + (j0 / 8) * b;
  const int nb = (n * b + 7) / 8;
  for (int i = 0; i < nb; ++i) dst[i] = (uint8_t)(word >> (8 * i));
}

__device__ __forceinline__ int read_codes(const uint8_t* __restrict__ codes, const int64_t* __restrict__ row_off,
                                          const int64_t* __restrict__ seg_byte_off, long q0, int k, long j0, int n,
                                          int b, unsigned long long& word) {
  const uint8_t* src = codes + row_off[k] + seg_byte_off[q0] + (j0 / 8) * b;
  const int nb = (n * b + 7) / 8;
  word = 0;
  for (int i = 0; i < nb; ++i) word |= (unsigned long long)src[i] << (8 * i);
  return nb;
}

// dense rows: out[k][i] = x̂ (0 for tensors not sent and for padding)
__global__ void quant_unpack_kernel(const uint8_t* __restrict__ codes, const int* __restrict__ seg,
                                    const int64_t* __restrict__ seg_off, const int64_t* __restrict__ seg_numel,
                                    const uint8_t* __restrict__ bits, const float* __restrict__ lo,
                                    const float* __restrict__ scale, const int64_t* __restrict__ seg_byte_off,
                                    const int64_t* __restrict__ row_off, int nseg, long ngroups,
                                    float* __restrict__ out, long ld) {
#pragma clang fp contract(off)  // x̂ = lo + q·scale rounded twice, as the CPU oracle (no FMA)
  const int k = blockIdx.y;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ngroups) return;
  const long e0 = t * 8;
  float* o = out + (long)k * ld + e0;
  const int s = seg[e0];
  const long q0 = (long)k * nseg + s;
  const int b = s < nseg ? bits[q0] : 0;
  if (b == 0) {
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
    return;
  }
  const long j0 = e0 - seg_off[s];
  const int n = (int)min(8L, seg_numel[s] - j0);
  unsigned long long word;
  read_codes(codes, row_off, seg_byte_off, q0, k, j0, n, b, word);
  const unsigned long long m = (1ull << b) - 1;
  const float l = lo[q0], sc = scale[q0];
  for (int e = 0; e < 8; ++e) {
    const float q = (float)((word >> (e * b)) & m);
    const float prod = q * sc;  // plain operators under contract(off): two roundings, no FMA
    o[e] = e < n ? l + prod : 0.f;
  }
}

// fused server accumulate: acc[i] += Σ_k w[k]·x̂_k[i] in fp64 (one writer per element)
__global__ void quant_unpack_acc_kernel(const uint8_t* __restrict__ codes, const int* __restrict__ seg,
                                        const int64_t* __restrict__ seg_off, const int64_t* __restrict__ seg_numel,
                                        const uint8_t* __restrict__ bits, const float* __restrict__ lo,
                                        const float* __restrict__ scale, const int64_t* __restrict__ seg_byte_off,
                                        const int64_t* __restrict__ row_off, int nseg, long ngroups, int K,
                                        const double* __restrict__ w, double* __restrict__ acc) {
#pragma clang fp contract(off)
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ngroups) return;
  const long e0 = t * 8;
  const int s = seg[e0];
  if (s >= nseg) return;
  const long j0 = e0 - seg_off[s];
  const int n = (int)min(8L, seg_numel[s] - j0);
  double sum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sum[e] = 0.0;
  for (int k = 0; k < K; ++k) {
    const long q0 = (long)k * nseg + s;
    const int b = bits[q0];
    if (b == 0) continue;
    unsigned long long word;
    read_codes(codes, row_off, seg_byte_off, q0, k, j0, n, b, word);
    const unsigned long long m = (1ull << b) - 1;
    const float l = lo[q0], sc = scale[q0];
    const double wk = w[k];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float prod = (float)((word >> (e * b)) & m) * sc;
      const float v = l + prod;
      sum[e] += wk * (double)v;
    }
  }
  for (int e = 0; e < n; ++e) acc[e0 + e] += sum[e];
}

}  // namespace

void quant_pack(const float* x, long ld, const int* seg, const int64_t* seg_off, const int64_t* seg_numel,
                const uint8_t* bits, const float* lo, const float* scale, const int64_t* seg_byte_off,
                const int64_t* row_off, int K, int nseg, long P, int stochastic, const uint32_t* seeds, uint8_t* out,
                hipStream_t s) {
  const long ngroups = P / 8;
  if (ngroups == 0 || K == 0) return;
  hipLaunchKernelGGL(quant_pack_kernel, dim3(cdiv(ngroups, 256), K), dim3(256), 0, s, x, ld, seg, seg_off, seg_numel,
                     bits, lo, scale, seg_byte_off, row_off, nseg, ngroups, stochastic, seeds, out);
}

void quant_unpack(const uint8_t* codes, const int* seg, const int64_t* seg_off, const int64_t* seg_numel,
                  const uint8_t* bits, const float* lo, const float* scale, const int64_t* seg_byte_off,
                  const int64_t* row_off, int K, int nseg, long P, float* out, long ld, hipStream_t s) {
  const long ngroups = P / 8;
  if (ngroups == 0 || K == 0) return;
  hipLaunchKernelGGL(quant_unpack_kernel, dim3(cdiv(ngroups, 256), K), dim3(256), 0, s, codes, seg, seg_off,
                     seg_numel, bits, lo, scale, seg_byte_off, row_off, nseg, ngroups, out, ld);
}

void quant_unpack_acc(const uint8_t* codes, const int* seg, const int64_t* seg_off, const int64_t* seg_numel,
                      const uint8_t* bits, const float* lo, const float* scale, const int64_t* seg_byte_off,
                      const int64_t* row_off, int K, int nseg, long P, const double* w, double* acc, hipStream_t s) {
  const long ngroups = P / 8;
  if (ngroups == 0 || K == 0) return;
  hipLaunchKernelGGL(quant_unpack_acc_kernel, dim3(cdiv(ngroups, 256)), dim3(256), 0, s, codes, seg, seg_off,
                     seg_numel, bits, lo, scale, seg_byte_off, row_off, nseg, ngroups, K, w, acc);
}
