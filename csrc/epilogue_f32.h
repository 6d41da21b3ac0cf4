// fp32 epilogue of the NT GEMMs (conv_f32.hip register-staged tiles, conv_pl.hip pre-split
// planes): bias (+ReLU) → optional BN statistics partials straight from the accumulators →
// per-wave 32-row fp32 LDS slab → 16-B coalesced stores with the optional gate (ReLU' of the
// next layer's input), dropout mask and accumulate (second gradient branch).
#pragma once
#include "dls.h"
#include "gemm_common.h"

// acc[TM][TN]: the wave's 32x32 accumulator tiles (v_mfma_f32_32x32x16 C layout); smem: ≥
// NW·32·SW floats, free (the caller has retired every read of the main-loop images)
// PF > 0: the global operands of the store loop (second gradient, BN input x, ReLU mask) are
// fetched PF column quads ahead of use; PF < 0: the rolled loop, each quad's operands loaded at
// its turn. The prefetch costs up to 9·PF VGPRs: a kernel opts in only where that keeps its
// occupancy and spills nothing (-Rpass-analysis=kernel-resource-usage; conv_halo.hip).
// YP: the output-planes stores (ConvNTParams::yp) are compiled in — off for the halo convs,
// whose occupancy the two extra registers would cost (l1 halo dgrad: 128 → 130 VGPRs, 4 → 3
// waves/SIMD, +45 % time measured)
// PIX: pixel-major GEMM rows (ConvNTParams::pix): row m is image m % B at pixel m / B; the
// valid-row limits (statistics, BN partials) are compared on the output row
template <int TM, int TN, int NW, int PF = -1, bool YP = true, bool PIX = false>
__device__ __forceinline__ void nt_f32_epilogue(const ConvNTParams& p, f32x16 (&acc)[TM][TN], unsigned char* smem,
                                                int client, int m0, int n0, int wm0, int wn0, int wid, int lane) {
  constexpr int SW = TN * 32 + 4;  // slab row (fp32), 16-B aligned
  float* __restrict__ y = reinterpret_cast<float*>(p.y) + (long)client * p.y_cs;
  const float* accp =
      p.acc ? reinterpret_cast<const float*>(p.acc) + (long)client * (p.acc_compact ? p.acc_cs : p.y_cs) : nullptr;
  const float* gatep = p.gate ? reinterpret_cast<const float*>(p.gate) + (long)client * p.y_cs : nullptr;
  // (acc_mask: acc's ReLU bits, [rows][N / 8] bytes per client, ldy == N; gate acc per column)
  const uint8_t* amask = (accp && p.acc_mask) ? p.acc_mask + (long)client * (p.y_cs >> 3) : nullptr;
  bf16_t* ypl = (YP && p.yp) ? p.yp + (long)client * p.yp_cs : nullptr;  // (output planes, ConvNTParams::yp)
  auto store_pl4 = [&](long off, const float4& v) {
    uint32_t h0, l0, h1, l1;
    split_pair(v.x, v.y, h0, l0);
    split_pair(v.z, v.w, h1, l1);
    *reinterpret_cast<uint2*>(ypl + off) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(ypl + p.yp_lo + off) = make_uint2(l0, l1);
  };
  auto store_pl1 = [&](long off, float v) {
    uint32_t h, l;
    split_pair(v, 0.f, h, l);
    ypl[off] = (bf16_t)(h & 0xffffu);
    ypl[p.yp_lo + off] = (bf16_t)(l & 0xffffu);
  };
  auto abits = [&](long row, int n, bool ok) -> uint32_t {
    return amask ? (ok ? (uint32_t)(amask[row * (p.N >> 3) + (n >> 3)] >> (n & 4)) : 0u) : 0xFu;
  };
  const float* bias = p.bias ? reinterpret_cast<const float*>(p.bias) + (long)(client / p.rep) * p.b_cs : nullptr;
  // epilogue scale (dropout's 1/(1-p), or the dgrad gate's) and dropout mask of this client row
  const bool drop = p.drop_p > 0.f && p.drop_seeds != nullptr;
  const uint32_t dseed = drop ? p.drop_seeds[client] : 0u;
  const float oscale = (p.out_scale != 0.f ? p.out_scale : 1.f) * (drop ? 1.f / (1.f - p.drop_p) : 1.f);
  float bvals[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + j * 32 + (lane & 31);
    bvals[j] = (bias && n < p.N) ? bias[n] : 0.f;
  }
  float* slab = reinterpret_cast<float*>(smem) + wid * 32 * SW;
  const bool vec_ok = (p.N % 4) == 0 && (p.ldy % 4) == 0 && ((uintptr_t)y & 15) == 0;
  // BN statistics rows: GEMM rows of this client's valid samples
  const int stat_rows = p.stats ? (p.stats_valid ? min(p.M, p.stats_valid[client] * p.OH * p.OW) : p.M) : 0;
  // BN-backward partials (ConvNTParams::bnb, stride-1 dgrad: GEMM row m is dX row m). In the store
  // loop below a lane always handles the same 4 columns (64 is a multiple of the Q = 8·TN column
  // quads per row), so it sums ĝ and ĝ·x̂ of its rows in registers; the Q-strided lanes then
  // combine with xor-shuffles and lanes < Q write the group's partial row
  static_assert(TN == 1 || TN == 2 || TN == 4 || TN == 8, "column quads per row must divide the wave");
  constexpr int Q = TN * 8;
  const bool bnb = p.bnb != nullptr;
  const int bnb_rows = bnb ? (p.bnb_valid ? min(p.M, p.bnb_valid[client]) : p.M) : 0;
  float4 bmu = make_float4(0.f, 0.f, 0.f, 0.f), brs = bmu;
  {
    const int n = n0 + wn0 + (lane % Q) * 4;
    if (bnb && n < p.N) {
      bmu = *reinterpret_cast<const float4*>(p.bnb_mean + (long)client * p.N + n);
      brs = *reinterpret_cast<const float4*>(p.bnb_rstd + (long)client * p.N + n);
    }
  }
  constexpr int QPL = 4 * TN;  // column quads per lane per 32-row group
  const float* bx_base = bnb ? p.bnb_x + (long)client * p.M * p.bnb_xld : nullptr;
  const unsigned char* bm_base = (bnb && p.bnb_mask) ? p.bnb_mask + (long)client * p.M * (p.N >> 3) : nullptr;
  const float* by_base = (bnb && p.bnb_y) ? p.bnb_y + (long)client * p.y_cs : nullptr;
  // an invalid quad loads from its tensor's client base (always mapped) and is zeroed after: no
  // branch around the load, so the loads of two quads issue back to back
  auto ld4 = [](const float* base, long off, bool ok) {
    const float4 v = *reinterpret_cast<const float4*>(ok ? base + off : base);
    return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  // GEMM row → output row (sub-pixel dgrad classes write every out_s-th pixel; pixel-major rows)
  auto row_of = [&](int m) -> long {
    if constexpr (PIX) {
      const uint32_t px = fdiv((uint32_t)m, p.fd_pb);
      return (long)((uint32_t)m - px * (uint32_t)p.B) * (p.OH * p.OW) + px;
    }
    if (p.out_s > 1) {
      const uint32_t b = fdiv(m, p.fd_ohw);
      const uint32_t rem = m - b * p.OH * p.OW;
      const uint32_t oh = fdiv(rem, p.fd_ow);
      const uint32_t ow = rem - oh * p.OW;
      return ((long)b * p.out_H + oh * p.out_s + p.out_ph) * p.out_W + ow * p.out_s + p.out_pw;
    }
    return m;
  };
  // the row the valid-row limits count (the GEMM row itself unless rows are pixel-major)
  auto vrow = [&](int m) -> long {
    if constexpr (PIX) return row_of(m);
    return m;
  };
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int g0 = m0 + wm0 + i * 32;  // this wave's 32-row group (a multiple of 32)
    if (p.stats && g0 < p.M) {
      // per-column Σy, Σy² of the group straight from the accumulators: lane (c, h) holds rows
      // (e&3) + 8(e>>2) + 4h of column c; the two half-waves combine with one xor-shuffle
      float* part = p.stats + ((long)client * ((p.M + 31) / 32) + g0 / 32) * 2 * p.N;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = g0 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          float v = acc[i][j][e] + bvals[j];
          if (p.relu) v = fmaxf(v, 0.f);
          if (vrow(m) < stat_rows) {
            s0 += v;
            s1 = fmaf(v, v, s1);
          }
        }
        s0 += __shfl_xor(s0, 32, 64);
        s1 += __shfl_xor(s1, 32, 64);
        const int n = n0 + wn0 + j * 32 + (lane & 31);
        if (lane < 32 && n < p.N) {
          part[n] = s0;
          part[p.N + n] = s1;
        }
      }
    }
    float4 bs0 = make_float4(0.f, 0.f, 0.f, 0.f), bs1 = bs0;
    if constexpr (PF > 0) {
      // 16-B column quads: lane l always owns columns cc = (l % Q)·4 of rows l / Q + t·(64 / Q). The
      // global operands of a quad (second gradient, BN input x and its ReLU mask) are fetched PF
      // quads ahead of their use — the first ones while the accumulators go through the slab — and
      // always together: a rolled load → wait → store loop serialised ≈3 L2/HBM round trips per
      // quad per wave (l1 dgrad with acc + BN partials: +34 % over the plain dgrad,
      // bench/epilogue_bench.py). (All quads in flight pushed the halo kernels from 4 to 2 waves
      // per SIMD.)
      const int cc = (lane % Q) * 4, n = n0 + wn0 + cc;
      constexpr int NS = PF > 0 ? PF : 1;  // operand slots
      float4 av[NS], xv[NS];
      uint32_t mv[NS], amv[NS];
      auto issue = [&](int t) {  // (t: compile-time after unrolling; slot t % NS)
        const int m = m0 + wm0 + i * 32 + lane / Q + t * (64 / Q);
        const bool ok = n < p.N && m < p.M;
        const long row = row_of(m);
        if (accp) av[t % NS] = ld4(accp, (p.acc_compact ? (long)m : row) * p.ldy + n, ok);
        if (amask) amv[t % NS] = abits(row, n, ok);
        if (bnb) {
          const bool okb = ok && vrow(m) < bnb_rows;
          xv[t % NS] = ld4(bx_base, row * p.bnb_xld + n, okb);
          if (bm_base) {
            const uint32_t mb = *(okb ? bm_base + vrow(m) * (p.N >> 3) + (n >> 3) : bm_base);
            mv[t % NS] = okb ? (mb >> (n & 4)) : 0u;
          } else if (by_base) {
            const float4 yv = ld4(by_base, row * p.ldy + n, okb);
            mv[t % NS] = (yv.x > 0.f ? 1u : 0u) | (yv.y > 0.f ? 2u : 0u) | (yv.z > 0.f ? 4u : 0u) | (yv.w > 0.f ? 8u : 0u);
          } else {
            mv[t % NS] = okb ? 0xFu : 0u;
          }
        }
      };
      if (vec_ok) {
#pragma unroll
        for (int t = 0; t < PF && t < QPL; ++t) issue(t);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float v = acc[i][j][e] + bvals[j];
          if (p.relu) v = fmaxf(v, 0.f);
          v *= oscale;
          if (drop) {
            const int rr = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            if (!drop_keep(dseed, m0 + wm0 + i * 32 + rr, p.N, n0 + wn0 + j * 32 + (lane & 31), p.drop_p)) v = 0.f;
          }
          slab[((e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * SW + j * 32 + (lane & 31)] = v;
        }
      }
      // LDS barrier only: __syncthreads()'s fence would also drain the operand loads in flight
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      if (vec_ok) {
#pragma unroll
        for (int t = 0; t < QPL; ++t) {
          const int r = lane / Q + t * (64 / Q);
          const int m = m0 + wm0 + i * 32 + r;
          const long row = row_of(m);
          float4 v = *reinterpret_cast<const float4*>(slab + r * SW + cc);
          if (gatep) {
            const float4 gv = ld4(gatep, row * p.ldy + n, n < p.N && m < p.M);
            v.x = gv.x > 0.f ? v.x : 0.f;
            v.y = gv.y > 0.f ? v.y : 0.f;
            v.z = gv.z > 0.f ? v.z : 0.f;
            v.w = gv.w > 0.f ? v.w : 0.f;
          }
          if (accp) {
            const uint32_t ab = amask ? amv[t % NS] : 0xFu;
            v.x += (ab & 1u) ? av[t % NS].x : 0.f;
            v.y += (ab & 2u) ? av[t % NS].y : 0.f;
            v.z += (ab & 4u) ? av[t % NS].z : 0.f;
            v.w += (ab & 8u) ? av[t % NS].w : 0.f;
          }
          if (n < p.N && m < p.M) {
            *reinterpret_cast<float4*>(y + row * p.ldy + n) = v;
            if (YP && ypl) store_pl4(row * p.ldy + n, v);
          }
          if (bnb) {  // ĝ = dX·relu', x̂ = (x − μ)·rstd of the BN whose dY this is (none past bnb_rows)
            const uint32_t mb = mv[t % NS];
            const float g0 = (mb & 1u) ? v.x : 0.f, g1 = (mb & 2u) ? v.y : 0.f;
            const float g2 = (mb & 4u) ? v.z : 0.f, g3 = (mb & 8u) ? v.w : 0.f;
            bs0.x += g0;
            bs0.y += g1;
            bs0.z += g2;
            bs0.w += g3;
            bs1.x = fmaf(g0, (xv[t % NS].x - bmu.x) * brs.x, bs1.x);
            bs1.y = fmaf(g1, (xv[t % NS].y - bmu.y) * brs.y, bs1.y);
            bs1.z = fmaf(g2, (xv[t % NS].z - bmu.z) * brs.z, bs1.z);
            bs1.w = fmaf(g3, (xv[t % NS].w - bmu.w) * brs.w, bs1.w);
          }
          if (PF > 0 && t + PF < QPL) issue(t + PF);
        }
      } else {  // scalar columns (N or the row stride not a multiple of 4; no BN partials here)
        for (int qd = lane; qd < 32 * TN * 8; qd += 64) {
          const int r = qd / (TN * 8), c4 = (qd % (TN * 8)) * 4;
          const int m = m0 + wm0 + i * 32 + r, nn = n0 + wn0 + c4;
          if (m >= p.M || nn >= p.N) continue;
          const long row = row_of(m);
          const long arow = p.acc_compact ? (long)m : row;  // (compact acc: the class-grid row)
          for (int t2 = 0; t2 < 4 && nn + t2 < p.N; ++t2) {
            float o = slab[r * SW + c4 + t2];
            if (gatep && !(gatep[row * p.ldy + nn + t2] > 0.f)) o = 0.f;
            if (accp && ((abits(row, nn + t2, true) >> ((nn + t2) & 3)) & 1u)) o += accp[arow * p.ldy + nn + t2];
            y[row * p.ldy + nn + t2] = o;
            if (YP && ypl) store_pl1(row * p.ldy + nn + t2, o);
          }
        }
      }
    } else {  // PF < 0: the rolled store loop (kernels without VGPRs to spare)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float v = acc[i][j][e] + bvals[j];
          if (p.relu) v = fmaxf(v, 0.f);
          v *= oscale;
          if (drop) {
            const int rr = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            if (!drop_keep(dseed, m0 + wm0 + i * 32 + rr, p.N, n0 + wn0 + j * 32 + (lane & 31), p.drop_p)) v = 0.f;
          }
          slab[((e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * SW + j * 32 + (lane & 31)] = v;
        }
      }
      __syncthreads();
      for (int qd = lane; qd < 32 * TN * 8; qd += 64) {
        const int r = qd / (TN * 8), cc = (qd % (TN * 8)) * 4;
        const int m = m0 + wm0 + i * 32 + r, n = n0 + wn0 + cc;
        if (m >= p.M || n >= p.N) continue;
        const long row = row_of(m);
        float* dst = y + row * p.ldy + n;
        const float* src = slab + r * SW + cc;
        const long arow = p.acc_compact ? (long)m : row;  // (compact acc: the class-grid row)
        if (vec_ok && n + 4 <= p.N) {
          float4 v = *reinterpret_cast<const float4*>(src);
          if (gatep) {
            const float4 gv = *reinterpret_cast<const float4*>(gatep + row * p.ldy + n);
            v.x = gv.x > 0.f ? v.x : 0.f;
            v.y = gv.y > 0.f ? v.y : 0.f;
            v.z = gv.z > 0.f ? v.z : 0.f;
            v.w = gv.w > 0.f ? v.w : 0.f;
          }
          if (accp) {
            const float4 av = *reinterpret_cast<const float4*>(accp + arow * p.ldy + n);
            const uint32_t ab = abits(row, n, true);
            v.x += (ab & 1u) ? av.x : 0.f;
            v.y += (ab & 2u) ? av.y : 0.f;
            v.z += (ab & 4u) ? av.z : 0.f;
            v.w += (ab & 8u) ? av.w : 0.f;
          }
          *reinterpret_cast<float4*>(dst) = v;
          if (YP && ypl) store_pl4(row * p.ldy + n, v);
          if (bnb && vrow(m) < bnb_rows) {  // ĝ = dX·relu', x̂ = (x − μ)·rstd of the BN whose dY this is
            const float4 xv =
                *reinterpret_cast<const float4*>(p.bnb_x + ((long)client * p.M + row) * p.bnb_xld + n);
            uint32_t mb = 0xFu;
            if (p.bnb_mask) {
              mb = p.bnb_mask[((long)client * p.M + vrow(m)) * (p.N >> 3) + (n >> 3)] >> (n & 4);
            } else if (p.bnb_y) {
              const float4 yv = *reinterpret_cast<const float4*>(p.bnb_y + (long)client * p.y_cs + row * p.ldy + n);
              mb = (yv.x > 0.f ? 1u : 0u) | (yv.y > 0.f ? 2u : 0u) | (yv.z > 0.f ? 4u : 0u) | (yv.w > 0.f ? 8u : 0u);
            }
            const float g0 = (mb & 1u) ? v.x : 0.f, g1 = (mb & 2u) ? v.y : 0.f;
            const float g2 = (mb & 4u) ? v.z : 0.f, g3 = (mb & 8u) ? v.w : 0.f;
            bs0.x += g0;
            bs0.y += g1;
            bs0.z += g2;
            bs0.w += g3;
            bs1.x = fmaf(g0, (xv.x - bmu.x) * brs.x, bs1.x);
            bs1.y = fmaf(g1, (xv.y - bmu.y) * brs.y, bs1.y);
            bs1.z = fmaf(g2, (xv.z - bmu.z) * brs.z, bs1.z);
            bs1.w = fmaf(g3, (xv.w - bmu.w) * brs.w, bs1.w);
          }
        } else {
          for (int t2 = 0; t2 < 4 && n + t2 < p.N; ++t2) {
            float o = src[t2];
            if (gatep && !(gatep[row * p.ldy + n + t2] > 0.f)) o = 0.f;
            if (accp && ((abits(row, n + t2, true) >> ((n + t2) & 3)) & 1u)) o += accp[arow * p.ldy + n + t2];
            dst[t2] = o;
            if (YP && ypl) store_pl1(row * p.ldy + n + t2, o);
          }
        }
      }
    }
    if (bnb) {
#pragma unroll
      for (int off = Q; off < 64; off <<= 1) {
        bs0.x += __shfl_xor(bs0.x, off, 64);
        bs0.y += __shfl_xor(bs0.y, off, 64);
        bs0.z += __shfl_xor(bs0.z, off, 64);
        bs0.w += __shfl_xor(bs0.w, off, 64);
        bs1.x += __shfl_xor(bs1.x, off, 64);
        bs1.y += __shfl_xor(bs1.y, off, 64);
        bs1.z += __shfl_xor(bs1.z, off, 64);
        bs1.w += __shfl_xor(bs1.w, off, 64);
      }
      const int g0 = m0 + wm0 + i * 32, n = n0 + wn0 + lane * 4;
      if (lane < Q && g0 < p.M && n < p.N) {
        float* part = p.bnb + ((long)client * ((p.M + 31) / 32) + g0 / 32) * 2 * p.N;
        *reinterpret_cast<float4*>(part + n) = bs0;
        *reinterpret_cast<float4*>(part + p.N + n) = bs1;
      }
    }
    __syncthreads();
  }
}
