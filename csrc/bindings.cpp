// pybind11 module `_dls_hip`: thin launch bindings. Python passes raw device pointers
// (tensor.data_ptr()) and the current HIP stream handle; shapes/strides are validated on
// the Python side (ops/hip.py) before any launch.
#include <pybind11/pybind11.h>

#include "dls.h"

namespace py = pybind11;
typedef uintptr_t ptr;

template <typename T>
static T* P(ptr p) {
  return reinterpret_cast<T*>(p);
}
static hipStream_t S(ptr s) { return reinterpret_cast<hipStream_t>(s); }

PYBIND11_MODULE(_dls_hip, m) {
  m.doc() = "gfx950 kernels for the MI355X-native cohort FL simulator";

  m.def("conv_nt", [](ptr x, ptr w, ptr y, ptr bias, long x_cs, long y_cs, long w_cs, long b_cs, int B, int H, int W,
                      int C, int OH, int OW, int KH, int KW, int stride, int pad, int dil, int M, int N, int R, int rep,
                      int relu, int K, int b_kmajor, int variant, ptr acc, ptr gate, int f32, ptr s, int ldx, int ldy,
                      ptr stats, ptr stats_valid, ptr drop_seeds, float drop_p, float out_scale, ptr wsplit,
                      long ws_cs, long ws_plane, long x_lo) {
    ConvNTParams p{};
    p.x_lo = x_lo;
    p.wsplit = P<const bf16_t>(wsplit);
    p.ws_cs = ws_cs;
    p.ws_plane = ws_plane;
    p.drop_seeds = P<const uint32_t>(drop_seeds);
    p.drop_p = drop_p;
    p.out_scale = out_scale;
    p.stats = P<float>(stats);
    p.stats_valid = P<const int>(stats_valid);
    p.f32 = f32;
    p.ldx = ldx;
    p.ldy = ldy;
    p.acc = P<const bf16_t>(acc);
    p.gate = P<const bf16_t>(gate);
    p.x = P<const bf16_t>(x);
    p.w = P<const bf16_t>(w);
    p.y = P<bf16_t>(y);
    p.bias = P<const bf16_t>(bias);
    p.x_cs = x_cs; p.y_cs = y_cs; p.w_cs = w_cs; p.b_cs = b_cs;
    p.B = B; p.H = H; p.W = W; p.C = C; p.OH = OH; p.OW = OW; p.KH = KH; p.KW = KW;
    p.stride = stride; p.pad = pad; p.dil = dil; p.M = M; p.N = N; p.R = R; p.rep = rep; p.relu = relu;
    p.b_kmajor = b_kmajor;
    conv_nt(p, K, variant, S(s));
  });
  m.def("conv_dgrad", [](ptr dy, ptr w, ptr dx, ptr acc, long w_cs, int K, int rep, int B, int OH, int OW, int Co, int H,
                         int W, int Ci, int KH, int KW, int stride, int pad, int variant, int f32, ptr s, int ld_dy,
                         long dy_cs, ptr wsplit, long ws_cs, long ws_plane, long x_lo) {
    conv_dgrad(P<const bf16_t>(dy), P<const bf16_t>(w), P<bf16_t>(dx), P<const bf16_t>(acc), w_cs, K, rep, B, OH, OW, Co, H, W, Ci, KH, KW,
               stride, pad, variant, f32, S(s), ld_dy, dy_cs, P<const bf16_t>(wsplit), ws_cs, ws_plane, x_lo);
  });
  m.def("conv_gl_wanted", &conv_gl_wanted);
  m.def("conv_gl_fwd", [](ptr x, ptr w, ptr y, ptr bias, long x_cs, long y_cs, long w_cs, long b_cs, int K, int rep,
                          int B, int H, int W, int C, int OH, int OW, int KH, int KW, int stride, int pad, int N,
                          int relu, ptr s) {
    conv_gl_fwd(P<const bf16_t>(x), P<const bf16_t>(w), P<bf16_t>(y), P<const bf16_t>(bias), x_cs, y_cs, w_cs, b_cs,
                K, rep, B, H, W, C, OH, OW, KH, KW, stride, pad, N, relu, S(s));
  });
  m.def("conv_weight_flip_t", [](ptr w, ptr wt, long w_cs, int Kw, int Co, int KH, int KW, int Ci, ptr s) {
    conv_weight_flip_t(P<const bf16_t>(w), P<bf16_t>(wt), w_cs, Kw, Co, KH, KW, Ci, S(s));
  });
  m.def("conv_gl_dgrad", [](ptr dy, ptr wt, ptr dx, ptr acc, int K, int rep, int B, int OH, int OW, int Co, int H, int W,
                            int Ci, int KH, int KW, int stride, int pad, ptr s) {
    conv_gl_dgrad(P<const bf16_t>(dy), P<const bf16_t>(wt), P<bf16_t>(dx), P<const bf16_t>(acc), K, rep, B, OH, OW, Co, H, W, Ci, KH, KW,
                  stride, pad, S(s));
  });
  m.def("conv_nt_num_variants", &conv_nt_num_variants);
  m.def("conv_nt_default_variant", &conv_nt_default_variant);
  m.def("conv_tn", [](ptr dy, ptr x, ptr dw, long dy_cs, long x_cs, long dw_cs, int B, int H, int W, int C, int OH,
                      int OW, int KH, int KW, int stride, int pad, int M, int Co, int R, int K, int variant, int f32,
                      ptr s, int ldy, int ldx, ptr part, long dy_lo, long x_lo) {
    ConvTNParams p{};
    p.part = P<float>(part);
    p.dy_lo = dy_lo;
    p.x_lo = x_lo;
    p.f32 = f32;
    p.ldy = ldy;
    p.ldx = ldx;
    p.dy = P<const bf16_t>(dy);
    p.x = P<const bf16_t>(x);
    p.dw = P<float>(dw);
    p.dy_cs = dy_cs; p.x_cs = x_cs; p.dw_cs = dw_cs;
    p.B = B; p.H = H; p.W = W; p.C = C; p.OH = OH; p.OW = OW; p.KH = KH; p.KW = KW; p.stride = stride; p.pad = pad;
    p.M = M; p.Co = Co; p.R = R; p.splitk = 1; p.m_per_split = M;
    conv_tn(p, K, variant, S(s));
  });
  m.def("conv_tn_splitk", &conv_tn_splitk, py::arg("K"), py::arg("Co"), py::arg("R"), py::arg("M"), py::arg("C"),
        py::arg("variant"), py::arg("f32"), py::arg("ldy") = 0, py::arg("ldx") = 0, py::arg("planes") = 0);
  m.def("conv_tn_pl_num_variants", &conv_tn_pl_num_variants);
  m.def("conv_tn_pl_set_variant", &conv_tn_pl_set_variant);
  m.def("conv_tn_pl_variant", &conv_tn_pl_variant);
  m.def("conv_tn_num_variants", &conv_tn_num_variants);
  m.def("conv_nt_f32_num_variants", &conv_nt_f32_num_variants);
  m.def("conv_nt_pl_num_variants", &conv_nt_pl_num_variants);
  m.def("conv_nt_pl_set_variant", &conv_nt_pl_set_variant);
  m.def("conv_halo_set_mode", &conv_halo_set_mode);
  m.def("conv_halo_set_variant", &conv_halo_set_variant);
  m.def("conv_tn_f32_num_variants", &conv_tn_f32_num_variants);

  m.def("bn_workspace_floats", &bn_workspace_floats);
  m.def("bn_fwd", [](ptr x, ptr gamma, ptr beta, ptr res, ptr y, ptr mean, ptr rstd, ptr valid, long g_cs, int K,
                     int R, int C, int relu, float eps, int rep, ptr ws, ptr mask, ptr counters, int f32, ptr s,
                     int ldx, ptr pre_part, int pre_nparts, ptr yp, int y_f32) {
    bn_fwd(P<const void>(x), P<const void>(gamma), P<const void>(beta), P<const void>(res), P<void>(y), P<float>(mean),
           P<float>(rstd), P<const int>(valid), g_cs, K, R, C, relu, eps, rep, P<float>(ws), P<uint8_t>(mask),
           P<unsigned>(counters), f32, S(s), ldx, P<const float>(pre_part), pre_nparts, P<bf16_t>(yp), y_f32);
  });
  m.def("bn_bwd", [](ptr dy, ptr x, ptr y, ptr mean, ptr rstd, ptr gamma, ptr valid, long g_cs, int K, int R, int C,
                     int relu, ptr dx, ptr dpre, ptr dgamma, ptr dbeta, long dg_cs, ptr ws, ptr mask, ptr counters,
                     int f32, ptr s, int ldx, int acc_dx, ptr dxp, int dx_f32) {
    bn_bwd(P<const void>(dy), P<const void>(x), P<const void>(y), P<const float>(mean), P<const float>(rstd),
           P<const void>(gamma), P<const int>(valid), g_cs, K, R, C, relu, P<void>(dx), P<void>(dpre), P<float>(dgamma),
           P<float>(dbeta), dg_cs, P<float>(ws), P<const uint8_t>(mask), P<unsigned>(counters), f32, S(s), ldx,
           acc_dx, P<bf16_t>(dxp), dx_f32);
  });
  m.def("ln_fwd", [](ptr x, ptr gamma, ptr beta, ptr y, ptr mean, ptr rstd, long g_cs, int K, long rpc, int C,
                     float eps, int rep, int f32, ptr s) {
    ln_fwd(P<const void>(x), P<const void>(gamma), P<const void>(beta), P<void>(y), P<float>(mean), P<float>(rstd),
           g_cs, K, rpc, C, eps, rep, f32, S(s));
  });
  m.def("ln_bwd", [](ptr dy, ptr x, ptr mean, ptr rstd, ptr gamma, long g_cs, int K, long rpc, int C, ptr dx,
                     ptr dgamma, ptr dbeta, long dg_cs, int f32, ptr s) {
    ln_bwd(P<const void>(dy), P<const void>(x), P<const float>(mean), P<const float>(rstd), P<const void>(gamma), g_cs,
           K, rpc, C, P<void>(dx), P<float>(dgamma), P<float>(dbeta), dg_cs, nullptr, f32, S(s));
  });
  m.def("col_sum", [](ptr x, ptr out, long out_cs, int K, long rows, int C, int f32, ptr s) {
    col_sum(P<const void>(x), P<float>(out), out_cs, K, rows, C, f32, S(s));
  });

  m.def("pool_fwd", [](ptr x, ptr y, ptr idx, int K, int B, int H, int W, int C, int OH, int OW, int k, int stride,
                       int pad, int mode, int f32, ptr s) {
    pool_fwd(P<const void>(x), P<void>(y), P<int>(idx), K, B, H, W, C, OH, OW, k, stride, pad, mode, f32, S(s));
  });
  m.def("pool_bwd", [](ptr dy, ptr idx, ptr dx, int K, int B, int H, int W, int C, int OH, int OW, int k, int stride,
                       int pad, int mode, int f32, ptr s) {
    pool_bwd(P<const void>(dy), P<const int>(idx), P<void>(dx), K, B, H, W, C, OH, OW, k, stride, pad, mode, f32, S(s));
  });
  m.def("gap_fwd", [](ptr x, ptr y, int KB, int HW, int C, int f32, ptr s) {
    gap_fwd(P<const void>(x), P<void>(y), KB, HW, C, f32, S(s));
  });
  m.def("gap_bwd", [](ptr dy, ptr dx, int KB, int HW, int C, int f32, ptr s) {
    gap_bwd(P<const void>(dy), P<void>(dx), KB, HW, C, f32, S(s));
  });
  m.def("ce_fwd_bwd", [](ptr logits, ptr labels, ptr valid, ptr loss, ptr correct, ptr dlogits, int K, int B, int NC,
                         int f32, ptr s) {
    ce_fwd_bwd(P<const void>(logits), P<const int>(labels), P<const int>(valid), P<float>(loss), P<float>(correct),
               P<void>(dlogits), K, B, NC, f32, S(s));
  });
  m.def("relu_bwd", [](ptr dy, ptr y, ptr dx, long n, int f32, ptr s) {
    relu_bwd(P<const void>(dy), P<const void>(y), P<void>(dx), n, f32, S(s));
  });

  m.def("sgd_step", [](ptr theta, ptr grad, ptr mom, ptr shadow, ptr split, ptr lr, ptr active, ptr first, int K,
                       long Pn, long ld, float wd, float momentum, float dampening, int nesterov, ptr s) {
    sgd_step(P<float>(theta), P<const float>(grad), P<float>(mom), P<bf16_t>(shadow), P<bf16_t>(split),
             P<const float>(lr), P<const uint8_t>(active), P<const uint8_t>(first), K, Pn, ld, wd, momentum, dampening,
             nesterov, S(s));
  });
  m.def("split_rows", [](ptr theta, ptr split, int K, long Pn, long ld, ptr s) {
    split_rows(P<const float>(theta), P<bf16_t>(split), K, Pn, ld, S(s));
  });
  m.def("adam_step", [](ptr theta, ptr grad, ptr mm, ptr v, ptr shadow, ptr lr, ptr active, ptr step, int K, long Pn,
                        long ld, float b1, float b2, float eps, float wd, ptr s) {
    adam_step(P<float>(theta), P<const float>(grad), P<float>(mm), P<float>(v), P<bf16_t>(shadow), P<const float>(lr),
              P<const uint8_t>(active), P<const float>(step), K, Pn, ld, b1, b2, eps, wd, S(s));
  });
  m.def("broadcast_rows", [](ptr theta, ptr shadow, ptr src, int K, long Pn, long ld, ptr s) {
    broadcast_rows(P<float>(theta), P<bf16_t>(shadow), P<const float>(src), K, Pn, ld, S(s));
  });
  m.def("delta_rows", [](ptr theta, ptr base, ptr out, int K, long Pn, long ld, ptr s) {
    delta_rows(P<const float>(theta), P<const float>(base), P<float>(out), K, Pn, ld, S(s));
  });
  m.def("weighted_sum", [](ptr x, ptr w, ptr out, int K, long Pn, long ld, ptr s) {
    weighted_sum(P<const float>(x), P<const double>(w), P<double>(out), K, Pn, ld, S(s));
  });
  m.def("mix_rows", [](ptr x, ptr w, ptr out, int K, int M, long Pn, long ld, long ld_out, int f32, ptr s) {
    mix_rows(P<const float>(x), P<const float>(w), P<void>(out), K, M, Pn, ld, ld_out, f32, S(s));
  });
  m.def("masked_weighted_sum", [](ptr x, ptr mask, ptr w, ptr num, ptr den, int K, long Pn, long ld, ptr s) {
    masked_weighted_sum(P<const float>(x), P<const uint8_t>(mask), P<const double>(w), P<double>(num), P<double>(den), K,
                        Pn, ld, S(s));
  });
  m.def("dropout_mask", [](ptr mask, int K, long Pn, float p, ptr seeds, ptr s) {
    dropout_mask(P<uint8_t>(mask), K, Pn, p, P<const uint32_t>(seeds), S(s));
  });
  m.def("block_sq_norms", [](ptr x, ptr ids, ptr out, int K, long Pn, long ld, int nb, ptr s) {
    block_sq_norms(P<const float>(x), P<const int>(ids), P<float>(out), K, Pn, ld, nb, S(s));
  });
  m.def("seg_minmax", [](ptr x, ptr seg, ptr mn, ptr mx, int K, long Pn, long ld, int nseg, ptr s) {
    seg_minmax(P<const float>(x), P<const int>(seg), P<float>(mn), P<float>(mx), K, Pn, ld, nseg, S(s));
  });
  m.def("stochastic_qdq", [](ptr x, ptr seg, ptr mn, ptr mx, int K, long Pn, long ld, int nseg, ptr seeds,
                             int levels, ptr s) {
    stochastic_qdq(P<float>(x), P<const int>(seg), P<const float>(mn), P<const float>(mx), K, Pn, ld, nseg,
                   P<const uint32_t>(seeds), levels,
                   S(s));
  });
  m.def("sign_pack", [](ptr g, ptr out, int K, long Pn, long ld, ptr s) { sign_pack(P<const float>(g), P<uint8_t>(out), K, Pn, ld, S(s)); });
  m.def("sign_vote", [](ptr packed, ptr active, ptr votes, int K, long Pn, ptr s) {
    sign_vote(P<const uint8_t>(packed), P<const uint8_t>(active), P<int>(votes), K, Pn, S(s));
  });
  m.def("embedding_fwd", [](ptr tok, ptr table, ptr out, int K, long n_tok, int D, long t_cs, int rep, int f32, ptr s,
                            float scale, ptr pe, int L) {
    embedding_fwd(P<const int>(tok), P<const void>(table), P<void>(out), K, n_tok, D, t_cs, rep, f32, S(s), scale,
                  P<const float>(pe), L);
  });
  m.def("embedding_bwd", [](ptr tok, ptr dy, ptr dtable, int K, long n_tok, int D, long t_cs, int f32, ptr s,
                            float scale) {
    embedding_bwd(P<const int>(tok), P<const void>(dy), P<float>(dtable), K, n_tok, D, t_cs, f32, S(s), scale);
  });
  m.def("seq_mean_fwd", [](ptr x, ptr len, ptr y, long S_, int L, int D, int f32, ptr s) {
    seq_mean_fwd(P<const void>(x), P<const int>(len), P<void>(y), S_, L, D, f32, S(s));
  });
  m.def("seq_mean_bwd", [](ptr dy, ptr len, ptr dx, long S_, int L, int D, int f32, ptr s) {
    seq_mean_bwd(P<const void>(dy), P<const int>(len), P<void>(dx), S_, L, D, f32, S(s));
  });
  m.def("attn_supported", &attn_supported);
  m.def("attn_packed_supported", &attn_packed_supported);
  m.def("attn_fwd", [](ptr q, ptr k, ptr v, ptr kv, ptr o, ptr lse, long KBH, int H, int L, int DH, int f32, ptr s,
                       int ldqkv, int ldo) {
    return attn_fwd(P<const void>(q), P<const void>(k), P<const void>(v), P<const int>(kv), P<void>(o), P<float>(lse),
                    KBH, H, L, DH, f32, S(s), ldqkv, ldo);
  });
  m.def("attn_bwd", [](ptr dout, ptr q, ptr k, ptr v, ptr o, ptr lse, ptr kv, ptr dq, ptr dk, ptr dv, ptr delta,
                       long KBH, int H, int L, int DH, int f32, ptr s, int ldqkv, int ldo) {
    return attn_bwd(P<const void>(dout), P<const void>(q), P<const void>(k), P<const void>(v), P<const void>(o),
                    P<const float>(lse), P<const int>(kv), P<void>(dq), P<void>(dk), P<void>(dv), P<float>(delta), KBH,
                    H, L, DH, f32, S(s), ldqkv, ldo);
  });
  m.def("dropout_apply", [](ptr x, ptr out, int K, long rows, int N, long ld, ptr seeds, float p, float scale,
                            int f32, ptr s) {
    dropout_apply(P<const void>(x), P<void>(out), K, rows, N, ld, P<const uint32_t>(seeds), p, scale, f32, S(s));
  });
  m.def("synth_images", [](ptr idx, long n, long npix, int C, int Cout, ptr source, ptr proto,
                           unsigned long long salt, float sqrt6, float noise, ptr out, ptr s) {
    synth_images(P<const int64_t>(idx), n, npix, C, Cout, P<const int>(source), P<const float>(proto), salt, sqrt6,
                 noise, P<float>(out), S(s));
  });
  m.def("quant_pack", [](ptr x, long ld, ptr seg, ptr seg_off, ptr seg_numel, ptr bits, ptr lo, ptr scale,
                         ptr seg_byte_off, ptr row_off, int K, int nseg, long Pn, int stochastic, ptr seeds, ptr out,
                         ptr s) {
    quant_pack(P<const float>(x), ld, P<const int>(seg), P<const int64_t>(seg_off), P<const int64_t>(seg_numel),
               P<const uint8_t>(bits), P<const float>(lo), P<const float>(scale), P<const int64_t>(seg_byte_off),
               P<const int64_t>(row_off), K, nseg, Pn, stochastic, P<const uint32_t>(seeds), P<uint8_t>(out), S(s));
  });
  m.def("quant_unpack", [](ptr codes, ptr seg, ptr seg_off, ptr seg_numel, ptr bits, ptr lo, ptr scale,
                           ptr seg_byte_off, ptr row_off, int K, int nseg, long Pn, ptr out, long ld, ptr s) {
    quant_unpack(P<const uint8_t>(codes), P<const int>(seg), P<const int64_t>(seg_off), P<const int64_t>(seg_numel),
                 P<const uint8_t>(bits), P<const float>(lo), P<const float>(scale), P<const int64_t>(seg_byte_off),
                 P<const int64_t>(row_off), K, nseg, Pn, P<float>(out), ld, S(s));
  });
  m.def("quant_unpack_acc", [](ptr codes, ptr seg, ptr seg_off, ptr seg_numel, ptr bits, ptr lo, ptr scale,
                               ptr seg_byte_off, ptr row_off, int K, int nseg, long Pn, ptr w, ptr acc, ptr s) {
    quant_unpack_acc(P<const uint8_t>(codes), P<const int>(seg), P<const int64_t>(seg_off),
                     P<const int64_t>(seg_numel), P<const uint8_t>(bits), P<const float>(lo), P<const float>(scale),
                     P<const int64_t>(seg_byte_off), P<const int64_t>(row_off), K, nseg, Pn, P<const double>(w),
                     P<double>(acc), S(s));
  });
  m.def("neighbor_sample", [](ptr rowptr, ptr col, ptr owner, ptr is_val, ptr nodes, ptr clients, int n, int fanout,
                              unsigned long long seed_h, ptr out_nbr, ptr out_cnt, ptr s) {
    neighbor_sample(P<const int>(rowptr), P<const int>(col), P<const int>(owner), P<const uint8_t>(is_val),
                    P<const int64_t>(nodes), P<const int64_t>(clients), n, fanout, seed_h, P<int>(out_nbr),
                    P<int>(out_cnt), S(s));
  });
  m.def("spmm", [](ptr rowptr, ptr col, ptr val, ptr x, ptr y, int K, int N, int Nx, int F, long x_cs, long y_cs,
                   int f32, ptr s) {
    spmm(P<const int>(rowptr), P<const int>(col), P<const float>(val), P<const void>(x), P<void>(y), K, N, Nx, F, x_cs,
         y_cs, f32, S(s));
  });
  m.def("nnadq_qdq", [](ptr x, ptr seg, ptr lo, ptr scale, ptr levels, int K, long Pn, long ld, int nseg, ptr s) {
    nnadq_qdq(P<float>(x), P<const int>(seg), P<const float>(lo), P<const float>(scale), P<const float>(levels), K, Pn,
              ld, nseg, S(s));
  });
  m.def("gather_rows", [](ptr src, ptr idx, ptr dst, long n, long row_bytes, ptr s) {
    gather_rows(P<const void>(src), P<const int>(idx), P<void>(dst), n, row_bytes, S(s));
  });
}
