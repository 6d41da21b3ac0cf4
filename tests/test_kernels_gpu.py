"""Numerics of every gfx950 kernel vs the plain-PyTorch fp32 reference (`ops.ref`)."""

import pytest
import torch

from distributed_learning_simulator_amd.ops import ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def _close(out, exp, tol=2e-2):
    out = out.float()
    exp = exp.float()
    err = (out - exp).abs().max().item()
    mag = exp.abs().max().item() + 1e-6
    assert err <= tol * mag, f"max err {err} vs magnitude {mag}"


CONV_CASES = [
    # K, B, H, W, Ci, Co, k, stride, pad
    (3, 4, 8, 8, 16, 32, 3, 1, 1),
    (2, 2, 8, 8, 64, 64, 3, 1, 1),
    (2, 3, 9, 9, 64, 128, 3, 2, 1),
    (2, 2, 8, 8, 64, 128, 1, 2, 0),
    (3, 2, 8, 8, 3, 64, 3, 1, 1),       # stem: Ci=3 scalar path
    (2, 2, 6, 6, 36, 12, 3, 1, 1),      # DenseNet-like: Ci%8==4, Co=12
    (2, 2, 12, 12, 1, 6, 5, 1, 2),      # LeNet conv1
    (2, 2, 7, 7, 128, 256, 3, 1, 1),
    (1, 2, 16, 16, 8, 8, 7, 2, 3),
    (2, 2, 9, 7, 16, 32, 3, 3, 1),      # stride 3, non-square: 9 parity classes
    (2, 2, 10, 10, 16, 16, 5, 2, 2),
    (2, 2, 8, 8, 16, 16, 3, 2, 0),      # unpadded stride 2
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(hip, case):
    K, B, H, W, Ci, Co, k, s, p = case
    torch.manual_seed(0)
    x = _bf(K, B, H, W, Ci)
    w = _bf(K, Co, k, k, Ci, scale=0.2)
    y = hip.conv_fwd(x, w, s, p)
    y_ref = ref.conv_fwd(x.float(), w.float(), s, p)
    assert y.shape == y_ref.shape
    _close(y, y_ref)
    dy = _bf(*y.shape)
    dx = hip.conv_dgrad(dy, w, (H, W), s, p)
    _close(dx, ref.conv_dgrad(dy.float(), w.float(), (H, W), s, p))
    P = Co * k * k * Ci + 16
    gbuf = torch.full((K, P), 7.0, device=DEV)
    gw = gbuf[:, 8 : 8 + Co * k * k * Ci].unflatten(1, (Co, k, k, Ci))
    hip.conv_wgrad(dy, x, gw, s, p)
    _close(gw, ref.conv_wgrad(dy.float(), x.float(), (K, Co, k, k, Ci), s, p))
    assert torch.all(gbuf[:, :8] == 7.0) and torch.all(gbuf[:, 8 + Co * k * k * Ci :] == 7.0)


@pytest.mark.parametrize("case", [(2, 2, 9, 9, 64, 128, 3, 2, 1), (2, 3, 8, 8, 128, 64, 3, 1, 1),
                                  (2, 2, 6, 6, 24, 40, 3, 1, 1)])
def test_conv_nt_every_variant(hip, case):
    # every NT tile configuration (the heuristic picks one per shape; the benchmark sweeps all)
    K, B, H, W, Ci, Co, k, s, p = case
    x = _bf(K, B, H, W, Ci)
    w = _bf(K, Co, k, k, Ci, scale=0.2)
    dy = _bf(K, B, (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1, Co)
    y_ref = ref.conv_fwd(x.float(), w.float(), s, p)
    dx_ref = ref.conv_dgrad(dy.float(), w.float(), (H, W), s, p)
    try:
        for v in range(hip._C.conv_nt_num_variants()):
            hip.nt_variant = v
            _close(hip.conv_fwd(x, w, s, p), y_ref)
            _close(hip.conv_dgrad(dy, w, (H, W), s, p), dx_ref)
    finally:
        hip.nt_variant = -1


@pytest.mark.parametrize("case", [(2, 2, 9, 9, 64, 128, 3, 2, 1), (2, 3, 8, 8, 128, 64, 3, 1, 1),
                                  (3, 2, 6, 6, 24, 40, 3, 1, 1), (2, 8, 16, 16, 64, 64, 3, 1, 1)])
def test_conv_tn_every_variant(hip, case):
    K, B, H, W, Ci, Co, k, s, p = case
    x = _bf(K, B, H, W, Ci)
    dy = _bf(K, B, (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1, Co)
    exp = ref.conv_wgrad(dy.float(), x.float(), (K, Co, k, k, Ci), s, p)
    try:
        for v in range(hip._C.conv_tn_num_variants()):
            hip.tn_variant = v
            gw = torch.full((K, Co, k, k, Ci), 5.0, device=DEV)
            hip.conv_wgrad(dy, x, gw, s, p)
            _close(gw, exp)
    finally:
        hip.tn_variant = -1


GL_CASES = [
    # K, B, H, W, Ci, Co, k, stride, pad — csrc/conv_gl.hip (forced on: gl_mode = 1)
    (2, 2, 8, 8, 64, 128, 3, 1, 1),      # M = 128: a partial 256-row tile
    (2, 3, 9, 9, 64, 128, 3, 2, 1),      # stride 2, odd size: 4 dgrad parity classes
    (2, 2, 8, 8, 64, 128, 1, 2, 0),      # 1x1 stride 2: three empty dgrad classes (dx = 0)
    (1, 4, 16, 16, 128, 256, 3, 1, 1),   # 256-wide tiles, 4 row tiles
    (2, 2, 7, 7, 128, 384, 3, 1, 1),     # N tail of a 256-wide tile
    (2, 2, 8, 8, 128, 64, 3, 1, 1),      # N = 64 forward; dgrad N = Ci = 128
    (3, 2, 6, 6, 64, 200, 3, 1, 1),      # N % 8 == 0 tail (dgrad C = 200: falls back to conv_nt)
    (2, 8, 16, 16, 128, 128, 3, 1, 1),   # M = 2048 per client
]


@pytest.mark.parametrize("case", GL_CASES)
def test_conv_gl_fwd_dgrad(hip, case):
    K, B, H, W, Ci, Co, k, s, p = case
    torch.manual_seed(1)
    x = _bf(K, B, H, W, Ci)
    w = _bf(K, Co, k, k, Ci, scale=0.2)
    OH = (H + 2 * p - k) // s + 1
    assert hip._C.conv_gl_wanted(K, B * OH * OH, Co, Ci, k * k, 1)
    old = hip.gl_mode
    hip.gl_mode = 1
    try:
        y = hip.conv_fwd(x, w, s, p)
        _close(y, ref.conv_fwd(x.float(), w.float(), s, p))
        dy = _bf(*y.shape)
        dx = hip.conv_dgrad(dy, w, (H, W), s, p)
        _close(dx, ref.conv_dgrad(dy.float(), w.float(), (H, W), s, p))
        # the same results as the register-staged kernels
        hip.gl_mode = 0
        _close(hip.conv_fwd(x, w, s, p), y, tol=1e-2)
    finally:
        hip.gl_mode = old


@pytest.mark.parametrize("gl", [0, 1])
@pytest.mark.parametrize("case", [(2, 3, 8, 8, 64, 64, 3), (2, 2, 8, 8, 128, 128, 3), (3, 2, 6, 6, 64, 256, 1),
                                  (2, 2, 5, 5, 8, 24, 3)])
def test_conv_dgrad_accumulate(hip, gl, case):
    """dX + acc fused in the dgrad epilogue (identity-shortcut gradient, Fn.ResidualLink) on
    both the LDS-DMA and the register-staged kernels."""
    K, B, H, W, Ci, Co, k = case
    torch.manual_seed(2)
    w = _bf(K, Co, k, k, Ci, scale=0.2)
    dy = _bf(K, B, H, W, Co)
    acc = _bf(K, B, H, W, Ci)
    old = hip.gl_mode
    hip.gl_mode = gl
    try:
        dx = hip.conv_dgrad(dy, w, (H, W), 1, k // 2, acc=acc)
    finally:
        hip.gl_mode = old
    _close(dx, ref.conv_dgrad(dy.float(), w.float(), (H, W), 1, k // 2, acc=acc.float()))


def test_conv_gl_shared_weights_rep(hip):
    x = _bf(6, 4, 8, 8, 64)
    w = _bf(2, 128, 3, 3, 64, scale=0.2)
    old = hip.gl_mode
    hip.gl_mode = 1
    try:
        _close(hip.conv_fwd(x, w, 1, 1), ref.conv_fwd(x.float(), w.float(), 1, 1))
    finally:
        hip.gl_mode = old


def test_conv_weight_flip_t(hip):
    w = _bf(3, 72, 3, 3, 136)  # tails in both 64-wide tile dims
    wt = torch.empty((3, 136, 3, 3, 72), dtype=torch.bfloat16, device=DEV)
    hip._C.conv_weight_flip_t(w.data_ptr(), wt.data_ptr(), w.stride(0), 3, 72, 3, 3, 136,
                              torch.cuda.current_stream().cuda_stream)
    exp = w.flip(2, 3).permute(0, 4, 2, 3, 1).contiguous()
    assert torch.equal(wt, exp)


def test_conv_shared_weights_rep(hip):
    # eval path: 6 virtual clients share 2 weight rows (rep = 3)
    x = _bf(6, 2, 8, 8, 16)
    w = _bf(2, 32, 3, 3, 16, scale=0.2)
    _close(hip.conv_fwd(x, w, 1, 1), ref.conv_fwd(x.float(), w.float(), 1, 1))
    w1 = _bf(1, 32, 3, 3, 16, scale=0.2)
    _close(hip.conv_fwd(x, w1, 1, 1), ref.conv_fwd(x.float(), w1.float(), 1, 1))


def test_conv_large_wgrad_splitk(hip):
    # forces split-K atomics (few tiles, long pixel reduction)
    K, B, H, W, Ci, Co = 2, 32, 16, 16, 64, 64
    x = _bf(K, B, H, W, Ci)
    dy = _bf(K, B, H, W, Co)
    gw = torch.empty((K, Co, 3, 3, Ci), device=DEV)
    hip.conv_wgrad(dy, x, gw, 1, 1)
    _close(gw, ref.conv_wgrad(dy.float(), x.float(), (K, Co, 3, 3, Ci), 1, 1))


@pytest.mark.parametrize("N,Fi,Fo", [(96, 100, 300), (64, 2048, 100), (40, 24, 36)])
def test_linear_epilogue_fusions(hip, N, Fi, Fo):
    """ReLU / residual epilogues of the forward and the ReLU' gate of the dgrad (Transformer FFN)."""
    K = 3
    x = _bf(K, N, Fi)
    w = _bf(K, Fo, Fi, scale=0.1)
    b = _bf(K, Fo, scale=0.1)
    res = _bf(K, N, Fo)
    _close(hip.linear_fwd(x, w, b, relu=True), ref.linear_fwd(x.float(), w.float(), b.float(), relu=True))
    _close(hip.linear_fwd(x, w, b, acc=res), ref.linear_fwd(x.float(), w.float(), b.float(), acc=res.float()))
    dy = _bf(K, N, Fo)
    gate = torch.relu(_bf(K, N, Fi))
    out = hip.linear_dgrad(dy, w, gate=gate)
    _close(out, ref.linear_dgrad(dy.float(), w.float(), gate=gate.float()))
    assert torch.all(out[gate <= 0] == 0)


@pytest.mark.parametrize("N,Fi,Fo", [(64, 512, 10), (33, 100, 300), (128, 784, 200), (5, 84, 10)])
def test_linear(hip, N, Fi, Fo):
    K = 3
    x = _bf(K, N, Fi)
    w = _bf(K, Fo, Fi, scale=0.1)
    b = _bf(K, Fo)
    _close(hip.linear_fwd(x, w, b), ref.linear_fwd(x.float(), w.float(), b.float()))
    dy = _bf(K, N, Fo)
    _close(hip.linear_dgrad(dy, w), ref.linear_dgrad(dy.float(), w.float()))
    gw = torch.empty((K, Fo, Fi), device=DEV)
    gb = torch.empty((K, Fo), device=DEV)
    hip.linear_wgrad(dy, x, gw, gb)
    dw_ref, db_ref = ref.linear_wgrad(dy.float(), x.float(), True)
    _close(gw, dw_ref)
    _close(gb, db_ref)


@pytest.mark.parametrize("C", [64, 12, 3, 512])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_batchnorm(hip, C, relu, res):
    K, R = 3, 300
    x = _bf(K, R, C, scale=2.0) + 0.5
    g = _bf(K, C) + 1
    b = _bf(K, C)
    valid = torch.tensor([300, 150, 7], dtype=torch.int32, device=DEV)
    r = _bf(K, R, C) if res else None
    y, mean, rstd = hip.bn_fwd(x, g, b, valid, relu, r)
    y2, mean2, rstd2 = ref.bn_fwd(x.float(), g.float(), b.float(), valid, relu, r.float() if res else None)
    _close(mean, mean2, 1e-3)
    _close(rstd, rstd2, 1e-2)
    _close(y, y2)
    dy = _bf(K, R, C)
    gg = torch.zeros((K, C), device=DEV)
    gbeta = torch.zeros((K, C), device=DEV)
    dx, dpre = hip.bn_bwd(dy, x, y, mean, rstd, g, valid, relu, gg, gbeta, res)
    dx2, dg2, db2, dpre2 = ref.bn_bwd(dy.float(), x.float(), y.float(), mean2, rstd2, g.float(), valid, relu)
    if relu and C % 8 == 0:  # the 1-bit ReLU mask path gives the same gradients bit for bit
        y_m, _, _, mask = hip.bn_fwd(x, g, b, valid, relu, r, with_mask=True)
        assert torch.equal(y_m, y)
        bits = torch.stack([(mask >> j) & 1 for j in range(8)], -1).reshape(K, 300, C).bool()
        assert torch.equal(bits, y.float() > 0)
        gg2, gb2 = torch.zeros_like(gg), torch.zeros_like(gbeta)
        dx_m, dpre_m = hip.bn_bwd(dy, x, y, mean, rstd, g, valid, relu, gg2, gb2, res, relu_mask=mask)
        assert torch.equal(dx_m, dx) and torch.equal(gg2, gg)
    _close(dx, dx2, 3e-2)
    _close(gg, dg2, 2e-2)
    _close(gbeta, db2, 2e-2)
    if res:
        _close(dpre, dpre2)


def test_layernorm(hip):
    K, N, C = 2, 37, 100
    x = _bf(K, N, C)
    g = _bf(K, C) + 1
    b = _bf(K, C)
    y, mean, rstd = hip.ln_fwd(x, g, b)
    y2, m2, r2 = ref.ln_fwd(x.float(), g.float(), b.float())
    _close(y, y2)
    dy = _bf(K, N, C)
    dx, dg, db = hip.ln_bwd(dy, x, mean, rstd, g)
    dx2, dg2, db2 = ref.ln_bwd(dy.float(), x.float(), m2, r2, g.float())
    _close(dx, dx2, 3e-2)
    _close(dg, dg2, 2e-2)
    _close(db, db2, 2e-2)


@pytest.mark.parametrize("k,s,pad", [(2, 2, 0), (3, 2, 1)])
@pytest.mark.parametrize("C", [16, 6])  # 8-channel vector form and the scalar form
def test_maxpool(hip, k, s, pad, C):
    x = _bf(2, 3, 9, 9, C)
    y, idx = hip.maxpool_fwd(x, k, s, pad)
    y2, idx2 = ref.maxpool_fwd(x.float(), k, s, pad)
    _close(y, y2, 1e-6)
    dy = _bf(*y.shape)
    _close(hip.maxpool_bwd(dy, idx, x.shape, k, s, pad), ref.maxpool_bwd(dy.float(), idx2, x.shape, k, s, pad))


def test_avgpool_gap(hip):
    x = _bf(2, 3, 8, 8, 24)
    _close(hip.avgpool_fwd(x, 2, 2), ref.avgpool_fwd(x.float(), 2, 2))
    dy = _bf(2, 3, 4, 4, 24)
    _close(hip.avgpool_bwd(dy, x.shape, 2, 2), ref.avgpool_bwd(dy.float(), x.shape, 2, 2))
    _close(hip.gap_fwd(x), ref.gap_fwd(x.float()))
    dg = _bf(2, 3, 24)
    _close(hip.gap_bwd(dg, x.shape), ref.gap_bwd(dg.float(), x.shape))


@pytest.mark.parametrize("NC", [10, 100, 1000])
def test_cross_entropy(hip, NC):
    K, B = 3, 64
    logits = _bf(K, B, NC, scale=3)
    labels = torch.randint(0, NC, (K, B), device=DEV)
    valid = torch.tensor([64, 30, 1], dtype=torch.int32, device=DEV)
    l, c, d = hip.ce_fwd_bwd(logits, labels, valid)
    l2, c2, d2 = ref.ce_fwd_bwd(logits.float(), labels, valid)
    _close(l, l2, 1e-3)
    assert torch.equal(c, c2)
    _close(d, d2, 2e-2)


def test_sgd_and_fl_math(hip):
    K, P = 5, 4096
    theta = torch.randn(K, P, device=DEV)
    grad = torch.randn(K, P, device=DEV)
    mom = torch.randn(K, P, device=DEV)
    lr = torch.rand(K, device=DEV)
    active = torch.tensor([1, 1, 0, 1, 1], dtype=torch.bool, device=DEV)
    first = torch.tensor([1, 0, 0, 0, 1], dtype=torch.bool, device=DEV)
    t2, m2 = theta.clone(), mom.clone()
    shadow = theta.to(torch.bfloat16)  # inactive rows keep their shadow
    hip.sgd_step(theta, grad, mom, lr, active, 5e-4, 0.9, 0.0, False, first, shadow)
    ref.sgd_step(t2, grad, m2, lr, active, 5e-4, 0.9, 0.0, False, first)
    torch.testing.assert_close(theta, t2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mom, m2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(shadow.float(), theta.to(torch.bfloat16).float())
    w = torch.rand(K, device=DEV)
    torch.testing.assert_close(hip.weighted_sum(theta, w), ref.weighted_sum(theta, w), rtol=1e-5, atol=1e-5)
    base = torch.randn(P, device=DEV)
    torch.testing.assert_close(hip.delta_rows(theta, base), theta - base)
    rows = torch.empty(K, P, device=DEV)
    hip.broadcast_rows(rows, base)
    assert torch.equal(rows, base.expand(K, P))
    mask = torch.rand(K, P, device=DEV) > 0.5
    n1, d1 = hip.masked_weighted_sum(theta, mask, w)
    n2, d2 = ref.masked_weighted_sum(theta, mask, w)
    torch.testing.assert_close(n1, n2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(d1, d2)


@pytest.mark.parametrize("K,M", [(5, 3), (32, 32), (32, 70), (100, 33)])
def test_mix_rows(hip, K, M):
    P = 4096 + 48
    x = torch.randn(K, P, device=DEV)
    w = torch.rand(M, K, device=DEV)
    w = w / w.sum(1, keepdim=True)
    out = hip.mix_rows(x, w)
    assert out.dtype == torch.bfloat16 and out.shape == (M, P)
    torch.testing.assert_close(out.float(), ref.mix_rows(x, w, torch.float32), rtol=1e-2, atol=1e-2)


def test_compression_kernels(hip):
    """Native masks / sign packs / stochastic quantisation against the CPU torch oracle
    (the CPU path of ops.quant / ops.fl is the reference implementation)."""
    from distributed_learning_simulator_amd.ops import fl, quant

    K, P = 3, 1024
    seeds = fl.row_seeds(1234, [5, 0, 17])
    m_hip = hip.dropout_mask((K, P), 0.3, seeds)
    m_ref = fl.uniform_rows(seeds, P, DEV) >= 0.3
    assert torch.equal(m_hip, m_ref)
    g = torch.randn(K, P, device=DEV)
    g[0, :5] = 0.0  # sign(0) -> bit 1 on both paths
    packed = hip.sign_pack(g)
    assert torch.equal(packed.cpu(), quant.sign_pack(g.cpu()))
    votes = hip.sign_vote(packed, P)
    assert torch.equal(votes.cpu(), quant.sign_vote(packed.cpu(), P))
    active = torch.tensor([1, 0, 1], dtype=torch.bool, device=DEV)
    assert torch.equal(hip.sign_vote(packed, P, active).cpu(), quant.sign_vote(packed.cpu(), P, active.cpu()))
    seg = torch.cat([torch.zeros(500, dtype=torch.int32), torch.ones(524, dtype=torch.int32)]).to(DEV)
    seg_sizes = torch.tensor([500, 524])
    x = torch.randn(K, P, device=DEV)
    rs = fl.row_seeds(7, [0, 1, 2])
    dq, wire = quant.stochastic_quantize(x, seg, seg_sizes.to(DEV), rs)
    dq_cpu, wire_cpu = quant.stochastic_quantize(x.cpu(), seg.cpu(), seg_sizes, rs)
    assert wire == wire_cpu
    step = (x.abs().max() / 127).item()  # QSGD: 255 signed levels of the max-abs norm
    assert (dq - x).abs().max().item() <= step * 1.01
    # the same rounding decisions as the oracle (up to fp-contraction ties at a level boundary)
    diff = (dq.cpu() - dq_cpu).abs()
    assert (diff > 1e-5).float().mean().item() < 1e-3 and diff.max().item() <= step * 1.01
    # unbiasedness E[Q(x)] = x
    reps = torch.stack([hip.stochastic_qdq(x, seg, 2, fl.row_seeds(s, [0, 1, 2]), 255) for s in range(64)]).mean(0)
    assert (reps - x).abs().mean() < step * 0.1


def test_embedding_gather(hip):
    K, V, D = 2, 50, 16
    table = _bf(K, V, D)
    tok = torch.randint(0, V, (K, 3, 7), device=DEV)
    _close(hip.embedding_fwd(tok, table), ref.embedding_fwd(tok, table.float()))
    dy = _bf(K, 3, 7, D)
    gt = torch.empty(K, V, D, device=DEV)
    hip.embedding_bwd(dy, tok, gt)
    _close(gt, ref.embedding_bwd(dy.float(), tok, V))
    src = _bf(100, 4, 4, 8)
    idx = torch.randint(0, 100, (3, 5), device=DEV)
    assert torch.equal(hip.gather_rows(src, idx), src[idx.reshape(-1)])


@pytest.mark.parametrize("L,dh,masked", [(300, 20, True), (64, 32, False), (128, 64, True), (37, 16, True), (700, 8, True)])
def test_attention_fwd_bwd(hip, L, dh, masked):
    K, B, H = 2, 3, 2
    q, k, v = (_bf(K, B, H, L, dh) for _ in range(3))
    kv = torch.randint(1, L + 1, (K, B), device=DEV, dtype=torch.int32) if masked else None
    o, lse = hip.attn_fwd(q, k, v, kv)
    o_ref, lse_ref = ref.attn_fwd(q.float(), k.float(), v.float(), kv)
    _close(o, o_ref)
    torch.testing.assert_close(lse, lse_ref, rtol=1e-3, atol=1e-3)
    do = _bf(K, B, H, L, dh)
    dq, dk, dv = hip.attn_bwd(do, q, k, v, o, lse, kv)
    rq, rk, rv = ref.attn_bwd(do.float(), q.float(), k.float(), v.float(), o.float(), lse_ref, kv)
    _close(dq, rq, tol=3e-2)
    _close(dk, rk, tol=3e-2)
    _close(dv, rv, tol=3e-2)


def test_spmm_shared_and_flat(hip):
    torch.manual_seed(0)
    N, F, K, E = 500, 64, 3, 4000
    src = torch.randint(0, N, (E,), device=DEV)
    dst = torch.randint(0, N, (E,), device=DEV)
    val = torch.rand(E, device=DEV)
    from distributed_learning_simulator_amd.data.graph import EdgeSet

    es = EdgeSet(src, dst, val, 1, N)
    csr = es.csr()
    x = _bf(K, N, F)
    y = hip.spmm(csr.rowptr, csr.col, csr.val, x)
    exp = torch.zeros(K, N, F, device=DEV).index_add_(1, dst, x.float()[:, src] * val[None, :, None])
    _close(y, exp)
    yt = hip.spmm(csr.rowptr_t, csr.col_t, csr.val_t, x)
    expt = torch.zeros(K, N, F, device=DEV).index_add_(1, src, x.float()[:, dst] * val[None, :, None])
    _close(yt, expt)


def test_nnadq_native_matches_oracle(hip):
    from distributed_learning_simulator_amd.data.datasets import get_spec
    from distributed_learning_simulator_amd.models.zoo import build_model
    from distributed_learning_simulator_amd.ops import quant

    layout = build_model("LeNet5", get_spec("MNIST")).layout
    seg = layout.segment_ids()
    sizes = layout.segment_sizes()
    x = torch.randn(3, layout.padded_size) * layout.valid_mask().float()
    dq_cpu, wire_cpu, bits_cpu = quant.nnadq_quantize(x, seg, sizes, 0.001)
    dq_gpu, wire_gpu, bits_gpu = quant.nnadq_quantize(x.to(DEV), seg.to(DEV), sizes.to(DEV), 0.001)
    valid = layout.valid_mask()
    torch.testing.assert_close(dq_gpu.cpu()[:, valid], dq_cpu[:, valid], rtol=1e-5, atol=1e-6)
    assert wire_gpu == wire_cpu
    torch.testing.assert_close(bits_gpu.cpu(), bits_cpu)
