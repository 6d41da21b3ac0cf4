"""Reference-precision (fp32) kernels vs a float64 CPU oracle at <= 1e-5 relative error.

The reference trains in fp32 (`/root/reference/conf/global.yaml:7` `use_amp: false`). On gfx950
the GEMMs of this mode run as split-bf16 ("bf16x3") MFMA with fp32 storage and accumulation
(csrc/conv_f32.hip); every other kernel computes in fp32 on fp32 storage. Error metric: max
|out - exact| over max |exact| (the scale of the output), as in tests/test_kernels_gpu.py.
"""

import pytest
import torch

from distributed_learning_simulator_amd.ops import ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5


def _f(*shape, scale=1.0):
    return torch.randn(*shape, device=DEV) * scale


def _d(t):
    return t.detach().cpu().double()


def _vimg(t, valid):
    """The valid samples' images of a [K, B, ...] tensor, concatenated (the rows a tile-skipping
    halo conv leaves unwritten past a client's valid samples are never read: ConvNTParams::skip_valid)."""
    if valid is None:
        return t
    return torch.cat([t[k, : int(valid[k])].reshape(-1) for k in range(t.shape[0])])


def _close(out, exp, tol=TOL):
    out = out.detach().cpu().double()
    exp = exp.detach().cpu().double()
    assert out.shape == exp.shape, (out.shape, exp.shape)
    err = (out - exp).abs().max().item()
    mag = exp.abs().max().item() + 1e-12
    assert err <= tol * mag, f"rel err {err / mag:.3g} > {tol}"


CONV_CASES = [
    # K, B, H, W, Ci, Co, k, stride, pad
    (3, 4, 8, 8, 16, 32, 3, 1, 1),
    (2, 2, 8, 8, 64, 64, 3, 1, 1),
    (2, 3, 9, 9, 64, 128, 3, 2, 1),
    (2, 2, 8, 8, 64, 128, 1, 2, 0),
    (3, 2, 8, 8, 3, 64, 3, 1, 1),       # stem: Ci=3 scalar path
    (2, 2, 8, 8, 8, 64, 3, 1, 1),       # stem with RGB zero-padded to 8 channels
    (2, 2, 6, 6, 36, 12, 3, 1, 1),      # DenseNet-like: Ci%8==4, Co=12
    (2, 2, 12, 12, 1, 6, 5, 1, 2),      # LeNet conv1
    (2, 2, 7, 7, 128, 256, 3, 1, 1),
    (2, 2, 9, 7, 16, 32, 3, 3, 1),      # stride 3, non-square: 9 parity classes
    (2, 8, 16, 16, 64, 64, 3, 1, 1),    # long pixel reduction (split-K wgrad)
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_f32(hip, case):
    K, B, H, W, Ci, Co, k, s, p = case
    torch.manual_seed(0)
    x = _f(K, B, H, W, Ci)
    w = _f(K, Co, k, k, Ci, scale=0.2)
    y = hip.conv_fwd(x, w, s, p)
    assert y.dtype == torch.float32
    _close(y, ref.conv_fwd(_d(x), _d(w), s, p))
    dy = _f(*y.shape)
    dx = hip.conv_dgrad(dy, w, (H, W), s, p)
    _close(dx, ref.conv_dgrad(_d(dy), _d(w), (H, W), s, p))
    P = Co * k * k * Ci + 16
    gbuf = torch.full((K, P), 7.0, device=DEV)
    gw = gbuf[:, 8 : 8 + Co * k * k * Ci].unflatten(1, (Co, k, k, Ci))
    hip.conv_wgrad(dy, x, gw, s, p)
    _close(gw, ref.conv_wgrad(_d(dy), _d(x), (K, Co, k, k, Ci), s, p))
    assert torch.all(gbuf[:, :8] == 7.0) and torch.all(gbuf[:, 8 + Co * k * k * Ci :] == 7.0)


@pytest.mark.parametrize("case", [(2, 2, 9, 9, 64, 128, 3, 2, 1), (2, 3, 8, 8, 128, 64, 3, 1, 1),
                                  (2, 2, 6, 6, 24, 40, 3, 1, 1), (3, 2, 8, 8, 36, 12, 3, 1, 1)])
def test_conv_f32_every_variant(hip, case):
    """Every fp32 NT and TN tile configuration (the driver's fp32 `--variant` sweep ids)."""
    K, B, H, W, Ci, Co, k, s, p = case
    torch.manual_seed(3)
    x = _f(K, B, H, W, Ci)
    w = _f(K, Co, k, k, Ci, scale=0.2)
    OH = (H + 2 * p - k) // s + 1
    dy = _f(K, B, OH, (W + 2 * p - k) // s + 1, Co)
    y_ref = ref.conv_fwd(_d(x), _d(w), s, p)
    dx_ref = ref.conv_dgrad(_d(dy), _d(w), (H, W), s, p)
    dw_ref = ref.conv_wgrad(_d(dy), _d(x), (K, Co, k, k, Ci), s, p)
    stream = torch.cuda.current_stream().cuda_stream
    M = B * OH * ((W + 2 * p - k) // s + 1)
    for v in range(hip._C.conv_nt_f32_num_variants()):
        y = torch.empty_like(dy)
        hip._C.conv_nt(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, B * H * W * Ci, M * Co, w.stride(0), 0, B, H, W,
                       Ci, OH, y.shape[3], k, k, s, p, 1, M, Co, k * k * Ci, 1, 0, K, 0, v, 0, 0, 1, stream, 0, 0, 0, 0, 0, 0.0, 0.0,
                       0, 0, 0, 0, 0, 0, 0)
        _close(y, y_ref)
        dx = torch.empty_like(x)
        hip._C.conv_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), 0, w.stride(0), K, 1, B, OH, y.shape[3], Co, H,
                          W, Ci, k, k, s, p, v, 1, stream, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
        _close(dx, dx_ref)
    for v in range(hip._C.conv_tn_f32_num_variants()):
        gw = torch.zeros((K, Co, k, k, Ci), device=DEV)
        hip._C.conv_tn(dy.data_ptr(), x.data_ptr(), gw.data_ptr(), M * Co, B * H * W * Ci, gw.stride(0), B, H, W, Ci,
                       OH, dy.shape[3], k, k, s, p, M, Co, k * k * Ci, K, v, 1, stream, 0, 0, 0, 0, 0, None)
        _close(gw, dw_ref)


@pytest.mark.parametrize("N,Fi,Fo", [(64, 512, 10), (33, 100, 300), (128, 784, 200), (5, 84, 10), (96, 512, 2048)])
def test_linear_f32(hip, N, Fi, Fo):
    K = 3
    torch.manual_seed(1)
    x = _f(K, N, Fi)
    w = _f(K, Fo, Fi, scale=0.1)
    b = _f(K, Fo)
    _close(hip.linear_fwd(x, w, b), ref.linear_fwd(_d(x), _d(w), _d(b)))
    res = _f(K, N, Fo)
    _close(hip.linear_fwd(x, w, b, acc=res), ref.linear_fwd(_d(x), _d(w), _d(b), acc=_d(res)))
    _close(hip.linear_fwd(x, w, b, relu=True), ref.linear_fwd(_d(x), _d(w), _d(b), relu=True))
    dy = _f(K, N, Fo)
    _close(hip.linear_dgrad(dy, w), ref.linear_dgrad(_d(dy), _d(w)))
    gate = torch.relu(_f(K, N, Fi))
    _close(hip.linear_dgrad(dy, w, gate=gate), ref.linear_dgrad(_d(dy), _d(w), gate=_d(gate)))
    gw = torch.empty((K, Fo, Fi), device=DEV)
    gb = torch.empty((K, Fo), device=DEV)
    hip.linear_wgrad(dy, x, gw, gb)
    dw_ref, db_ref = ref.linear_wgrad(_d(dy), _d(x), True)
    _close(gw, dw_ref)
    _close(gb, db_ref)


def test_conv_f32_dgrad_accumulate_and_bias(hip):
    K, B, H, W, Ci, Co = 2, 3, 8, 8, 64, 64
    w = _f(K, Co, 3, 3, Ci, scale=0.2)
    dy = _f(K, B, H, W, Co)
    acc = _f(K, B, H, W, Ci)
    _close(hip.conv_dgrad(dy, w, (H, W), 1, 1, acc=acc), ref.conv_dgrad(_d(dy), _d(w), (H, W), 1, 1, acc=_d(acc)))
    x = _f(K, B, H, W, Ci)
    b = _f(K, Co)
    _close(hip.conv_fwd(x, w, 1, 1, bias=b), ref.conv_fwd(_d(x), _d(w), 1, 1, bias=_d(b)))
    gb = torch.empty((K, Co), device=DEV)
    hip.bias_grad(dy, gb)
    _close(gb, _d(dy).sum(dim=(1, 2, 3)))


@pytest.mark.parametrize("C", [64, 12, 3])
@pytest.mark.parametrize("relu,res", [(False, False), (True, True)])
def test_batchnorm_f32(hip, C, relu, res):
    K, R = 3, 300
    torch.manual_seed(2)
    x = _f(K, R, C, scale=2.0) + 0.5
    g = _f(K, C) + 1
    b = _f(K, C)
    valid = torch.tensor([300, 150, 7], dtype=torch.int32, device=DEV)
    r = _f(K, R, C) if res else None
    y, mean, rstd = hip.bn_fwd(x, g, b, valid, relu, r)
    y2, mean2, rstd2 = ref.bn_fwd(_d(x), _d(g), _d(b), valid.cpu(), relu, _d(r) if res else None)
    _close(mean, mean2, 1e-5)
    _close(rstd, rstd2, 1e-5)
    _close(y, y2)
    dy = _f(K, R, C)
    gg = torch.zeros((K, C), device=DEV)
    gbeta = torch.zeros((K, C), device=DEV)
    dx, dpre = hip.bn_bwd(dy, x, y, mean, rstd, g, valid, relu, gg, gbeta, res)
    dx2, dg2, db2, dpre2 = ref.bn_bwd(_d(dy), _d(x), y2, mean2, rstd2, _d(g), valid.cpu(), relu)
    _close(dx, dx2, 2e-5)
    _close(gg, dg2)
    _close(gbeta, db2)
    if res:
        _close(dpre, dpre2)


def test_layernorm_f32(hip):
    K, N, C = 2, 37, 100
    x, g, b = _f(K, N, C), _f(K, C) + 1, _f(K, C)
    y, mean, rstd = hip.ln_fwd(x, g, b)
    y2, m2, r2 = ref.ln_fwd(_d(x), _d(g), _d(b))
    _close(y, y2)
    dy = _f(K, N, C)
    dx, dg, db = hip.ln_bwd(dy, x, mean, rstd, g)
    dx2, dg2, db2 = ref.ln_bwd(_d(dy), _d(x), m2, r2, _d(g))
    _close(dx, dx2, 2e-5)
    _close(dg, dg2)
    _close(db, db2)


def test_pool_gap_ce_f32(hip):
    x = _f(2, 3, 9, 9, 16)
    y, idx = hip.maxpool_fwd(x, 3, 2, 1)
    y2, idx2 = ref.maxpool_fwd(_d(x), 3, 2, 1)
    _close(y, y2)
    dy = _f(*y.shape)
    _close(hip.maxpool_bwd(dy, idx, x.shape, 3, 2, 1), ref.maxpool_bwd(_d(dy), idx2, x.shape, 3, 2, 1))
    x = _f(2, 3, 8, 8, 24)
    _close(hip.avgpool_fwd(x, 2, 2), ref.avgpool_fwd(_d(x), 2, 2))
    dy = _f(2, 3, 4, 4, 24)
    _close(hip.avgpool_bwd(dy, x.shape, 2, 2), ref.avgpool_bwd(_d(dy), x.shape, 2, 2))
    _close(hip.gap_fwd(x), _d(x).mean(dim=(2, 3)))
    K, B, NC = 3, 64, 100
    logits = _f(K, B, NC, scale=3)
    labels = torch.randint(0, NC, (K, B), device=DEV)
    valid = torch.tensor([64, 30, 1], dtype=torch.int32, device=DEV)
    l, c, d = hip.ce_fwd_bwd(logits, labels, valid)
    l2, c2, d2 = ref.ce_fwd_bwd(_d(logits), labels.cpu(), valid.cpu())
    _close(l, l2)
    assert torch.equal(c.cpu(), c2.float())
    _close(d, d2)


@pytest.mark.parametrize("L,dh", [(300, 20), (128, 64)])
def test_attention_embedding_f32(hip, L, dh):
    K, B, H = 2, 2, 2
    q, k, v = (_f(K, B, H, L, dh) for _ in range(3))
    kv = torch.randint(1, L + 1, (K, B), device=DEV, dtype=torch.int32)
    o, lse = hip.attn_fwd(q, k, v, kv)
    o2, lse2 = ref.attn_fwd(_d(q), _d(k), _d(v), kv.cpu())
    _close(o, o2, 3e-5)
    do = _f(K, B, H, L, dh)
    dq, dk, dv = hip.attn_bwd(do, q, k, v, o, lse, kv)
    rq, rk, rv = ref.attn_bwd(_d(do), _d(q), _d(k), _d(v), o2, lse2, kv.cpu())
    _close(dq, rq, 3e-5)
    _close(dk, rk, 3e-5)
    _close(dv, rv, 3e-5)
    table = _f(K, 50, 16)
    tok = torch.randint(0, 50, (K, 3, 7), device=DEV)
    assert torch.equal(hip.embedding_fwd(tok, table), ref.embedding_fwd(tok, table))


def test_mix_rows_f32_and_gather(hip):
    K, M, P = 300, 40, 4096 + 48  # K > 256: chunked native passes
    x = torch.randn(K, P, device=DEV)
    w = torch.rand(M, K, device=DEV)
    out = hip.mix_rows(x, w, torch.float32)
    assert out.dtype == torch.float32
    _close(out, _d(w) @ _d(x))
    src = _f(100, 4, 4, 4)
    idx = torch.randint(0, 100, (3, 5), device=DEV)
    assert torch.equal(hip.gather_rows(src, idx), src[idx.reshape(-1)])


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 6e-2)])
def test_dense_block_strided_kernels_match_cpu(hip, dtype, tol):
    """DenseNet block on the GPU: BN reads channel prefixes of the block buffer in place, convs
    write their 12 new channels through the epilogue row stride, the backward accumulates into
    channel slices of dF — against the CPU autograd-verified path (tests/test_models.py)."""
    from distributed_learning_simulator_amd.data.datasets import get_spec
    from distributed_learning_simulator_amd.engine.params import BoundParams
    from distributed_learning_simulator_amd.models.layers import RunCtx
    from distributed_learning_simulator_amd.models.zoo import build_model
    from distributed_learning_simulator_amd.ops import functional as Fn

    model = build_model("densenet10", get_spec("CIFAR10"))
    layout = model.layout
    K = 3
    theta = torch.stack([layout.init_flat(torch.Generator().manual_seed(s)) for s in range(K)])
    g = torch.Generator().manual_seed(7)  # (fixed data: a ReLU input within rounding of 0 may gate
    x = torch.randn(K, 6, 32, 32, 8, generator=g)  # differently on the two paths)
    x[..., 3:] = 0
    y = torch.randint(0, 10, (K, 6), generator=g)
    valid = torch.tensor([6, 4, 1], dtype=torch.int32)
    out = {}
    for dev in ("cpu", "cuda"):
        th = theta.to(dev)
        comp = th if (dev == "cpu" or dtype == torch.float32) else th.to(dtype)
        grad = torch.zeros_like(th)
        ctx = RunCtx(BoundParams(layout, comp, grad), valid.to(dev))
        xi = x.to(dev, torch.float32 if dev == "cpu" else dtype)
        loss, _ = Fn.cross_entropy(model.forward(xi, ctx), y.to(dev), ctx.valid)
        loss.sum().backward()
        out[dev] = (loss.detach().cpu(), grad.cpu())
    _close(out["cuda"][0], out["cpu"][0], tol)
    _close(out["cuda"][1], out["cpu"][1], tol * 5)


@pytest.mark.parametrize("L,dh", [(37, 32), (200, 64), (128, 64), (300, 32)])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 3e-5), (torch.bfloat16, 2.5e-2)])
def test_attention_mfma(hip, L, dh, dtype, tol):
    """MFMA flash attention (csrc/attention_mfma.hip): ragged key padding, partial 128-row blocks,
    bf16 and split-bf16 fp32, against the float64 oracle."""
    K, B, H = 2, 2, 2
    torch.manual_seed(L + dh)
    q, k, v = (_f(K, B, H, L, dh).to(dtype) for _ in range(3))
    kv = torch.randint(1, L + 1, (K, B), device=DEV, dtype=torch.int32)
    kv[0, 0] = L
    o, lse = hip.attn_fwd(q, k, v, kv)
    o2, lse2 = ref.attn_fwd(_d(q), _d(k), _d(v), kv.cpu())
    _close(o, o2, tol)
    _close(lse, lse2, max(tol, 1e-5))
    do = _f(K, B, H, L, dh).to(dtype)
    dq, dk, dv = hip.attn_bwd(do, q, k, v, o, lse, kv)
    rq, rk, rv = ref.attn_bwd(_d(do), _d(q), _d(k), _d(v), o2, lse2, kv.cpu())
    _close(dq, rq, tol * 2)
    _close(dk, rk, tol * 2)
    _close(dv, rv, tol * 2)
    # padded keys get exactly zero gradient
    for kk in range(K):
        for bb in range(B):
            n = int(kv[kk, bb])
            assert torch.all(dk[kk, bb, :, n:] == 0) and torch.all(dv[kk, bb, :, n:] == 0)


@pytest.mark.parametrize("L,H,D", [(200, 8, 512), (37, 4, 128), (130, 2, 64)])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 3e-5), (torch.bfloat16, 2.5e-2)])
def test_attention_packed_qkv(hip, L, H, D, dtype, tol):
    """Attention read straight from the QKV projection rows [K, B, L, 3D] (strided heads, no
    permute copies) and the gradient written back in that layout: against the float64 oracle
    applied to the explicitly split / permuted q, k, v."""
    K, B = 2, 2
    dh = D // H
    if not hip.attn_packed_supported(L, dh):
        pytest.skip("no packed kernel for this head dim")
    torch.manual_seed(L + D)
    qkv = _f(K, B, L, 3 * D).to(dtype)
    kv = torch.randint(1, L + 1, (K, B), device=DEV, dtype=torch.int32)
    o, lse = hip.attn_fwd_packed(qkv, H, kv)
    assert o.shape == (K, B, L, D)

    def heads(t):  # [K,B,L,D] → [K,B,H,L,dh]
        return t.reshape(K, B, L, H, dh).permute(0, 1, 3, 2, 4)

    q, k, v = (heads(_d(t)) for t in qkv.split(D, dim=-1))
    o2, lse2 = ref.attn_fwd(q, k, v, kv.cpu())
    _close(o, o2.permute(0, 1, 3, 2, 4).reshape(K, B, L, D), tol)
    _close(lse, lse2, max(tol, 1e-5))
    do = _f(K, B, L, D).to(dtype)
    dqkv = hip.attn_bwd_packed(do, qkv, o, lse, H, kv)
    rq, rk, rv = ref.attn_bwd(heads(_d(do)), q, k, v, o2, lse2, kv.cpu())
    flat = lambda t: t.permute(0, 1, 3, 2, 4).reshape(K, B, L, D)  # noqa: E731
    _close(dqkv, torch.cat([flat(rq), flat(rk), flat(rv)], -1), tol * 2)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-6), (torch.bfloat16, 1e-2)])
def test_embedding_scale_pe_and_seq_mean(hip, dtype, tol):
    """Fused Transformer input (table[tok]·√d + PE) and masked mean pooling, fwd + bwd."""
    K, B, L, V, D = 3, 4, 37, 100, 64
    table = _f(K, V, D).to(dtype)
    tok = torch.randint(0, V, (K, B, L), device=DEV)
    pe = torch.randn(L, D, device=DEV)
    s = D ** 0.5
    out = hip.embedding_fwd(tok, table, s, pe)
    exp = ref.embedding_fwd(tok.cpu(), _d(table), s, pe.cpu().double())
    _close(out, exp, tol)
    dy = _f(K, B, L, D).to(dtype)
    g = torch.empty(K, V, D, device=DEV, dtype=torch.float32)
    hip.embedding_bwd(dy, tok, g, s)
    _close(g, ref.embedding_bwd(_d(dy), tok.cpu(), V, s), max(tol, 1e-5))
    x = _f(K, B, L, D).to(dtype)
    lengths = torch.randint(1, L + 1, (K, B), device=DEV, dtype=torch.int32)
    _close(hip.seq_mean_fwd(x, lengths), ref.seq_mean_fwd(_d(x), lengths.cpu()), tol)
    dp = _f(K, B, D).to(dtype)
    _close(hip.seq_mean_bwd(dp, lengths, L), ref.seq_mean_bwd(_d(dp), lengths.cpu(), L), tol)


@pytest.mark.parametrize("case", [(3, 4, 8, 8, 16, 64, 3, 1, 1), (2, 5, 9, 9, 64, 128, 3, 2, 1),
                                  (2, 3, 8, 8, 32, 256, 1, 1, 0), (3, 41, 8, 8, 16, 24, 3, 1, 1)])
def test_conv_epilogue_bn_stats(hip, case):
    """fp32 conv epilogue writes the BN partial sums (per 32 GEMM rows, valid samples only):
    their totals match fp64 sums over y, and bn_fwd(pre_stats=) equals bn_fwd's own pass (the
    last case has 82 partials per client: the wide fp64 fold stage runs, with a ragged last fold)."""
    K, B, H, W, Ci, Co, k, s, p = case
    x = _f(K, B, H, W, Ci)
    w = _f(K, Co, k, k, Ci, scale=0.2)
    valid = torch.tensor([B, B - 2, 1][:K], dtype=torch.int32, device=DEV)
    OH = (H + 2 * p - k) // s + 1
    M = B * OH * OH
    stats = torch.full((K, hip.conv_stats_parts(M), 2, Co), float("nan"), device=DEV)
    y = hip.conv_fwd(x, w, s, p, stats=stats, stats_valid=valid)
    assert torch.isfinite(stats).all()  # every partial slot written
    y3 = _d(y).reshape(K, M, Co)
    for kk in range(K):
        rows = int(valid[kk]) * OH * OH
        _close(stats[kk, :, 0].double().sum(0), y3[kk, :rows].sum(0), 1e-5)
        _close(stats[kk, :, 1].double().sum(0), (y3[kk, :rows] ** 2).sum(0), 1e-5)
    g = torch.rand(K, Co, device=DEV) + 0.5
    b = _f(K, Co)
    vr = valid * OH * OH
    ya, ma, ra, mka = hip.bn_fwd(y.reshape(K, M, Co), g, b, vr, True, None, with_mask=True)
    yb, mb, rb, mkb = hip.bn_fwd(y.reshape(K, M, Co), g, b, vr, True, None, with_mask=True, pre_stats=stats)
    _close(mb, ma, 1e-5)
    _close(rb, ra, 1e-4)
    _close(yb, ya, 1e-4)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
def test_linear_epilogue_dropout_matches_cpu_rule(hip, dtype, tol):
    """Dropout in the GEMM epilogue (before the residual add) and the standalone dropout_apply
    use exactly the CPU oracle's keep rule (ref.dropout_keep); the dgrad gate carries the scale."""
    K, N, Fi, Fo, p = 3, 200, 96, 64, 0.3
    x, w, b, r = _f(K, N, Fi).to(dtype), _f(K, Fo, Fi, scale=0.1).to(dtype), _f(K, Fo).to(dtype), _f(K, N, Fo).to(dtype)
    seeds = torch.tensor([5, -7, 123456789], dtype=torch.int32, device=DEV)
    y = hip.linear_fwd(x, w, b, acc=r, drop_p=p, drop_seeds=seeds)
    exp = ref.linear_fwd(_d(x), _d(w), _d(b), acc=_d(r), drop_p=p, drop_seeds=seeds.cpu())
    _close(y, exp, tol)
    keep = ref.dropout_keep(K, N, Fo, seeds.cpu(), p)
    y0 = hip.linear_fwd(x, w, b, drop_p=p, drop_seeds=seeds)  # (no residual: drops are exact zeros)
    assert torch.equal(y0.cpu() != 0, keep)  # dropped exactly where the rule says
    d = _f(K, N, Fo).to(dtype)
    torch.testing.assert_close(hip.dropout_apply(d, seeds, p).cpu().float(),
                               ref.dropout_apply(d.cpu().float(), seeds.cpu(), p), rtol=tol, atol=tol)
    gate = torch.relu(_f(K, N, Fi)).to(dtype)
    dy = _f(K, N, Fo).to(dtype)
    _close(hip.linear_dgrad(dy, w, gate=gate, gate_scale=1 / (1 - p)),
           ref.linear_dgrad(_d(dy), _d(w), gate=_d(gate), gate_scale=1 / (1 - p)), tol)


def test_synthetic_image_generator_matches_cpu(hip):
    """ImageNet-size synthetic images are generated by one HIP pass, bit-identical to the
    torch generator the CPU path uses (same data on every device)."""
    from distributed_learning_simulator_amd.data.datasets import ImageDataset, get_spec

    spec = get_spec("ImageNet", {"scale": 0.0005})
    cpu = ImageDataset(spec, "train", 3, torch.device("cpu"), torch.float32, materialize_limit=0, channels=8)
    gpu = ImageDataset(spec, "train", 3, torch.device(DEV), torch.float32, materialize_limit=0, channels=8)
    idx = torch.tensor([0, 5, 17, spec.n_train - 1])
    a = gpu.gather(idx.to(DEV)).cpu()
    b = cpu.gather(idx)
    assert a.shape == b.shape == (4, 224, 224, 8)
    assert torch.equal(a, b)


@pytest.mark.parametrize("case", [(3, 2, 8, 8, 64, 128, 3, 1, 1), (2, 2, 9, 9, 64, 128, 3, 2, 1),
                                  (2, 3, 8, 8, 64, 64, 3, 1, 1), (2, 2, 8, 8, 128, 256, 1, 2, 0)])
def test_conv_presplit_weight_planes(hip, case):
    """Pre-split weight planes (the SGD kernel's `split` output, read by the fp32 conv fwd / dgrad
    instead of splitting w per workgroup) give bit-identical results to the in-kernel split, and
    sgd_step(split=) writes exactly split_rows(θ_new)."""
    from distributed_learning_simulator_amd.ops import ref

    K, B, H, W, Ci, Co, k, s, p = case
    torch.manual_seed(5)
    n = Co * k * k * Ci
    P = ((n + 32 + 15) // 16) * 16
    theta = _f(K, P, scale=0.2)
    grad, mom = _f(K, P), torch.zeros(K, P, device=DEV)
    split = torch.zeros((K, 2, P), dtype=torch.bfloat16, device=DEV)
    lr = torch.full((K,), 0.05, device=DEV)
    on = torch.ones(K, dtype=torch.bool, device=DEV)
    hip.sgd_step(theta, grad, mom, lr, on, 0.0, 0.9, 0.0, False, on, None, split)
    exp = torch.zeros_like(split)
    hip.split_rows(theta, exp)
    assert torch.equal(split, exp)
    ref_split = torch.zeros_like(split)
    ref.split_rows(theta, ref_split)
    assert torch.equal(split, ref_split)  # CPU rule == GPU planes (RNE hi, RNE lo)
    w = theta[:, 16 : 16 + n].unflatten(1, (Co, k, k, Ci))
    ws = split[:, 0, 16 : 16 + n].unflatten(1, (Co, k, k, Ci))
    x = _f(K, B, H, W, Ci)
    y0 = hip.conv_fwd(x, w, s, p)
    y1 = hip.conv_fwd(x, w, s, p, w_split=ws)
    assert torch.equal(y0, y1)
    dy = _f(*y0.shape)
    dx0 = hip.conv_dgrad(dy, w, (H, W), s, p)
    dx1 = hip.conv_dgrad(dy, w, (H, W), s, p, w_split=ws)
    assert torch.equal(dx0, dx1)
    _close(y1, ref.conv_fwd(_d(x), _d(w), s, p))


def test_linear_presplit_weight_planes(hip):
    """Linear fwd / dgrad with pre-split weight planes == the in-kernel split, bit for bit."""
    torch.manual_seed(6)
    K, N, Fi, Fo = 3, 77, 256, 512
    P = Fo * Fi + 16
    theta = _f(K, P, scale=0.05)
    split = torch.zeros((K, 2, P), dtype=torch.bfloat16, device=DEV)
    hip.split_rows(theta, split)
    w = theta[:, :Fo * Fi].unflatten(1, (Fo, Fi))
    ws = split[:, 0, :Fo * Fi].unflatten(1, (Fo, Fi))
    x, b = _f(K, N, Fi), _f(K, Fo)
    assert torch.equal(hip.linear_fwd(x, w, b), hip.linear_fwd(x, w, b, w_split=ws))
    dy = _f(K, N, Fo)
    assert torch.equal(hip.linear_dgrad(dy, w), hip.linear_dgrad(dy, w, w_split=ws))


def _wsplit(hip, w):
    """Pre-split weight planes as the SGD step keeps them: hi-plane view into a [K, 2, P] buffer."""
    K = w.shape[0]
    ws = torch.empty((K, 2, w[0].numel()), dtype=torch.bfloat16, device=DEV)
    hip.split_rows(w.reshape(K, -1).contiguous(), ws)
    return ws[:, 0].view(w.shape)


PLANES_CASES = [
    # K, B, H, W, Ci, Co, k, stride, pad
    (2, 2, 8, 8, 64, 64, 3, 1, 1),
    (2, 3, 9, 9, 64, 128, 3, 2, 1),    # stride 2: four dgrad parity classes
    (2, 2, 8, 8, 64, 128, 1, 2, 0),    # 1x1 downsample shortcut (a class with no tap)
    (3, 2, 7, 7, 128, 256, 3, 1, 1),
    (2, 2, 5, 5, 32, 40, 3, 1, 1),     # N tail (40 of a 64 / 128 tile)
    (2, 4, 4, 4, 256, 512, 3, 1, 1),
]


@pytest.mark.parametrize("case", PLANES_CASES)
def test_conv_planes_every_variant(hip, case):
    """LDS-DMA GEMMs on pre-split operands (csrc/conv_pl.hip): every tile variant is bit-identical
    to the register-staged split-bf16 kernel (same hi / lo values, same product order) and within
    1e-5 of the fp64 oracle, forward and dgrad (k-major weight read in place, parity classes)."""
    K, B, H, W, Ci, Co, k, s, p = case
    torch.manual_seed(5)
    x = _f(K, B, H, W, Ci)
    w = _f(K, Co, k, k, Ci, scale=0.2)
    ws = _wsplit(hip, w)
    y_base = hip.conv_fwd(x, w, s, p, w_split=ws)
    _close(y_base, ref.conv_fwd(_d(x), _d(w), s, p))
    dy = _f(*y_base.shape)
    acc = _f(K, B, H, W, Ci)
    dx_base = hip.conv_dgrad(dy, w, (H, W), s, p, acc=acc, w_split=ws)
    _close(dx_base, ref.conv_dgrad(_d(dy), _d(w), (H, W), s, p) + _d(acc))
    xp, dyp = hip.split_planes(x), hip.split_planes(dy)
    try:
        for v in range(hip._C.conv_nt_pl_num_variants()):
            hip._C.conv_nt_pl_set_variant(v)
            y = hip.conv_fwd(x, w, s, p, w_split=ws, x_planes=xp)
            assert torch.equal(y, y_base), f"variant {v} fwd differs"
            dx = hip.conv_dgrad(dy, w, (H, W), s, p, acc=acc, w_split=ws, dy_planes=dyp)
            assert torch.equal(dx, dx_base), f"variant {v} dgrad differs"
    finally:
        hip._C.conv_nt_pl_set_variant(-1)


@pytest.mark.parametrize("case", PLANES_CASES + [(2, 8, 16, 16, 64, 64, 3, 1, 1), (3, 2, 8, 8, 8, 64, 3, 1, 1)])
def test_wgrad_planes_every_variant(hip, case):
    """Pre-split wgrad (csrc/conv_pl.hip TN, split-K slabs + ordered fold): every tile variant
    within 1e-5 of the fp64 oracle and bitwise-reproducible run to run; the register-staged
    fp32 wgrad with the deterministic fold likewise reproducible."""
    K, B, H, W, Ci, Co, k, s, p = case
    torch.manual_seed(7)
    x = _f(K, B, H, W, Ci)
    OH = (H + 2 * p - k) // s + 1
    OW = (W + 2 * p - k) // s + 1
    dy = _f(K, B, OH, OW, Co)
    exp = ref.conv_wgrad(_d(dy), _d(x), (K, Co, k, k, Ci), s, p)
    gw0 = torch.empty((K, Co, k, k, Ci), device=DEV)
    hip.conv_wgrad(dy, x, gw0, s, p)
    _close(gw0, exp)
    gw1 = torch.full_like(gw0, 3.0)
    hip.conv_wgrad(dy, x, gw1, s, p)
    assert torch.equal(gw0, gw1), "fp32 wgrad not reproducible"
    xp, dyp = hip.split_planes(x), hip.split_planes(dy)
    try:
        for v in range(hip._C.conv_tn_pl_num_variants()):
            hip._C.conv_tn_pl_set_variant(v)
            ga = torch.full_like(gw0, 5.0)
            hip.conv_wgrad(dy, x, ga, s, p, dy_planes=dyp, x_planes=xp)
            _close(ga, exp)
            gb = torch.full_like(gw0, -5.0)
            hip.conv_wgrad(dy, x, gb, s, p, dy_planes=dyp, x_planes=xp)
            assert torch.equal(ga, gb), f"variant {v} not reproducible"
    finally:
        hip._C.conv_tn_pl_set_variant(-1)


@pytest.mark.parametrize("case", [
    # K, B, H, Ci, Co  (3x3, stride 1, pad 1, H = W): one case per compiled halo tile shape
    (2, 2, 32, 32, 64),     # 1 x 8 x 32 rows, BN 64
    (2, 2, 16, 64, 128),    # 1 x 16 x 16, BN 128
    (2, 4, 8, 64, 96),      # 2 x 8 x 8, BN 128 (N tail)
    (3, 8, 4, 128, 128),    # 8 x 4 x 4
])
def test_conv_halo(hip, case):
    """3x3 stride-1 split-plane conv with LDS halo reuse (csrc/conv_halo.hip): forward and
    dgrad (+acc) within 1e-5 of the fp64 oracle and close to the implicit-GEMM plane kernel
    (different K-loop order: chunk-major instead of tap-major)."""
    K, B, H, Ci, Co = case
    torch.manual_seed(11)
    x = _f(K, B, H, H, Ci)
    w = _f(K, Co, 3, 3, Ci, scale=0.2)
    ws = _wsplit(hip, w)
    dy = _f(K, B, H, H, Co)
    acc = _f(K, B, H, H, Ci)
    xp, dyp = hip.split_planes(x), hip.split_planes(dy)
    outs = {}
    try:
        for mode, v in ((1, 0), (1, 1), (1, 2), (0, -1)):
            hip._C.conv_halo_set_mode(mode)
            hip._C.conv_halo_set_variant(v)
            outs[(mode, v)] = (hip.conv_fwd(x, w, 1, 1, w_split=ws, x_planes=xp),
                               hip.conv_dgrad(dy, w, (H, H), 1, 1, acc=acc, w_split=ws, dy_planes=dyp))
    finally:
        hip._C.conv_halo_set_mode(-1)
        hip._C.conv_halo_set_variant(-1)
    y_ref = ref.conv_fwd(_d(x), _d(w), 1, 1)
    dx_ref = ref.conv_dgrad(_d(dy), _d(w), (H, H), 1, 1) + _d(acc)
    for key, (y, dx) in outs.items():
        _close(y, y_ref)
        _close(dx, dx_ref)
    for key in ((1, 1), (1, 2)):  # every halo variant: same K order, bitwise equal
        assert torch.equal(outs[key][0], outs[(1, 0)][0]) and torch.equal(outs[key][1], outs[(1, 0)][1])
    _close(outs[(1, 0)][0], outs[(0, -1)][0].double(), tol=2e-6)
    _close(outs[(1, 0)][1], outs[(0, -1)][1].double(), tol=2e-6)


@pytest.mark.parametrize("L,H,D", [(300, 5, 100), (128, 8, 512), (37, 2, 16)])
@pytest.mark.parametrize("drop_p", [0.0, 0.1])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 3e-5), (torch.bfloat16, 2.5e-2)])
def test_attention_padded_heads_and_dropout(hip, L, H, D, drop_p, dtype, tol):
    """MFMA flash attention at the reference imdb model's dh = 20 (d_model 100, 5 heads: padded
    to 32 on the MFMA, packed QKV rows read in place) and with attention-probability dropout
    (nn.MultiheadAttention's dropout): against the float64 oracle with the same hash mask."""
    K, B = 2, 3
    dh = D // H
    assert hip.attn_packed_supported(L, dh)
    torch.manual_seed(L + D)
    qkv = _f(K, B, L, 3 * D).to(dtype)
    kv = torch.randint(1, L + 1, (K, B), device=DEV, dtype=torch.int32)
    seeds = torch.tensor([5, -9], dtype=torch.int32, device=DEV)
    dr = {"drop_p": drop_p, "drop_seeds": seeds} if drop_p else {}
    rdr = {"drop_p": drop_p, "drop_seeds": seeds.cpu()} if drop_p else {}
    o, lse = hip.attn_fwd_packed(qkv, H, kv, **dr)

    def heads(t):
        return t.reshape(K, B, L, H, dh).permute(0, 1, 3, 2, 4)

    q, k, v = (heads(_d(t)) for t in qkv.split(D, dim=-1))
    o2, lse2 = ref.attn_fwd(q, k, v, kv.cpu(), **rdr)
    flat = lambda t: t.permute(0, 1, 3, 2, 4).reshape(K, B, L, D)  # noqa: E731
    _close(o, flat(o2), tol)
    _close(lse, lse2, max(tol, 1e-5))
    do = _f(K, B, L, D).to(dtype)
    dqkv = hip.attn_bwd_packed(do, qkv, o, lse, H, kv, **dr)
    rq, rk, rv = ref.attn_bwd(heads(_d(do)), q, k, v, o2, lse2, kv.cpu(), **rdr)
    _close(dqkv, torch.cat([flat(rq), flat(rk), flat(rv)], -1), tol * 2)
    # the unpacked layout agrees with the packed one
    qc, kc, vc = (heads(t).contiguous() for t in qkv.split(D, dim=-1))
    o3, _ = hip.attn_fwd(qc, kc, vc, kv, **dr)
    _close(flat(o3), o.double(), 1e-6)


@pytest.mark.parametrize("H,planes", [(16, True), (15, True), (8, False)])
def test_dgrad_compact_shortcut_acc(hip, H, planes):
    """Stride-2 dgrad adding a 1x1 stride-2 shortcut's input gradient held only on the stride grid
    (acc_compact: read by the parity class (0, 0) launch alone) == the same dgrad with that
    gradient expanded to full size; and the compact gradient itself == the stride-1 1x1 dgrad
    of the shortcut's dY (its value on the grid), odd sizes included."""
    torch.manual_seed(7)
    K, B, Ci, Co = 2, 3, 64, 128
    W = H
    OH = (H + 2 - 3) // 2 + 1
    w = _f(K, Co, 3, 3, Ci, scale=0.2)
    wsc = _f(K, Co, 1, 1, Ci, scale=0.2)
    dy = _f(K, B, OH, OH, Co)
    dysc = _f(K, B, (H + 1) // 2, (W + 1) // 2, Co)
    kw = {}
    if planes:
        kw = {"w_split": _wsplit(hip, w), "dy_planes": hip.split_planes(dy)}
    comp = hip.conv_dgrad(dysc, wsc, dysc.shape[2:4], 1, 0)
    full = hip.conv_dgrad(dysc, wsc, (H, W), 2, 0)
    assert torch.equal(full[:, :, ::2, ::2], comp)
    assert float(full[:, :, 1::2].abs().max()) == 0.0 and float(full[:, :, :, 1::2].abs().max()) == 0.0
    a = hip.conv_dgrad(dy, w, (H, W), 2, 1, acc=comp, acc_compact=True, **kw)
    b = hip.conv_dgrad(dy, w, (H, W), 2, 1, acc=full, **kw)
    assert torch.equal(a, b)
    _close(a, ref.conv_dgrad(_d(dy), _d(w), (H, W), 2, 1) + _d(full))


@pytest.mark.parametrize("case", [
    # K, B, H (= W), Ci, Co, k, planes, relu, acc: conv_halo (3x3 planes), conv_pl (1x1 planes),
    # conv_f32 (no planes), a 41-sample batch (> FOLD partials: the fp64 fold stage), no ReLU
    (2, 3, 16, 64, 64, 3, True, True, True),
    (3, 2, 8, 256, 64, 1, True, True, False),
    (2, 2, 8, 32, 48, 3, False, True, True),
    (2, 41, 8, 64, 64, 3, True, True, False),
    (2, 3, 8, 64, 128, 1, True, False, True),
    # DenseNet block backward: x a channel prefix of the block buffer (Ci % 8 == 4: no bit mask,
    # the ReLU gate is y > 0; Ci % 8 == 0: bit mask), growth-12 dY, no planes
    (2, 3, 8, 36, 12, 3, False, True, False, 48),
    (2, 2, 8, 48, 12, 3, False, True, False, 36),
])
def test_dgrad_epilogue_bn_bwd_parts(hip, case):
    """Stride-1 fp32 dgrad whose dX is a BatchNorm's dY writes that BN's backward partial sums
    (Σĝ, Σĝ·x̂ per 32 rows, ĝ = dX·relu', valid rows only) in its epilogue: dX is bitwise the same
    as without them, the partial totals match fp64 sums, and bn_bwd(pre_part=) matches bn_bwd's own
    reduction pass (dX, dγ, dβ)."""
    K, B, H, Ci, Co, k, planes, relu, with_acc = case[:9]
    wide = case[9] if len(case) > 9 else 0
    torch.manual_seed(B * 7 + Ci)
    pad = k // 2
    R = B * H * H
    # the BN's input (the producing conv's output), possibly a channel prefix of a wider buffer
    xbuf = _f(K, B, H, H, Ci + wide) * 1.5 + 0.3
    xb = xbuf[..., :Ci]
    x3 = xb.reshape(K, R, Ci)
    g = torch.rand(K, Ci, device=DEV) + 0.5
    b = _f(K, Ci)
    valid = torch.tensor([B, max(1, B - 2), 1][:K], dtype=torch.int32, device=DEV)
    vr = (valid * H * H).to(torch.int32)
    y, mean, rstd, mask = hip.bn_fwd(x3, g, b, vr, relu, None, with_mask=True)
    if not relu:
        mask = None
    ygate = y if (relu and mask is None) else None
    w = _f(K, Co, k, k, Ci, scale=0.2)
    dy = _f(K, B, H, H, Co)
    acc = _f(K, B, H, H, Ci) if with_acc else None
    kw = {"w_split": _wsplit(hip, w), "dy_planes": hip.split_planes(dy)} if planes else {}
    base = hip.conv_dgrad(dy, w, (H, H), 1, pad, acc=acc, **kw)
    part = torch.full((K, hip.conv_stats_parts(R), 2, Ci), float("nan"), device=DEV)
    dx = hip.conv_dgrad(dy, w, (H, H), 1, pad, acc=acc, bnb=(part, x3, mask, mean, rstd, vr, ygate), **kw)
    # (halo tiles past the valid samples skip their work: those rows are never read)
    assert torch.equal(_vimg(dx, valid), _vimg(base, valid))
    dx = torch.where((torch.arange(B, device=DEV).view(1, B) < valid.view(K, 1)).view(K, B, 1, 1, 1), dx, base)
    assert torch.isfinite(part).all()  # every partial slot written
    gd = _d(dx).reshape(K, R, Ci)
    if relu:
        gd = gd * (_d(y) > 0).double()
    xh = (_d(x3) - _d(mean)[:, None]) * _d(rstd)[:, None]
    for kk in range(K):
        rows = int(vr[kk])
        _close(part[kk, :, 0].double().sum(0), gd[kk, :rows].sum(0), 1e-5)
        _close(part[kk, :, 1].double().sum(0), (gd[kk, :rows] * xh[kk, :rows]).sum(0), 1e-5)
    outs = []
    for pre in (None, part):
        gg = torch.zeros(K, Ci, device=DEV)
        gb = torch.zeros(K, Ci, device=DEV)
        # (a strided x — DenseNet's block buffer — adds dX into a buffer of the same strides)
        dxo = torch.zeros(K, B, H, H, Ci + wide, device=DEV)[..., :Ci].reshape(K, R, Ci) if wide else None
        o = hip.bn_bwd(dx.reshape(K, R, Ci), x3, y, mean, rstd, g, vr, relu, gg, gb, True,
                       relu_mask=mask, pre_part=pre, dx_out=dxo)
        outs.append((o[0].contiguous(), o[1], gg, gb))
    for a, c in zip(outs[0], outs[1]):
        _close(c, a.double(), 1e-5)


@pytest.mark.parametrize("D", [100, 512, 300])
def test_embedding_bwd_skewed_tokens_deterministic(hip, D):
    """Deterministic embedding backward on skewed token counts (a padding token holding most rows:
    runs span many 64-row chunks, joined in chunk order): matches the fp64 oracle and is bitwise
    reproducible."""
    torch.manual_seed(D)
    K, B, L, V = 3, 16, 128, 97
    tok = torch.randint(1, V, (K, B, L), device=DEV)
    tok[torch.rand(K, B, L, device=DEV) < 0.7] = 0  # padding-heavy
    tok[1] = 5  # one client: a single token everywhere (one run over every chunk)
    dy = _f(K, B, L, D)
    g1 = torch.full((K, V, D), float("nan"), device=DEV)
    g2 = torch.full((K, V, D), float("nan"), device=DEV)
    hip.embedding_bwd(dy, tok, g1, 0.5)
    hip.embedding_bwd(dy, tok, g2, 0.5)
    assert torch.equal(g1, g2)
    _close(g1, ref.embedding_bwd(_d(dy), tok.cpu(), V, 0.5), 1e-5)


def test_layernorm_planes_feed_plane_linear(hip):
    """LayerNorm writing its output's split planes (hi = bf16(y), lo = bf16(y − hi)) bitwise equal
    to split_planes(y); a linear reading them runs the LDS-DMA plane GEMM within 1e-5 of fp64."""
    torch.manual_seed(3)
    K, B, L, D, Fo = 2, 3, 40, 512, 1536
    x = _f(K, B, L, D) * 2 + 0.5
    g = torch.rand(K, D, device=DEV) + 0.5
    b = _f(K, D)
    y, mean, rstd, yp = hip.ln_fwd(x, g, b, planes=True)
    y0, _, _ = hip.ln_fwd(x, g, b)
    assert torch.equal(y, y0)
    assert torch.equal(yp, hip.split_planes(y))
    w = _f(K, Fo, D, scale=0.05)
    bias = _f(K, Fo)
    ws = _wsplit(hip, w)
    before = hip.planes_launches["linear_fwd"]
    out = hip.linear_fwd(y.reshape(K, B * L, D), w, bias, w_split=ws, x_planes=yp.reshape(K, 2, B * L, D))
    assert hip.planes_launches["linear_fwd"] == before + 1
    _close(out, torch.einsum("knd,kod->kno", _d(y).reshape(K, B * L, D), _d(w)) + _d(bias)[:, None])


@pytest.mark.parametrize("case", [
    # K, B, H, Ci, Co, k, stride, route
    (3, 4, 32, 64, 64, 3, 1, "halo"),      # l1: pixel-group slabs + fold
    (3, 4, 8, 256, 256, 3, 1, "halo"),     # l3: G = 1, the kernel's own epilogue
    (3, 4, 4, 512, 512, 3, 1, "tn"),       # l4: 256x256 TN plane kernel
    (1, 8, 32, 64, 64, 3, 1, "tn"),        # one client, many pixels: split-K slabs + tn_fold
    (3, 4, 8, 256, 512, 1, 2, "tn"),       # 1x1 stride-2 downsample
])
def test_wgrad_sgd_epilogue_matches_flat_step(hip, case):
    """The SGD step applied by the weight-gradient kernels (csrc/sgd_epi.h: direct epilogues and
    split folds) == storing dW and running sgd_step: θ, momentum and the weight planes bit for
    bit, with an inactive client (untouched), a first-step client (m = g) and weight decay."""
    from distributed_learning_simulator_amd.engine.params import FusedSGD

    K, B, H, Ci, Co, k, s, route = case
    torch.manual_seed(11)
    pad = k // 2
    OH = (H + 2 * pad - k) // s + 1
    x = _f(K, B, H, H, Ci)
    dy = _f(K, B, OH, OH, Co)
    xp, dyp = hip.split_planes(x), hip.split_planes(dy)
    n = Co * k * k * Ci
    off, P = 32, 32 + n + 48
    theta = _f(K, P, scale=0.05)
    mom = _f(K, P, scale=0.01)
    split = torch.empty((K, 2, P), dtype=torch.bfloat16, device=DEV)
    hip.split_rows(theta, split)
    lr = torch.tensor([0.1, 0.05, 0.2][:K], device=DEV)
    active = torch.tensor([True, False, True][:K], device=DEV)
    first = torch.tensor([False, False, True][:K], device=DEV)
    wd, mu, damp = 5e-4, 0.9, 0.1
    # reference: dW into the gradient rows, then the flat step
    grad = torch.zeros_like(theta)
    gw = grad[:, off:off + n].unflatten(1, (Co, k, k, Ci))
    if route == "halo":
        assert hip.halo_wgrad(dy, x, gw, dy_planes=dyp, x_planes=xp)
    else:
        hip.conv_wgrad(dy, x, gw, s, pad, dy_planes=dyp, x_planes=xp)
    if K == 1:
        assert hip._C.conv_tn_splitk(K, Co, n // Co, B * OH * OH, Ci, hip._C.conv_tn_pl_variant(), 1, Co, Ci, 1) > 1
    t0, m0, s0 = theta.clone(), mom.clone(), split.clone()
    hip.sgd_step(t0, grad, m0, lr, active, wd, mu, damp, False, first, None, s0)
    # fused: the kernels step θ rows directly (the rest of the row untouched)
    t1, m1, s1 = theta.clone(), mom.clone(), split.clone()
    fused = FusedSGD(t1, m1, s1, lr, active, first, wd, mu, damp, False)
    gw_dummy = torch.full_like(grad, float("nan"))[:, off:off + n].unflatten(1, (Co, k, k, Ci))
    if route == "halo":
        assert hip.halo_wgrad(dy, x, gw_dummy, dy_planes=dyp, x_planes=xp, sgd=(fused, "w", off))
    else:
        assert hip.conv_wgrad(dy, x, gw_dummy, s, pad, dy_planes=dyp, x_planes=xp, sgd=(fused, "w", off))
    assert torch.isnan(gw_dummy).all(), "the fused step must not store dW"
    sl = slice(off, off + n)
    assert torch.equal(t1[:, sl], t0[:, sl]) and torch.equal(m1[:, sl], m0[:, sl])
    assert torch.equal(s1[:, :, sl], s0[:, :, sl])
    if K > 1:
        assert torch.equal(t1[1], theta[1]) and torch.equal(m1[1], mom[1])  # inactive client
    assert torch.equal(t1[:, :off], theta[:, :off]) and torch.equal(t1[:, off + n:], theta[:, off + n:])


def test_linear_epilogue_planes_and_plane_operands(hip):
    """The fp32 NT epilogue writing its output's split planes (forward with ReLU + dropout,
    dgrad with the ReLU' gate): planes bitwise == split_planes(output), fp32 output unchanged;
    dropout_apply(planes=1/2) == split_planes(dropout_apply); the dgrad and the weight gradient
    reading dY / X planes (LDS-DMA plane GEMMs) within 1e-5 of fp64."""
    torch.manual_seed(8)
    K, N, Fi, Fo, p = 2, 150, 512, 1024, 0.1
    x, w, b = _f(K, N, Fi), _f(K, Fo, Fi, scale=0.05), _f(K, Fo)
    ws = _wsplit(hip, w)
    seeds = torch.tensor([11, 12], dtype=torch.int32, device=DEV)
    h0 = hip.linear_fwd(x, w, b, relu=True, drop_p=p, drop_seeds=seeds, w_split=ws)
    h, hp = hip.linear_fwd(x, w, b, relu=True, drop_p=p, drop_seeds=seeds, w_split=ws, out_planes=True)
    assert torch.equal(h, h0) and torch.equal(hp, hip.split_planes(h))
    # the register-split kernels (no weight planes) write no planes in their epilogue: split after
    hr, hrp = hip.linear_fwd(x, w, b, relu=True, out_planes=True)
    assert torch.equal(hrp, hip.split_planes(hr))
    # dropout backward with planes: the fp32 values and the planes of the same masked gradient
    d = _f(K, N, Fo)
    m = hip.dropout_apply(d, seeds, p)
    m1, mp1 = hip.dropout_apply(d, seeds, p, planes=1)
    assert torch.equal(m1, m) and torch.equal(mp1, hip.split_planes(m))
    _, mp2 = hip.dropout_apply(d, seeds, p, planes=2)
    assert torch.equal(mp2, mp1)
    # with the column sums (the consuming linear's bias gradient) into a strided row: same planes
    cs = torch.full((K, Fo + 5), 3.0, device=DEV)
    _, mp3 = hip.dropout_apply(d, seeds, p, planes=2, colsum=cs[:, :Fo])
    assert torch.equal(mp3, mp1) and torch.all(cs[:, Fo:] == 3.0)
    _close(cs[:, :Fo], _d(m).sum(1))
    # dgrad: dY planes in, gated dX planes out
    w2 = _f(K, Fi, Fo, scale=0.05)  # a second linear Fo -> Fi reading h
    ws2 = _wsplit(hip, w2)
    dy = _f(K, N, Fi)
    before = hip.planes_launches["linear_dgrad"]
    dx0 = hip.linear_dgrad(dy, w2, gate=h, gate_scale=1 / (1 - p), w_split=ws2)
    dyp = hip.split_planes(dy)
    dx, dxp = hip.linear_dgrad(dy, w2, gate=h, gate_scale=1 / (1 - p), w_split=ws2, dy_planes=dyp, out_planes=True)
    assert hip.planes_launches["linear_dgrad"] == before + 1
    assert torch.equal(dxp, hip.split_planes(dx))
    exp = ref.linear_dgrad(_d(dy), _d(w2), gate=_d(h), gate_scale=1 / (1 - p))
    _close(dx, exp)
    _close(dx0, exp)
    # weight gradient from planes (dY, X) == fp64; bias from the fp32 dY
    gw, gb = torch.empty(K, Fi, Fo, device=DEV), torch.empty(K, Fi, device=DEV)
    before = hip.planes_launches["wgrad"]
    hip.linear_wgrad(dy, h, gw, gb, dy_planes=dyp, x_planes=hp)
    assert hip.planes_launches["wgrad"] == before + 1
    dw_ref, db_ref = ref.linear_wgrad(_d(dy), _d(h), True)
    _close(gw, dw_ref)
    _close(gb, db_ref)


def test_transformer_layer_planes_flow_matches_fp32(hip):
    """A Transformer classifier (2 encoder layers, dropout on) trained with the split-plane flow
    (LN / linear1 / dropout-backward / linear2-dgrad planes feeding the plane GEMMs) against the
    same step with planes disabled: loss and every parameter gradient within fp32 rounding of
    different summation orders; the plane dgrad and wgrad GEMMs did run."""
    from distributed_learning_simulator_amd import options
    from distributed_learning_simulator_amd.data.datasets import get_spec
    from distributed_learning_simulator_amd.engine.params import BoundParams
    from distributed_learning_simulator_amd.models.layers import RunCtx
    from distributed_learning_simulator_amd.models.zoo import build_model
    from distributed_learning_simulator_amd.ops import functional as Fn

    torch.manual_seed(0)
    spec = get_spec("imdb", {"max_len": 64})
    model = build_model("TransformerClassificationModel", spec,
                        {"d_model": 128, "nhead": 4, "num_encoder_layer": 2, "max_len": 64, "dim_feedforward": 256,
                         "dropout": 0.1})
    K, B, L = 2, 3, 64
    g = torch.Generator().manual_seed(3)
    theta = torch.stack([model.layout.init_flat(g) for _ in range(K)]).to(DEV)
    split = torch.empty((K, 2, theta.shape[1]), dtype=torch.bfloat16, device=DEV)
    hip.split_rows(theta, split)
    tokens = torch.randint(1, 100, (K, B, L), device=DEV)
    lengths = torch.tensor([[64, 40, 17], [64, 64, 3]], device=DEV)
    y = torch.randint(0, spec.num_classes, (K, B), device=DEV)

    def step(planes):
        grad = torch.zeros_like(theta)
        params = BoundParams(model.layout, theta, grad, split=split)
        ctx = RunCtx(params, torch.full((K,), B, dtype=torch.int32, device=DEV), training=True, seed=5)
        with options.override(planes=planes, tfm_planes=True):
            logits = model.forward((tokens, lengths), ctx)
            loss, _ = Fn.cross_entropy(logits, y, ctx.valid)
            loss.sum().backward()
        torch.cuda.synchronize()
        return loss.detach(), grad

    l0, g0 = step(False)
    before = dict(hip.planes_launches)
    l1, g1 = step(True)
    n = {k: hip.planes_launches[k] - before.get(k, 0) for k in ("linear_fwd", "linear_dgrad", "wgrad")}
    # per layer: fwd in_proj (but the first layer's, which reads the embedding) / linear1 / linear2
    # (out_proj reads the attention output: fp32); dgrad out_proj / linear1 / linear2 (in_proj's dY
    # is the attention backward's fp32 dqkv); wgrad linear1 / linear2
    assert n == {"linear_fwd": 5, "linear_dgrad": 6, "wgrad": 4}, n
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-5 * g0.abs().max().item())


@pytest.mark.parametrize("case", [
    # K, B, H (= W), C, N, relu, valid samples of client 0 (None: all): the three halo shapes
    (2, 2, 32, 64, 64, True, None),
    (3, 3, 16, 128, 128, True, 2),
    (2, 4, 8, 256, 256, False, 3),
    (1, 6, 8, 128, 256, True, None),   # two N tiles per row block
])
def test_halo_conv_with_fused_bn_input(hip, case):
    """conv_halo_bn_fwd (csrc/conv_halo.hip BNF: BatchNorm(+ReLU) applied in the halo loader)
    equals the unfused BN apply → split planes → halo conv bit for bit (same coefficients, same
    fma / max / split per element), output and its epilogue statistics alike; rows of invalid
    samples read as zero; and both agree with the fp64 oracle of conv(relu(bn(x)))."""
    K, B, H, C, N, relu, nv = case
    torch.manual_seed(3)
    x = _f(K, B, H, H, C, scale=2.0) + 0.5
    gamma, beta = _f(K, C) * 0.5 + 1.0, _f(K, C) * 0.2
    w = _f(K, N, 3, 3, C, scale=0.05)
    n = N * 9 * C
    wpl = torch.empty((K, 2, n), dtype=torch.bfloat16, device=DEV)
    hip.split_rows(w.reshape(K, n).contiguous(), wpl)
    ws = wpl[:, 0].unflatten(1, (N, 3, 3, C))
    valid = None if nv is None else torch.tensor([nv] + [B] * (K - 1), dtype=torch.int32, device=DEV)
    vrows = None if valid is None else valid * (H * H)
    x3 = x.reshape(K, -1, C)
    # unfused: BN apply writing planes only, then the plane (halo) conv with epilogue statistics
    y, mean, rstd, yp = hip.bn_fwd(x3, gamma, beta, vrows, relu, None, planes=2)
    parts = hip.conv_stats_parts(B * H * H)
    st_a = torch.empty((K, parts, 2, N), device=DEV)
    ref_out = hip.conv_fwd(y.view(K, B, H, H, C), w, 1, 1, w_split=ws, x_planes=yp.view(K, 2, B, H, H, C),
                           stats=st_a, stats_valid=valid)
    # fused
    coef, mean2, rstd2 = hip.bn_coef(x3, gamma, beta, vrows)
    assert torch.equal(mean, mean2) and torch.equal(rstd, rstd2)
    st_b = torch.empty_like(st_a)
    out = hip.conv_halo_bn_fwd(x, coef, relu, vrows, w, ws, stats=st_b, stats_valid=valid)
    assert out is not None
    # (tiles past the valid samples are skipped: compare the valid images)
    assert torch.equal(_vimg(out, valid), _vimg(ref_out, valid))
    assert torch.equal(st_a, st_b)
    # fp64 oracle
    xd = _d(x).view(K, -1, C)
    rows = xd.shape[1]
    keep = torch.ones(K, rows, 1, dtype=torch.float64)
    if vrows is not None:
        keep = (torch.arange(rows).view(1, rows) < vrows.cpu().view(K, 1)).double().unsqueeze(-1)
    cnt = keep.sum(1)
    mu = (xd * keep).sum(1) / cnt
    var = (((xd - mu[:, None]) ** 2) * keep).sum(1) / cnt
    z = (xd - mu[:, None]) / torch.sqrt(var[:, None] + 1e-5) * _d(gamma)[:, None] + _d(beta)[:, None]
    if relu:
        z = z.clamp(min=0)
    z = (z * keep).view(K, B, H, H, C)
    _close(_vimg(out, valid), _vimg(ref.conv_fwd(z, _d(w), 1, 1), valid))


DENSE_HALO_CASES = [
    # K, Kw, B, H, c (prefix), Ct (block buffer), N, valid samples of client 0
    (2, 2, 4, 32, 28, 160, 12, None),   # block 1, c % 8 == 4 (half a lane group real)
    (2, 2, 4, 32, 16, 160, 12, 3),      # first layer, invalid rows
    (3, 1, 4, 16, 172, 304, 12, None),  # block 2, one shared weight (rep = K)
    (2, 2, 4, 8, 436, 448, 12, 2),      # block 3: the last chunk runs to the buffer's end
    (2, 2, 4, 32, 64, 96, 32, None),    # 32 new channels: the full N tile
]


@pytest.mark.parametrize("case", DENSE_HALO_CASES)
def test_dense_growth_conv_with_fused_bn(hip, case):
    """DenseNet growth conv with BN + ReLU over the block buffer's channel prefix applied in the
    halo loader (csrc/conv_halo.hip BNM 2): the prefix is read in place, channels past it are
    never read (they hold NaN here), the normalised activation it writes equals bn_fwd's y bit for
    bit, its output lands in the buffer's new channels only, and the conv matches the unfused
    BN-apply → conv and the fp64 oracle of conv(relu(bn(x)))."""
    K, Kw, B, H, c, Ct, N, nv = case
    torch.manual_seed(5)
    F = _f(K, B, H, H, Ct, scale=2.0) + 0.5
    F[..., c:] = float("nan")
    x = F[..., :c]
    gamma, beta = _f(K, c) * 0.5 + 1.0, _f(K, c) * 0.2
    w = _f(Kw, N, 3, 3, c, scale=0.05)
    valid = None if nv is None else torch.tensor([nv] + [B] * (K - 1), dtype=torch.int32, device=DEV)
    vrows = None if valid is None else valid * (H * H)
    assert hip.halo_bn_dense_ok(x, w)
    x3 = x.reshape(K, -1, c)
    y_ref, mean, rstd, m_ref = hip.bn_fwd(x3, gamma, beta, vrows, True, None, with_mask=True)
    assert (m_ref is not None) == (c % 8 == 0)
    unfused = hip.conv_fwd(y_ref.view(K, B, H, H, c), w, 1, 1)
    coef, mean2, rstd2 = hip.bn_coef(x3, gamma, beta, vrows)
    assert torch.equal(mean, mean2) and torch.equal(rstd, rstd2)
    ny = torch.empty((K, B * H * H, c), device=DEV)
    before = F.clone()
    mask = torch.empty_like(m_ref) if m_ref is not None else None
    assert hip.conv_halo_bn_dense_fwd(x, coef, True, vrows, w, F[..., c : c + N], ny=ny, mask=mask)
    torch.cuda.synchronize()
    assert torch.equal(ny, y_ref), (ny - y_ref).abs().max()
    if mask is not None:
        assert torch.equal(mask, m_ref)
    if N <= 16:  # the recomputing weight gradient stages bitwise this ny from x and coef
        dyw = _f(K, B, H, H, N)
        g1, g2 = torch.empty((K, N, 3, 3, c), device=DEV), torch.empty((K, N, 3, 3, c), device=DEV)
        assert hip.dense_wgrad(dyw, ny, g1)
        assert hip.dense_wgrad(dyw, None, g2, x=x, bn_coef=coef, valid_rows=vrows)
        assert torch.equal(g1, g2)
    out = F[..., c : c + N]
    assert not torch.isnan(out).any()
    rest = torch.cat([F[..., :c], F[..., c + N :]], dim=-1)
    rest_b = torch.cat([before[..., :c], before[..., c + N :]], dim=-1)
    assert torch.equal(rest.nan_to_num(7.0), rest_b.nan_to_num(7.0)), "wrote outside its output channels"
    _close(out, unfused)
    # evaluation form: no activation written, same output
    F2 = before.clone()
    assert hip.conv_halo_bn_dense_fwd(F2[..., :c], coef, True, vrows, w, F2[..., c : c + N])
    assert torch.equal(F2[..., c : c + N], out)
    xd = _d(x3)
    rows = xd.shape[1]
    keep = torch.ones(K, rows, 1, dtype=torch.float64)
    if vrows is not None:
        keep = (torch.arange(rows).view(1, rows) < vrows.cpu().view(K, 1)).double().unsqueeze(-1)
    cnt = keep.sum(1)
    mu = (xd * keep).sum(1) / cnt
    var = (((xd - mu[:, None]) ** 2) * keep).sum(1) / cnt
    z = (xd - mu[:, None]) / torch.sqrt(var[:, None] + 1e-5) * _d(gamma)[:, None] + _d(beta)[:, None]
    z = (z.clamp(min=0) * keep).view(K, B, H, H, c)
    _close(out, ref.conv_fwd(z, _d(w).expand(K, -1, -1, -1, -1), 1, 1))


@pytest.mark.parametrize("K,nparts,g,Ct,c0", [(3, 2048, 12, 64, 28), (2, 7, 12, 40, 0), (2, 513, 16, 96, 80),
                                              (1, 64, 128, 256, 64)])
def test_part_sum_f64(hip, K, nparts, g, Ct, c0):
    """DenseNet running sums: the conv-epilogue partials [K, parts, 2, g] summed in fp64 into a
    channel slice of [K, 2, Ct], other channels untouched."""
    torch.manual_seed(0)
    part = _f(K, nparts, 2, g, scale=3.0)
    S = torch.full((K, 2, Ct), 7.0, dtype=torch.float64, device=DEV)
    hip.part_sum_f64(part, S[:, :, c0 : c0 + g])
    exp = torch.full((K, 2, Ct), 7.0, dtype=torch.float64)
    exp[:, :, c0 : c0 + g] = _d(part).sum(dim=1)
    out = S.cpu()
    assert torch.equal(out[:, :, :c0], exp[:, :, :c0]) and torch.equal(out[:, :, c0 + g :], exp[:, :, c0 + g :])
    assert (out - exp).abs().max().item() <= 1e-12 * exp.abs().max().item()


@pytest.mark.parametrize("K,R,C,ld,valid", [(3, 65536, 24, 168, None), (2, 4096, 312, 312, [4096, 1000]),
                                            (2, 1000, 168, 200, [999, 0]), (1, 300, 8, 8, [257])])
def test_chan_sums_f64(hip, K, R, C, ld, valid):
    """DenseNet block input's running sums: fp64 Σx, Σx² per channel over each client's valid rows,
    read from a channel prefix of a wider buffer."""
    torch.manual_seed(1)
    buf = _f(K, R, ld, scale=2.0)
    x = buf[..., :C]
    vr = torch.tensor(valid, dtype=torch.int32, device=DEV) if valid is not None else None
    S = torch.full((K, 2, C + 5), 3.0, dtype=torch.float64, device=DEV)
    hip.chan_sums_f64(x, vr, S[:, :, :C])
    xd = _d(x)
    if valid is not None:
        keep = torch.arange(R).view(1, R, 1) < torch.tensor(valid).view(K, 1, 1)
        xd = torch.where(keep, xd, torch.zeros((), dtype=xd.dtype))
    exp = torch.stack([xd.sum(dim=1), (xd * xd).sum(dim=1)], dim=1)
    out = S.cpu()
    assert torch.equal(out[:, :, C:], torch.full((K, 2, 5), 3.0, dtype=torch.float64))
    assert (out[:, :, :C] - exp).abs().max().item() <= 1e-12 * exp.abs().max().item()


@pytest.mark.parametrize("case", [(2, 4, 32, 28, 160, 12), (3, 4, 16, 172, 304, 12), (2, 4, 8, 436, 448, 12),
                                  (2, 2, 32, 16, 160, 12), (2, 4, 16, 64, 96, 16)])
def test_dense_wgrad_halo(hip, case):
    """DenseNet growth-conv weight gradient on the LDS-halo kernel (csrc/conv_dense_wgrad.hip:
    16x16x32 MFMA, pixel-major operands read with the transposed LDS read) against the fp64 oracle
    and the implicit-GEMM TN kernel; dY read in place from the block gradient's growth channels,
    the gradient rows' neighbours untouched, and deterministic (two runs bitwise equal)."""
    K, B, H, c, Ct, N = case
    torch.manual_seed(13)
    dG = _f(K, B, H, H, Ct)
    dy = dG[..., c : c + N]
    y = torch.relu(_f(K, B * H * H, c))
    P = N * 9 * c + 24
    gbuf = torch.full((K, P), 7.0, device=DEV)
    gw = gbuf[:, 8 : 8 + N * 9 * c].unflatten(1, (N, 3, 3, c))
    assert hip.dense_wgrad(dy, y, gw)
    torch.cuda.synchronize()
    assert torch.all(gbuf[:, :8] == 7.0) and torch.all(gbuf[:, 8 + N * 9 * c :] == 7.0)
    oracle = ref.conv_wgrad(_d(dy.contiguous()), _d(y).view(K, B, H, H, c), (K, N, 3, 3, c), 1, 1)
    _close(gw, oracle)
    gw2 = torch.empty_like(gw)
    hip.conv_wgrad(dy, y.view(K, B, H, H, c), gw2, 1, 1)
    _close(gw, gw2, 2e-5)
    again = torch.empty_like(gw)
    assert hip.dense_wgrad(dy, y, again)
    assert torch.equal(again, gw)


@pytest.mark.parametrize("case", [(2, 4, 32, 28, 160, 12, "y", False), (3, 4, 16, 172, 304, 12, "y", True),
                                  (2, 4, 8, 436, 448, 12, "y", True), (2, 2, 32, 16, 160, 12, "mask", False),
                                  (2, 4, 16, 64, 96, 16, "mask", False), (4, 2, 8, 100, 112, 12, "y", True),
                                  (2, 4, 16, 136, 160, 12, "mask", True), (2, 4, 32, 28, 160, 12, "coef", False),
                                  (3, 4, 8, 436, 448, 12, "coef", True), (2, 4, 16, 64, 96, 16, "coef", False)])
def test_dense_dgrad_bn_fused(hip, case):
    """DenseNet layer backward on the fused kernel pair (csrc/conv_dense_dgrad.hip: the growth
    conv's input gradient recomputed per tile in a sums pass and an apply pass, never stored)
    against a float64 oracle of conv3x3ᵀ → BN backward (batch statistics, ReLU gate from the bit
    mask, from y > 0 or recomputed from x and the BN scale / shift, ragged valid rows, shared or per-client weights / γ), and against the
    unfused conv_dgrad + bn_bwd; dF's growth channels and the rows past the valid samples are
    untouched, and two runs are bitwise equal."""
    K, B, H, c, Ct, N, gate, shared = case
    torch.manual_seed(29)
    R = B * H * H
    F = _f(K, B, H, H, Ct)
    dF0 = _f(K, B, H, H, Ct)
    Kw = 1 if shared else K
    w = _f(Kw, N, 3, 3, c, scale=0.2)
    gamma = torch.rand(Kw, c, device=DEV) + 0.5
    beta = _f(Kw, c, scale=0.3)
    ggamma = torch.full((K, c + 3), 5.0, device=DEV)[:, :c]  # (γ and β gradient rows share the client stride)
    gbeta = torch.full((K, c + 3), 5.0, device=DEV)[:, :c]
    valid = torch.tensor([B * H * H] + [(B - 1) * H * H] * (K - 1), dtype=torch.int32, device=DEV)
    x = F[..., :c].reshape(K, R, c)
    keep = (torch.arange(R, device=DEV)[None, :] < valid[:, None]).unsqueeze(-1)
    xv = torch.where(keep, x, torch.zeros_like(x))
    mean = (xv.sum(1) / valid[:, None]).contiguous()
    var = ((torch.where(keep, x - mean[:, None], torch.zeros_like(x))) ** 2).sum(1) / valid[:, None]
    rstd = torch.rsqrt(var + 1e-5).contiguous()
    gk = gamma.expand(K, c) if shared else gamma
    bk = beta.expand(K, c) if shared else beta
    sc = (gk * rstd).contiguous()
    sh = (bk - mean * sc).contiguous()
    # (no pre-activation within rounding of 0: every gate form — bits, y, or fmaf(x, scale, shift)
    # recomputed — then agrees with the oracle's)
    with torch.no_grad():
        near = (x * sc[:, None] + sh[:, None]).abs() < 1e-3
        x[near] += 0.01
    y = torch.relu(x * sc[:, None] + sh[:, None]).contiguous()
    bn_sc = torch.stack([sc, sh], -1).contiguous() if gate == "coef" else None
    mask = None
    if gate == "mask":
        bits = (y > 0).view(K, R, c // 8, 8).to(torch.int32)
        mask = (bits << torch.arange(8, device=DEV, dtype=torch.int32)).sum(-1).to(torch.uint8).contiguous()
    # fp64 oracle
    dyh = ref.conv_dgrad(_d(dF0[..., c : c + N].contiguous()), _d(w), (H, H), 1, 1).reshape(K, R, c)
    km = _d(keep.to(torch.float32))
    gg = dyh * (_d(y) > 0) * km
    xh = (_d(x) - _d(mean)[:, None]) * _d(rstd)[:, None] * km
    n = _d(valid.float())[:, None, None]
    s0, s1 = gg.sum(1), (gg * xh).sum(1)
    dx = _d(gk)[:, None] * _d(rstd)[:, None] * (gg - s0[:, None] / n - xh * s1[:, None] / n) * km
    exp = _d(dF0).clone()
    exp[..., :c] += dx.view(K, B, H, H, c)
    dF = dF0.clone()
    assert hip.dense_dgrad_bn(dF[..., c : c + N], w, F[..., :c], dF[..., :c], y, mask, mean, rstd, gamma, valid,
                              ggamma, gbeta, bn_coef=bn_sc)
    torch.cuda.synchronize()
    _close(dF[..., :c], exp[..., :c])
    assert torch.equal(dF[..., c:], dF0[..., c:])
    rows_past = ~keep.view(K, B, H, H)
    assert torch.equal(dF[..., :c][rows_past], dF0[..., :c][rows_past])
    _close(gbeta, s0)
    _close(ggamma, s1)
    # the unfused path
    dF2 = dF0.clone()
    dyu = hip.conv_dgrad(dF2[..., c : c + N], w, (H, H), 1, 1)
    g2, b2 = torch.empty(K, c, device=DEV), torch.empty(K, c, device=DEV)
    hip.bn_bwd(dyu.view(K, R, c), x, y, mean, rstd, gamma, valid, True, g2, b2, False, relu_mask=mask,
               dx_out=dF2[..., :c].reshape(K, R, c))
    _close(dF[..., :c], dF2[..., :c].double(), 2e-5)
    again = dF0.clone()
    assert hip.dense_dgrad_bn(again[..., c : c + N], w, F[..., :c], again[..., :c], y, mask, mean, rstd, gamma, valid,
                              ggamma, gbeta, bn_coef=bn_sc)
    assert torch.equal(again, dF)


def test_densenet40_eval_fused_bn_halo(hip):
    """DenseNet-40 batched evaluation with the growth convs' BN fused into the halo loader agrees
    with the unfused evaluation (the conv's K order differs — taps padded to 32-channel chunks —
    so equal to rounding, not bitwise), and the fused kernels ran."""
    from distributed_learning_simulator_amd import options
    from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
    from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
    from distributed_learning_simulator_amd.models.zoo import build_model

    dev = torch.device(DEV)
    dc = create_dataset_collection("CIFAR10", {"n_train": 256, "n_test": 300}, 0, dev, torch.float32, image_channels=8)
    model = build_model("densenet40", dc.spec)
    tr = CohortTrainer(model, dc, HyperParameter(epoch=1, batch_size=64), dev, torch.float32, capacity=1)
    g = torch.Generator().manual_seed(0)
    rows = torch.stack([model.layout.init_flat(g) for _ in range(2)]).to(dev)
    hip.planes_launches.clear()
    with options.override(dense_bn_halo=True):
        lf, cf, n = tr.evaluate(rows, max_images=512)
    assert hip.planes_launches["fwd_bn_dense"] > 0, hip.planes_launches
    with options.override(dense_bn_halo=False):
        lu, cu, _ = tr.evaluate(rows, max_images=512)
    with options.override(dense_bn_halo=True, dense_stats_cache=True):
        lc, cc, _ = tr.evaluate(rows, max_images=512)
    for lo, co in ((lf, cf), (lc, cc)):
        assert (co - cu).abs().max().item() <= 2
        assert (lo - lu).abs().max().item() <= 1e-5 * lu.abs().max().item(), (lo - lu).abs().max()


def test_resnet18_eval_fused_bn_equals_unfused(hip):
    """The batched utility evaluation (GTG-Shapley's cost) with bn1 fused into conv2's halo loader
    gives bitwise the same losses and correct counts as the unfused evaluation, and the fused
    kernels actually ran."""
    from distributed_learning_simulator_amd import options
    from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
    from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
    from distributed_learning_simulator_amd.models.zoo import build_model

    dev = torch.device(DEV)
    dc = create_dataset_collection("CIFAR10", {"n_train": 256, "n_test": 700}, 0, dev, torch.float32, image_channels=8)
    model = build_model("ResNet18", dc.spec)
    tr = CohortTrainer(model, dc, HyperParameter(epoch=1, batch_size=64), dev, torch.float32, capacity=1)
    g = torch.Generator().manual_seed(0)
    rows = torch.stack([model.layout.init_flat(g) for _ in range(3)]).to(dev)
    hip.planes_launches.clear()
    with options.override(bn_fused_halo=True):
        lf, cf, n = tr.evaluate(rows, max_images=1024)
    assert hip.planes_launches["fwd_bn_fused"] > 0, hip.planes_launches
    with options.override(bn_fused_halo=False):
        lu, cu, _ = tr.evaluate(rows, max_images=1024)
    assert torch.equal(cf, cu)
    assert torch.equal(lf, lu), (lf - lu).abs().max()


HALO_WGRAD_CASES = [(2, 3, 32, 64, 64), (2, 2, 16, 128, 128), (3, 4, 8, 256, 256), (2, 2, 16, 64, 128),
                    (2, 4, 8, 128, 64), (2, 2, 32, 128, 64)]


@pytest.mark.parametrize("case", HALO_WGRAD_CASES)
def test_halo_wgrad(hip, case):
    """ResNet 3x3 / stride-1 weight gradient on the LDS-halo kernel (csrc/conv_halo_wgrad.hip) against
    the fp64 oracle: fp32 operands split in the loader, pre-split planes (bitwise the same),
    deterministic, the unrolled k-loop bitwise the same, and the gradient rows' neighbours untouched."""
    from distributed_learning_simulator_amd import options

    K, B, H, C, N = case
    torch.manual_seed(17)
    dy = _f(K, B, H, H, N)
    x = _f(K, B, H, H, C)
    P = N * 9 * C + 24
    gbuf = torch.full((K, P), 7.0, device=DEV)
    gw = gbuf[:, 8 : 8 + N * 9 * C].unflatten(1, (N, 3, 3, C))
    assert hip.halo_wgrad(dy, x, gw)
    torch.cuda.synchronize()
    assert torch.all(gbuf[:, :8] == 7.0) and torch.all(gbuf[:, 8 + N * 9 * C :] == 7.0)
    oracle = ref.conv_wgrad(_d(dy), _d(x), (K, N, 3, 3, C), 1, 1)
    _close(gw, oracle)
    again = torch.empty_like(gw)
    assert hip.halo_wgrad(dy, x, again)
    assert torch.equal(again, gw)
    pl = torch.empty_like(gw)
    assert hip.halo_wgrad(dy, x, pl, dy_planes=hip.split_planes(dy), x_planes=hip.split_planes(x))
    assert torch.equal(pl, gw), "planes and in-loader split must give the same operand bits"
    with options.override(native={"halo_wgrad_unroll": 2}):  # (same order of operations: bitwise)
        other = torch.empty_like(gw)
        assert hip.halo_wgrad(dy, x, other)
        assert torch.equal(other, gw)


@pytest.mark.parametrize("case", [(2, 3, 32, 64, 64), (2, 2, 16, 128, 128), (2, 4, 8, 256, 256)])
@pytest.mark.parametrize("relu", [True, False])
def test_halo_wgrad_bn_loader(hip, case, relu):
    """The weight gradient of conv(relu?(BN(x))) with the BatchNorm applied in the halo wgrad's loader
    from the RAW x (no normalised tensor in memory): bitwise equal to the planes bn_apply writes
    (same operand bits), rows past a client's valid samples read as zero, and within 1e-5 of fp64."""
    K, B, H, C, N = case
    torch.manual_seed(19)
    xr = _f(K, B, H, H, C) * 2.0 + 0.5
    dy = _f(K, B, H, H, N)
    gamma = torch.rand(K, C, device=DEV) + 0.5
    beta = torch.randn(K, C, device=DEV) * 0.3
    valid = torch.tensor([B - 1] + [B] * (K - 1), dtype=torch.int32, device=DEV)
    R = B * H * H
    vr = valid * (H * H)
    coef, _, _ = hip.bn_coef(xr.view(K, R, C), gamma, beta, vr)
    gw = torch.empty((K, N, 3, 3, C), device=DEV)
    yp = torch.empty((K, 2, R, C), dtype=torch.bfloat16, device=DEV)
    hip.bn_apply_only(xr.view(K, R, C), coef, vr, relu, yp)
    xa = torch.empty((K, R, C), device=DEV)  # (shape carrier of the planes)
    pl = torch.empty_like(gw)
    assert hip.halo_wgrad(dy, xr, gw, bn=(coef, relu, vr))
    assert hip.halo_wgrad(dy, xa.view(K, B, H, H, C), pl, x_planes=yp.view(K, 2, B, H, H, C))
    assert torch.equal(pl, gw)
    a = _d(xr) * _d(coef[..., 0]).view(K, 1, 1, 1, C) + _d(coef[..., 1]).view(K, 1, 1, 1, C)
    if relu:
        a = a.clamp_min(0)
    a[0, B - 1] = 0  # client 0's last sample is past its valid rows
    _close(gw, ref.conv_wgrad(_d(dy), a, (K, N, 3, 3, C), 1, 1))
    # skipping the images past the valid samples (whose dY the BN backward zeroes): same result
    dyz = dy.clone()
    dyz[0, B - 1] = 0
    full = torch.empty_like(gw)
    assert hip.halo_wgrad(dyz, xr, full, bn=(coef, relu, vr))
    skip = torch.empty_like(gw)
    assert hip.halo_wgrad(dyz, xr, skip, bn=(coef, relu, vr), valid=valid)
    _close(skip, ref.conv_wgrad(_d(dyz), a, (K, N, 3, 3, C), 1, 1))
    _close(skip, full, 2e-6)


@pytest.mark.parametrize("case", [(2, 2, 32, 64, 64), (2, 2, 16, 128, 128), (2, 4, 8, 256, 256), (2, 2, 4, 512, 512),
                                  (2, 2, 16, 64, 128)])
def test_dgrad_transposed_weight_planes(hip, case):
    """3x3 stride-1 plane dgrad on the forward tiles with transposed, flipped weight planes (conv_dgrad
    wt=True) against the fp64 oracle and the k-major path, with the residual + BN-partial epilogue,
    and deterministic."""
    K, B, H, C, Co = case
    torch.manual_seed(23)
    dy = _f(K, B, H, H, Co)
    w = _f(K, Co, 3, 3, C, scale=0.1)
    n = Co * 9 * C
    wpl = torch.empty((K, 2, n), dtype=torch.bfloat16, device=DEV)
    hip.split_rows(w.reshape(K, n).contiguous(), wpl)
    ws = wpl[:, 0].unflatten(1, (Co, 3, 3, C))
    dyp = hip.split_planes(dy)
    acc = _f(K, B, H, H, C)
    out = hip.conv_dgrad(dy, w, (H, H), 1, 1, w_split=ws, dy_planes=dyp, acc=acc, wt=True)
    assert hip.planes_launches["dgrad_wt"] > 0
    exp = ref.conv_dgrad(_d(dy), _d(w), (H, H), 1, 1) + _d(acc)
    _close(out, exp)
    km = hip.conv_dgrad(dy, w, (H, H), 1, 1, w_split=ws, dy_planes=dyp, acc=acc, wt=False)
    _close(out, km, 2e-5)
    again = hip.conv_dgrad(dy, w, (H, H), 1, 1, w_split=ws, dy_planes=dyp, acc=acc, wt=True)
    assert torch.equal(again, out)


@pytest.mark.parametrize("case", [(2, 2, 32, 64, 64), (2, 2, 16, 128, 128), (2, 2, 4, 512, 512)])
def test_dgrad_acc_mask(hip, case):
    """The identity shortcut's gradient as factors: acc gated by ReLU bits in the dgrad epilogue
    (acc_mask) is bitwise the dgrad with the pre-gated acc, on the halo and implicit-GEMM tiles."""
    from distributed_learning_simulator_amd.ops.functional import MaskedGrad

    K, B, H, C, Co = case
    torch.manual_seed(29)
    dy = _f(K, B, H, H, Co)
    w = _f(K, Co, 3, 3, C, scale=0.1)
    n = Co * 9 * C
    wpl = torch.empty((K, 2, n), dtype=torch.bfloat16, device=DEV)
    hip.split_rows(w.reshape(K, n).contiguous(), wpl)
    ws = wpl[:, 0].unflatten(1, (Co, 3, 3, C))
    dyp = hip.split_planes(dy)
    g = _f(K, B, H, H, C)
    mask = torch.randint(0, 256, (K, B * H * H, C // 8), dtype=torch.uint8, device=DEV)
    dense = MaskedGrad(g, mask).dense()
    bits = ((mask.view(K, -1, C // 8, 1) >> torch.arange(8, device=DEV, dtype=torch.uint8)) & 1).reshape(g.shape)
    assert torch.equal(dense, torch.where(bits.bool(), g, torch.zeros_like(g)))
    for wt in (False, True):
        a = hip.conv_dgrad(dy, w, (H, H), 1, 1, w_split=ws, dy_planes=dyp, acc=g, acc_mask=mask, wt=wt)
        b = hip.conv_dgrad(dy, w, (H, H), 1, 1, w_split=ws, dy_planes=dyp, acc=dense, wt=wt)
        assert torch.equal(a, b), wt


@pytest.mark.parametrize("case", [(2, 3, 32, 64, 64), (2, 2, 16, 128, 128), (3, 2, 8, 256, 256), (2, 2, 16, 64, 128)])
@pytest.mark.parametrize("xmode", ["planes", "bn"])
@pytest.mark.parametrize("gate", [True, False])
def test_halo_wgrad_bn_bwd_loader(hip, case, xmode, gate):
    """The halo weight gradient with the BatchNorm BACKWARD applied in its dY loader (dy mode 2,
    ops.functional DeferredBNBwd): from the BN's output gradient, raw input, ReLU bits and the
    coefficients bn_bwd(coef_out=) computed, it builds dX = a·(dy·relu') + e·x + d exactly as
    bn_bwd_apply does — the dX planes it stores for the dgrad are bitwise the BN backward's own
    (zeros past a client's valid rows, also in the images it skips), the weight gradient is bitwise
    the one from those planes and within 1e-5 of fp64; the standalone apply stage
    (bn_bwd_apply_planes) writes the same bits."""
    K, B, H, C, N = case
    torch.manual_seed(31)
    R = B * H * H
    dyo = _f(K, R, N)  # the BN output's gradient
    xb = _f(K, R, N) * 1.5 + 0.25  # the BN's raw input (the conv output)
    mean = xb.mean(dim=1).contiguous()
    rstd = (1.0 / (xb.var(dim=1) + 1e-5).sqrt()).contiguous()
    gamma = torch.rand(K, N, device=DEV) + 0.5
    mask = torch.randint(0, 256, (K, R, N // 8), dtype=torch.uint8, device=DEV) if gate else None
    valid = torch.tensor([B - 1] + [B] * (K - 1), dtype=torch.int32, device=DEV)
    vr = (valid * (H * H)).contiguous()
    # the BN backward's own passes: fp32 dX + its planes, dγ / dβ
    g1, b1 = torch.empty(K, N, device=DEV), torch.empty(K, N, device=DEV)
    dx, _, dxp_ref = hip.bn_bwd(dyo, xb, None, mean, rstd, gamma, vr, gate, g1, b1, False, relu_mask=mask,
                                dx_planes=1)
    # coefficients only, then the loader
    coef = torch.empty((K, N, 3), device=DEV)
    g2, b2 = torch.empty(K, N, device=DEV), torch.empty(K, N, device=DEV)
    assert hip.bn_bwd(dyo, xb, None, mean, rstd, gamma, vr, gate, g2, b2, False, relu_mask=mask, coef_out=coef) is None
    assert torch.equal(g1, g2) and torch.equal(b1, b2)
    x = _f(K, B, H, H, C)
    xkw, xo = {}, x
    if xmode == "planes":
        xkw["x_planes"] = hip.split_planes(x)
    else:  # (the conv's input is itself a BN(+ReLU) applied in the x loader: x mode 2)
        xr = x * 2.0 + 0.5
        xcoef, _, _ = hip.bn_coef(xr.view(K, R, C), torch.rand(K, C, device=DEV) + 0.5,
                                  torch.randn(K, C, device=DEV) * 0.3, vr)
        xkw["bn"] = (xcoef, True, vr)
        xo = xr
        yp = torch.empty((K, 2, R, C), dtype=torch.bfloat16, device=DEV)
        hip.bn_apply_only(xr.view(K, R, C), xcoef, vr, True, yp)
        x = torch.empty((K, B, H, H, C), device=DEV)  # (shape carrier)
        xplanes = yp.view(K, 2, B, H, H, C)
    dxo = torch.empty((K, B, H, H, N), device=DEV)  # (shape carrier: the planes-only alias)
    for skip in (None, valid):
        dxp = torch.full((K, 2, R, N), 12345.0, dtype=torch.bfloat16, device=DEV)
        gw = torch.empty((K, N, 3, 3, C), device=DEV)
        assert hip.halo_wgrad(dxo, xo, gw, valid=skip, bn_bwd=(dyo, xb, mask, coef, vr, dxp), **xkw)
        assert torch.equal(dxp, dxp_ref), "the loader's dX planes must be bn_bwd_apply's bits"
        base = torch.empty_like(gw)
        pl = {"x_planes": xplanes} if xmode == "bn" else {"x_planes": xkw["x_planes"]}
        assert hip.halo_wgrad(dx.view(K, B, H, H, N), x, base, dy_planes=dxp_ref.view(K, 2, B, H, H, N), valid=skip,
                              **pl)
        assert torch.equal(gw, base), "same operand bits as the planes path"
    xd = _d(x) if xmode == "planes" else None
    if xd is None:
        xd = (_d(xo) * _d(xcoef[..., 0]).view(K, 1, 1, 1, C) + _d(xcoef[..., 1]).view(K, 1, 1, 1, C)).clamp_min(0)
        xd[0, B - 1] = 0
    _close(gw, ref.conv_wgrad(_d(dx).view(K, B, H, H, N), xd, (K, N, 3, 3, C), 1, 1))
    alone = torch.full((K, 2, R, N), 7.0, dtype=torch.bfloat16, device=DEV)
    hip.bn_bwd_apply_planes(dyo, xb, mask, coef, vr, alone)
    assert torch.equal(alone, dxp_ref)


@pytest.mark.parametrize("case", [
    # K, B, H (= W), Ci, Co, stride: ResNet-18 l4 (4x4), a batch that is no multiple of 32 (groups
    # straddle pixels), the strided l4a forward (8x8 -> 4x4) and a 7x7 image
    (2, 64, 4, 128, 128, 1),
    (2, 40, 4, 256, 512, 1),
    (2, 33, 8, 128, 128, 2),
    (2, 8, 7, 64, 128, 1),
])
def test_conv_pixel_major_tap_skip(hip, case):
    """Pixel-major GEMM rows with tap skipping on small images (csrc/conv_pl.hip PIX, native option
    conv_pix): forward (with BN statistics over the valid samples) and dgrad (with a residual
    gradient and BN-backward partials) are bitwise the plain walk's — a skipped tap only ever added
    zeros — on the 128x128 and 256x256 tiles; the weight gradient's pixel walk (other summation
    order) is within 1e-5 of the fp64 oracle and reproducible."""
    K, B, H, Ci, Co, s = case
    torch.manual_seed(B + H)
    x = _f(K, B, H, H, Ci)
    w = _f(K, Co, 3, 3, Ci, scale=0.2)
    ws = _wsplit(hip, w)
    xp = hip.split_planes(x)
    OH = (H + 2 - 3) // s + 1
    M = B * OH * OH
    valid = torch.tensor([B, max(1, B - 5)], dtype=torch.int32, device=DEV)
    dy = _f(K, B, OH, OH, Co)
    dyp = hip.split_planes(dy)
    acc = _f(K, B, H, H, Ci)
    # BN-backward partials of the BN whose dY the stride-1 dgrad is (x its input)
    x3 = x.reshape(K, B * H * H, Ci)
    vr = (valid * H * H).to(torch.int32)
    _, mean, rstd, mask = hip.bn_fwd(x3, torch.ones(K, Ci, device=DEV), torch.zeros(K, Ci, device=DEV), vr, True,
                                     None, with_mask=True)
    y_exp = ref.conv_fwd(_d(x), _d(w), s, 1)
    dx_exp = ref.conv_dgrad(_d(dy), _d(w), (H, H), s, 1) + _d(acc)
    gw_exp = ref.conv_wgrad(_d(dy), _d(x), (K, Co, 3, 3, Ci), s, 1)
    outs = {}
    try:
        for pix in (0, 1):
            hip._C.set_native_option("conv_pix", pix)
            for v in (1, 3):
                hip._C.conv_nt_pl_set_variant(v)
                st = torch.full((K, hip.conv_stats_parts(M), 2, Co), float("nan"), device=DEV)
                y = hip.conv_fwd(x, w, s, 1, w_split=ws, x_planes=xp, stats=st, stats_valid=valid)
                assert torch.isfinite(st).all()
                r = {"y": y, "st": st}
                if s == 1:
                    part = torch.full((K, hip.conv_stats_parts(B * H * H), 2, Ci), float("nan"), device=DEV)
                    r["dx"] = hip.conv_dgrad(dy, w, (H, H), 1, 1, acc=acc, w_split=ws, dy_planes=dyp,
                                             bnb=(part, x3, mask, mean, rstd, vr, None))
                    assert torch.isfinite(part).all()
                    r["part"] = part
                outs[(pix, v)] = r
            for tv in (0, 6):
                hip._C.conv_tn_pl_set_variant(tv)
                ga = torch.full((K, Co, 3, 3, Ci), 5.0, device=DEV)
                hip.conv_wgrad(dy, x, ga, s, 1, dy_planes=dyp, x_planes=xp)
                _close(ga, gw_exp)
                gb = torch.full_like(ga, -5.0)
                hip.conv_wgrad(dy, x, gb, s, 1, dy_planes=dyp, x_planes=xp)
                assert torch.equal(ga, gb), f"pix {pix} tn variant {tv} not reproducible"
    finally:
        hip._C.set_native_option("conv_pix", 1)
        hip._C.conv_nt_pl_set_variant(-1)
        hip._C.conv_tn_pl_set_variant(-1)
    y3 = y_exp.reshape(K, M, Co)
    xh = (_d(x3) - _d(mean)[:, None]) * _d(rstd)[:, None]
    gd = dx_exp.reshape(K, B * H * H, Ci) * (xh > 0).double()
    for (pix, v), r in outs.items():
        base = outs[(0, v)]
        assert torch.equal(r["y"], base["y"]), f"pix {pix} variant {v} fwd differs"
        _close(r["y"], y_exp)
        for kk in range(K):
            rows = int(valid[kk]) * OH * OH
            _close(r["st"][kk, :, 0].double().sum(0), y3[kk, :rows].sum(0))
            _close(r["st"][kk, :, 1].double().sum(0), (y3[kk, :rows] ** 2).sum(0))
        if s == 1:
            assert torch.equal(r["dx"], base["dx"]), f"pix {pix} variant {v} dgrad differs"
            _close(r["dx"], dx_exp)
            for kk in range(K):
                rows = int(vr[kk])
                _close(r["part"][kk, :, 0].double().sum(0), gd[kk, :rows].sum(0))
                _close(r["part"][kk, :, 1].double().sum(0), (gd[kk, :rows] * xh[kk, :rows]).sum(0))


@pytest.mark.parametrize("relu,valid", [(True, True), (False, False)])
def test_bn_fwd_folded_residual_bn(hip, relu, valid):
    """bn_fwd with `res_coef`: the residual is a second BN's raw input whose apply is folded in
    (ResNet downsample, ops.functional DeferredRes) — bitwise the apply-first result (y, ReLU bits,
    planes), and bn_apply_only(y=) materialises that second BN's output with bn_fwd's bits."""
    torch.manual_seed(3)
    K, R, C = 3, 517, 64
    x = _f(K, R, C) * 2 + 0.5
    xd = _f(K, R, C) * 3 - 0.2
    g, b = torch.rand(K, C, device=DEV) + 0.5, _f(K, C)
    gd, bd = torch.rand(K, C, device=DEV) + 0.5, _f(K, C)
    vr = torch.tensor([R, R - 100, 7], dtype=torch.int32, device=DEV) if valid else None
    yd, _, _ = hip.bn_fwd(xd, gd, bd, vr, False, None)
    coef, _, _ = hip.bn_coef(xd, gd, bd, vr)
    ym = torch.full_like(yd, float("nan"))
    hip.bn_apply_only(xd, coef, vr, False, None, y=ym)
    assert torch.equal(ym, yd)
    ref_out = hip.bn_fwd(x, g, b, vr, relu, yd, with_mask=True, planes=1)
    out = hip.bn_fwd(x, g, b, vr, relu, xd, with_mask=True, planes=1, res_coef=coef)
    for u, v in zip(out, ref_out):
        if u is not None or v is not None:
            assert torch.equal(u, v)
