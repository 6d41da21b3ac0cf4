"""Plain-PyTorch reference implementations of every client-batched primitive.

These are the numerics oracles for the HIP kernels (tests compare `ops.hip.*` against
`ops.ref.*` computed in fp32) and the CPU execution path used by the CPU test-suite.
Shapes follow the cohort layout used everywhere in this framework:

  images  x  [K, B, H, W, C]      (K = clients resident on the rank, NHWC per client)
  conv w     [K, Co, kh, kw, Ci]
  linear x   [K, N, Fi], w [K, Fo, Fi], b [K, Fo]
  bn x       [K, R, C]  (R = B*H*W rows, per-client batch statistics)

The reference never fuses anything (eager PyTorch inside cyy_torch_toolbox); the inventory
of implicit compute sites these replace is SURVEY §2.5 (K1-K23).
"""

from __future__ import annotations

import torch
import torch.nn.functional as F


def _match(w, K: int):
    """Weights are [M, ...] for K = M*rep virtual clients (rep clients share one weight
    row: evaluation of one model over many test batches, GTG subset models, ...)."""
    if w is None or w.shape[0] == K:
        return w
    assert K % w.shape[0] == 0, (K, w.shape)
    return w.repeat_interleave(K // w.shape[0], dim=0)


# ----------------------------------------------------------------------------- conv
def _to_grouped(x: torch.Tensor) -> torch.Tensor:
    K, B, H, W, C = x.shape
    return x.permute(1, 0, 4, 2, 3).reshape(B, K * C, H, W)


def _from_grouped(y: torch.Tensor, K: int) -> torch.Tensor:
    B, KC, H, W = y.shape
    return y.reshape(B, K, KC // K, H, W).permute(1, 0, 3, 4, 2)


def _w_grouped(w: torch.Tensor) -> torch.Tensor:
    K, Co, kh, kw, Ci = w.shape
    return w.permute(0, 1, 4, 2, 3).reshape(K * Co, Ci, kh, kw)


def conv_fwd(x, w, stride: int, pad: int, bias=None):
    K = x.shape[0]
    w = _match(w, K)
    b = _match(bias, K).reshape(-1).to(x.dtype) if bias is not None else None
    y = F.conv2d(_to_grouped(x), _w_grouped(w).to(x.dtype), b, stride=stride, padding=pad, groups=K)
    return _from_grouped(y, K).contiguous()


def conv_dgrad(dy, w, in_hw, stride: int, pad: int, acc=None):
    K, B = dy.shape[:2]
    w = _match(w, K)
    Ci = w.shape[-1]
    dx = torch.nn.grad.conv2d_input(
        (B, K * Ci, in_hw[0], in_hw[1]), _w_grouped(w), _to_grouped(dy),
        stride=stride, padding=pad, groups=K,
    )
    dx = _from_grouped(dx, K).contiguous()
    return dx if acc is None else dx + acc.to(dx.dtype)


def conv_wgrad(dy, x, w_shape, stride: int, pad: int):
    K = x.shape[0]
    _, Co, kh, kw, Ci = w_shape
    dw = torch.nn.grad.conv2d_weight(
        _to_grouped(x), (K * Co, Ci, kh, kw), _to_grouped(dy),
        stride=stride, padding=pad, groups=K,
    )
    return dw.reshape(K, Co, Ci, kh, kw).permute(0, 1, 3, 4, 2)


# ---------------------------------------------------------------------------- linear
def dropout_keep(K: int, rows: int, N: int, seeds, p: float) -> torch.Tensor:
    """[K, rows, N] keep mask of the GEMM-epilogue dropout (common.h drop_keep):
    mix32(m·N + n, seed_k) >= p·2^32."""
    import numpy as np

    from .fl import _mix

    thr = int(min(float(np.float32(p) * np.float32(4294967296.0)), 4294967040.0))
    idx = torch.arange(rows * N, dtype=torch.int64, device=seeds.device).view(1, rows * N)
    sk = (seeds.long() & 0xFFFFFFFF).view(K, 1)
    return (_mix(idx, sk) >= thr).view(K, rows, N)


def dropout_apply(x, seeds, p: float):
    K, N = x.shape[0], x.shape[-1]
    keep = dropout_keep(K, x.numel() // (K * N), N, seeds.to(x.device), p).view(x.shape)
    return torch.where(keep, x * (1.0 / (1.0 - p)), torch.zeros_like(x))


def linear_fwd(x, w, b=None, relu=False, acc=None, drop_p: float = 0.0, drop_seeds=None):
    K = x.shape[0]
    w = _match(w, K)
    y = torch.bmm(x, w.transpose(1, 2))
    if b is not None:
        b = _match(b, K)
        y = y + b[:, None, :]
    if relu:
        y = torch.relu(y)
    if drop_p:
        y = dropout_apply(y, drop_seeds, drop_p)
    if acc is not None:
        y = y.to(acc.dtype) + acc
    return y


def linear_dgrad(dy, w, gate=None, gate_scale: float = 1.0):
    K = dy.shape[0]
    w = _match(w, K)
    dx = torch.bmm(dy, w)
    if gate_scale != 1.0:
        dx = dx * gate_scale
    return dx if gate is None else dx * (gate > 0).to(dx.dtype)


def linear_wgrad(dy, x, with_bias: bool):
    dw = torch.bmm(dy.transpose(1, 2), x)
    db = dy.sum(dim=1) if with_bias else None
    return dw, db


# ------------------------------------------------------------------------ batch norm
def _row_mask(R: int, valid_rows, device):
    if valid_rows is None:
        return None
    ar = torch.arange(R, device=device)
    return (ar[None, :] < valid_rows[:, None].to(device)).unsqueeze(-1)  # [K,R,1]


def bn_fwd(x, gamma, beta, valid_rows=None, relu=False, residual=None, eps=1e-5):
    """Training-mode BN with batch statistics over valid rows (reference disables running
    stats: `util/model.py:23`, `server.py:48`), + optional residual add and ReLU."""
    K, R, C = x.shape
    xf = x.float()
    m = _row_mask(R, valid_rows, x.device)
    if m is None:
        n = torch.full((K, 1), float(R), device=x.device)
        mean = xf.mean(dim=1)
        var = ((xf - mean[:, None]) ** 2).mean(dim=1)
    else:
        n = valid_rows.to(x.device).float().clamp(min=1).unsqueeze(1)
        mean = (xf * m).sum(dim=1) / n
        var = (((xf - mean[:, None]) ** 2) * m).sum(dim=1) / n
    rstd = torch.rsqrt(var + eps)
    gamma, beta = _match(gamma, K), _match(beta, K)
    y = (xf - mean[:, None]) * rstd[:, None] * gamma.float()[:, None] + beta.float()[:, None]
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    if m is not None:
        y = y * m
    return y.to(x.dtype), mean, rstd


def bn_bwd(dy, x, y, mean, rstd, gamma, valid_rows=None, relu=False):
    """Returns (dx, dgamma, dbeta, dpre) where dpre = dL/d(bn_out + residual)."""
    K, R, C = x.shape
    m = _row_mask(R, valid_rows, x.device)
    g = dy.float()
    if relu:
        g = g * (y.float() > 0)
    if m is not None:
        g = g * m
        n = valid_rows.to(x.device).float().clamp(min=1).unsqueeze(1)
    else:
        n = torch.full((K, 1), float(R), device=x.device)
    xhat = (x.float() - mean[:, None]) * rstd[:, None]
    if m is not None:
        xhat = xhat * m
    dbeta = g.sum(dim=1)
    dgamma = (g * xhat).sum(dim=1)
    gamma = _match(gamma, K)
    dx = gamma.float()[:, None] * rstd[:, None] * (
        g - dbeta[:, None] / n[:, None] - xhat * dgamma[:, None] / n[:, None]
    )
    if m is not None:
        dx = dx * m
    return dx.to(x.dtype), dgamma, dbeta, g.to(x.dtype)


# ------------------------------------------------------------------------ layer norm
def ln_fwd(x, gamma, beta, eps=1e-5):
    K = x.shape[0]
    xf = x.float()
    mean = xf.mean(dim=-1)
    var = ((xf - mean[..., None]) ** 2).mean(dim=-1)
    rstd = torch.rsqrt(var + eps)
    gamma, beta = _match(gamma, K), _match(beta, K)
    shape = (K,) + (1,) * (x.dim() - 2) + (x.shape[-1],)
    y = (xf - mean[..., None]) * rstd[..., None] * gamma.float().reshape(shape) + beta.float().reshape(shape)
    return y.to(x.dtype), mean, rstd


def ln_bwd(dy, x, mean, rstd, gamma):
    K = x.shape[0]
    C = x.shape[-1]
    gamma = _match(gamma, K)
    shape = (K,) + (1,) * (x.dim() - 2) + (C,)
    g = dy.float()
    xhat = (x.float() - mean[..., None]) * rstd[..., None]
    red = tuple(range(1, x.dim() - 1))
    dgamma = (g * xhat).sum(dim=red)
    dbeta = g.sum(dim=red)
    gg = g * gamma.float().reshape(shape)
    dx = rstd[..., None] * (gg - gg.mean(-1, keepdim=True) - xhat * (gg * xhat).mean(-1, keepdim=True))
    return dx.to(x.dtype), dgamma, dbeta


# -------------------------------------------------------------------------- pooling
def maxpool_fwd(x, k: int, s: int, pad: int = 0):
    K, B, H, W, C = x.shape
    g = _to_grouped(x)
    y, idx = F.max_pool2d(g, k, s, padding=pad, return_indices=True)
    return _from_grouped(y, K).contiguous(), idx


def maxpool_bwd(dy, idx, x_shape, k: int, s: int, pad: int = 0):
    # scatter-ADD (overlapping windows, e.g. 3x3/s2, route several grads to one input;
    # max_unpool2d would overwrite instead of accumulate)
    K, B, H, W, C = x_shape
    g = _to_grouped(dy).float()
    out = torch.zeros((B, K * C, H * W), dtype=torch.float32, device=dy.device)
    out.scatter_add_(2, idx.flatten(2), g.flatten(2))
    return _from_grouped(out.view(B, K * C, H, W), K).to(dy.dtype).contiguous()


def avgpool_fwd(x, k: int, s: int):
    K = x.shape[0]
    return _from_grouped(F.avg_pool2d(_to_grouped(x), k, s), K).contiguous()


def avgpool_bwd(dy, x_shape, k: int, s: int):
    K, B, H, W, C = x_shape
    xg = torch.zeros((B, K * C, H, W), dtype=dy.dtype, device=dy.device, requires_grad=True)
    with torch.enable_grad():
        y = F.avg_pool2d(xg, k, s)
        (g,) = torch.autograd.grad(y, xg, _to_grouped(dy))
    return _from_grouped(g, K).contiguous()


def gap_fwd(x):
    """Global average pool [K,B,H,W,C] -> [K,B,C]."""
    return x.float().mean(dim=(2, 3)).to(x.dtype)


def gap_bwd(dy, x_shape):
    K, B, H, W, C = x_shape
    return (dy.float()[:, :, None, None, :] / (H * W)).expand(K, B, H, W, C).to(dy.dtype).contiguous()


# -------------------------------------------------------------------- cross entropy
def ce_fwd_bwd(logits, labels, valid=None):
    """Per-client mean softmax cross-entropy over valid samples, correct counts and the
    gradient dlogits (already divided by n_k). logits [K,B,C], labels [K,B] int."""
    K, B, C = logits.shape
    lf = logits.float()
    logp = torch.log_softmax(lf, dim=-1)
    nll = -logp.gather(-1, labels.long().unsqueeze(-1)).squeeze(-1)  # [K,B]
    if valid is None:
        m = torch.ones((K, B), device=logits.device)
        n = torch.full((K,), float(B), device=logits.device)
    else:
        m = (torch.arange(B, device=logits.device)[None, :] < valid[:, None].to(logits.device)).float()
        n = valid.to(logits.device).float().clamp(min=1)
    loss = (nll * m).sum(dim=1) / n
    correct = ((lf.argmax(-1) == labels.long()).float() * m).sum(dim=1)
    p = logp.exp()
    p.scatter_add_(-1, labels.long().unsqueeze(-1), -torch.ones_like(p[..., :1]))
    dlogits = p * (m / n[:, None]).unsqueeze(-1)
    return loss, correct, dlogits.to(logits.dtype)


# ----------------------------------------------------------------------- embedding
def embedding_fwd(tokens, table, scale: float = 1.0, pe=None):
    K = tokens.shape[0]
    table = _match(table, K)
    flat = tokens.reshape(K, -1).long()
    out = torch.gather(table, 1, flat.unsqueeze(-1).expand(-1, -1, table.shape[-1]))
    out = out.reshape(*tokens.shape, table.shape[-1])
    if scale != 1.0 or pe is not None:
        out = out.float() * scale
        if pe is not None:
            out = out + pe.to(out.device, torch.float32)
        out = out.to(table.dtype)
    return out


def embedding_bwd(dy, tokens, vocab: int, scale: float = 1.0):
    K = tokens.shape[0]
    D = dy.shape[-1]
    flat = tokens.reshape(K, -1).long()
    out = torch.zeros((K, vocab, D), dtype=torch.float32, device=dy.device)
    out.scatter_add_(1, flat.unsqueeze(-1).expand(-1, -1, D), dy.reshape(K, -1, D).float() * scale)
    return out


def seq_mean_fwd(x, lengths):
    L = x.shape[-2]
    m = (torch.arange(L, device=x.device) < lengths.to(x.device)[..., None]).to(torch.float32)
    return ((x.float() * m[..., None]).sum(-2) / lengths.to(x.device).clamp(min=1)[..., None].float()).to(x.dtype)


def seq_mean_bwd(dy, lengths, L: int):
    m = (torch.arange(L, device=dy.device) < lengths.to(dy.device)[..., None]).to(torch.float32)
    g = dy.float()[..., None, :] * m[..., None] / lengths.to(dy.device).clamp(min=1)[..., None, None].float()
    return g.to(dy.dtype)


# ----------------------------------------------------------------------- attention
def attn_drop_scale(shape, seeds, p: float, device) -> torch.Tensor:
    """[K,B,Hh,L,L] attention-probability dropout factor M/(1−p) (attention_mfma.hip attn_keep):
    keep iff mix32(((b·Hh + h)·L + q)·L + key, seed_k) >= p·2³² (32-bit index)."""
    import numpy as np

    from .fl import _mix

    K, B, Hh, L = shape[:4]
    thr = int(min(float(np.float32(p) * np.float32(4294967296.0)), 4294967040.0))
    hl = torch.arange(B * Hh, dtype=torch.int64, device=device).view(B, Hh, 1, 1)
    qi = torch.arange(L, dtype=torch.int64, device=device).view(1, 1, L, 1)
    kj = torch.arange(L, dtype=torch.int64, device=device).view(1, 1, 1, L)
    idx = ((hl * L + qi) * L + kj) & 0xFFFFFFFF
    sk = (seeds.long().to(device) & 0xFFFFFFFF).view(K, 1, 1, 1, 1)
    keep = _mix(idx.unsqueeze(0), sk) >= thr
    return keep.float() * (1.0 / (1.0 - p))


def attn_fwd(q, k, v, key_valid=None, drop_p: float = 0.0, drop_seeds=None):
    """q,k,v [K,B,Hh,L,dh]; key_valid [K,B] number of valid keys (padding mask) or None;
    drop_p / drop_seeds [K]: dropout on the attention probabilities (nn.MultiheadAttention's
    `dropout`). Returns o and the log-sum-exp [K,B,Hh,L] (fp32, of the undropped scores)."""
    scale = q.shape[-1] ** -0.5
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if key_valid is not None:
        L = k.shape[-2]
        km = torch.arange(L, device=q.device)[None, None, :] < key_valid[..., None].to(q.device)
        s = s.masked_fill(~km[:, :, None, None, :], float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse[..., None])
    if drop_p:
        p = p * attn_drop_scale(q.shape, drop_seeds, drop_p, q.device)
    o = torch.matmul(p, v.float())
    return o.to(q.dtype), lse


def attn_bwd(do, q, k, v, o, lse, key_valid=None, drop_p: float = 0.0, drop_seeds=None):
    scale = q.shape[-1] ** -0.5
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if key_valid is not None:
        L = k.shape[-2]
        km = torch.arange(L, device=q.device)[None, None, :] < key_valid[..., None].to(q.device)
        s = s.masked_fill(~km[:, :, None, None, :], float("-inf"))
    p = torch.exp(s - lse[..., None])
    msk = attn_drop_scale(q.shape, drop_seeds, drop_p, q.device) if drop_p else None
    dof = do.float()
    dv = torch.matmul((p * msk if msk is not None else p).transpose(-1, -2), dof)
    dp = torch.matmul(dof, v.float().transpose(-1, -2))
    if msk is not None:
        dp = dp * msk
    delta = (dof * o.float()).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.matmul(ds, k.float())
    dk = torch.matmul(ds.transpose(-1, -2), q.float())
    return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)


# ------------------------------------------------------------------------- sparse
def spmm(rowptr, col, val, x):
    """CSR (shared graph) times per-client dense x [K,N,F] -> [K,N,F]."""
    N = rowptr.numel() - 1
    A = torch.sparse_csr_tensor(rowptr.long(), col.long(), val.float(), size=(N, x.shape[1]))
    return torch.stack([(A @ x[k].float()) for k in range(x.shape[0])]).to(x.dtype)


# ---------------------------------------------------------------- optimiser / FL math
def sgd_step(theta, grad, mom, lr, active, weight_decay, momentum, dampening, nesterov,
             first_step, shadow=None, split=None):
    """Fused SGD over flat [K,P] buffers (torch.optim.SGD semantics, per-client lr[K]).
    `first_step[k]` (bool) makes buf = g (torch initialises the momentum buffer with the
    first gradient). Inactive clients are left untouched."""
    a = active.to(theta.device).bool()
    g = grad + weight_decay * theta if weight_decay != 0 else grad.clone()
    if momentum != 0:
        fs = first_step.to(theta.device).bool()[:, None]
        buf = torch.where(fs, g, momentum * mom + (1 - dampening) * g)
        mom.copy_(torch.where(a[:, None], buf, mom))
        d = g + momentum * buf if nesterov else buf
    else:
        d = g
    new = theta - lr.to(theta.device).float()[:, None] * d
    theta.copy_(torch.where(a[:, None], new, theta))
    if shadow is not None:
        shadow.copy_(theta.to(shadow.dtype))
    if split is not None:
        split_rows(theta, split)


def adam_step(theta, grad, m, v, lr, active, step, beta1, beta2, eps, weight_decay, shadow=None):
    a = active.to(theta.device).bool()[:, None]
    g = grad + weight_decay * theta if weight_decay != 0 else grad
    m_new = beta1 * m + (1 - beta1) * g
    v_new = beta2 * v + (1 - beta2) * g * g
    t = step.to(theta.device).float()[:, None]
    mhat = m_new / (1 - beta1 ** t)
    vhat = v_new / (1 - beta2 ** t)
    new = theta - lr.to(theta.device).float()[:, None] * mhat / (vhat.sqrt() + eps)
    m.copy_(torch.where(a, m_new, m))
    v.copy_(torch.where(a, v_new, v))
    theta.copy_(torch.where(a, new, theta))
    if shadow is not None:
        shadow.copy_(theta.to(shadow.dtype))


def weighted_sum(x, w, out=None):
    """out (fp64) += Σ_k w_k x[k,:] accumulated in fp64 (reference FedAvg accumulates in
    float64: `fed_avg_algorithm.py:39-52`). Returns the fp64 [P] accumulator."""
    acc = (x.double() * w.double().to(x.device)[:, None]).sum(dim=0)
    if out is None:
        return acc
    return out.add_(acc)


def mix_rows(x, w, out_dtype=torch.float32):
    """Subset models W[M, K] · x[K, P] (fp64 accumulation), cast to `out_dtype`."""
    return (w.double().to(x.device) @ x.double()).to(out_dtype)


def masked_weighted_sum(x, mask, w, num=None, den=None):
    """FedDropoutAvg: numerator Σ w_k m_k x_k and per-element denominator Σ w_k m_k (fp64)."""
    wm = mask.double() * w.double().to(x.device)[:, None]
    n, d = (x.double() * wm).sum(0), wm.sum(0)
    if num is not None:
        n = num.add_(n)
        d = den.add_(d)
    return n, d


def broadcast_rows(dst, src, rows=None):
    if rows is None:
        dst.copy_(src.unsqueeze(0).expand_as(dst))
    else:
        dst[rows] = src.unsqueeze(0).to(dst.dtype)


def delta(theta, base):
    return theta - base.unsqueeze(0)


def split_rows(theta, split):
    """split[k] = (bf16 hi, bf16 lo) planes of theta[k]: hi = RNE(x), lo = RNE(x - hi)."""
    hi = theta.to(torch.bfloat16)
    split[:, 0].copy_(hi)
    split[:, 1].copy_((theta - hi.float()).to(torch.bfloat16))
