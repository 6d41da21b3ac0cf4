"""Autograd wiring for the client-batched primitives.

Every parameterised op takes the parameter's compute view `w [K,...]` and its fp32 gradient
view `gw [K,...]` (a strided view into the cohort's flat grad buffer). Backward writes the
weight gradient *directly into* `gw` — parameters are never autograd leaves, so there is no
per-tensor gradient accumulation or zero-fill pass; autograd only tracks activations.
A zero-size `token` tensor that requires grad is threaded through every op so backward runs
even when the op's activation input does not need a gradient (e.g. the stem conv).
"""

from __future__ import annotations

import collections

import torch

from ..options import OPTIONS
from . import backend, ref


def _be(t):
    return backend.get(t)


# --------------------------------------------------------------------------- conv2d
class ResidualLink:
    """Hands a second gradient of a residual block's input to the block's first conv, whose
    dgrad adds it in its epilogue: autograd then never materialises `dX_conv + dX_other` with a
    separate add pass over the block input.
    - identity shortcut: the block's last BN (whose backward runs first) deposits dX_shortcut;
    - downsample shortcut: the shortcut conv (`donor`) deposits its dX. Autograd normally runs
      it before the main branch reaches the first conv; if not, the first conv marks
      `receiver_done` and the donor returns its dX to autograd as usual (same result).
      A 1x1 stride-s donor (fp32 native) deposits only the stride grid — the only pixels its dX
      is non-zero on — as a dense [K, B, ceil(H/s), ceil(W/s), C] tensor (`compact` = s): one
      stride-1 GEMM instead of s² parity launches (s² − 1 of them writing zeros), and the
      receiver's class-(0, 0) launch alone reads it (ops.hip.conv_dgrad acc_compact)."""

    __slots__ = ("grad", "receiver_done", "compact", "receiver_stride")

    def __init__(self):
        self.grad = None
        self.receiver_done = False
        self.compact = 0
        self.receiver_stride = 1  # stride of the receiving conv (set by its forward)


class MaskedGrad:
    """A gradient g = dy · relu' kept as its factors: `dy` [K, ..., C] fp32 and the 1-bit ReLU mask
    [K, rows, C / 8]. The identity shortcut of a ResNet block hands its gradient to the block's first
    conv this way (ResidualLink.grad): that conv's dgrad epilogue gates dy by the bits while it adds
    it (ops.hip.conv_dgrad acc_mask), so the BN backward never writes dy·relu' and nobody reads it
    back. `dense()` builds the tensor for any other consumer."""

    __slots__ = ("dy", "mask")

    def __init__(self, dy, mask):
        self.dy, self.mask = dy, mask

    def dense(self):
        K, C = self.dy.shape[0], self.dy.shape[-1]
        bits = torch.arange(8, device=self.mask.device, dtype=torch.uint8)
        keep = ((self.mask.view(K, -1, C // 8, 1) >> bits) & 1).reshape(K, -1, C).bool()
        return torch.where(keep, self.dy.reshape(K, -1, C), torch.zeros((), dtype=self.dy.dtype,
                                                                          device=self.dy.device)).view(self.dy.shape)


# A/B switches (BN statistics from the conv epilogue, BN backward partials, split planes, ...)
# live in options.OPTIONS and are read when an op runs


class BNStats:
    """Links a conv to the BatchNorm that consumes its output:
    - statistics: the fp32 conv epilogue writes per-32-row Σy / Σy² partials (of the first
      `valid[k]` samples' rows) and the BN consumes them instead of re-reading y in a statistics
      pass. `part` stays None when the producing conv could not provide them (CPU oracle, bf16
      kernels, LDS-DMA path);
    - `dy_planes_ok`: the conv runs its dgrad and wgrad on split planes (csrc/conv_pl.hip), so
      the BN backward writes only dX's planes (ops.hip.bn_bwd dx_planes=2), never the fp32 dX."""

    __slots__ = ("valid", "part", "dy_planes_ok")

    def __init__(self, valid=None):
        self.valid = valid
        self.part = None
        self.dy_planes_ok = False


# BN backward passes that used a dgrad's partials ("used"), whose consumer wrote none (a strided
# or absent conv: "none"), or whose dY was not that dgrad's output ("fallback"): tests, reports
bn_bwd_parts_count = {"used": 0, "none": 0, "fallback": 0}


class BNBwdLink:
    """Links a training BatchNorm's output to the stride-1 conv that consumes it: that conv's dgrad
    epilogue writes the BN backward's partial sums Σĝ, Σĝ·x̂ (ĝ = dY·relu') while it stores dX
    (= the BN's dY), so the BN backward skips its reduction pass over dY and x (ops.hip.conv_dgrad
    bnb=). The BN uses them only if the dY autograd hands it is that very dgrad output, unmodified
    (`key` = storage pointer + version): any other gradient summed in (a second consumer, a late
    residual donor) makes it fall back to its own pass."""

    __slots__ = ("x", "mask", "mean", "rstd", "valid", "part", "key")

    def __init__(self, x, mask, mean, rstd, valid):
        self.x, self.mask, self.mean, self.rstd, self.valid = x, mask, mean, rstd, valid
        self.part = None
        self.key = None

    def args(self, part):
        return (part, self.x, self.mask, self.mean, self.rstd, self.valid, None)


# Split-plane operands (csrc/conv_pl.hip). A tensor produced together with its bf16 (hi, lo)
# planes carries them as attribute `_dls_planes` ([K, 2, *shape[1:]], ops.hip.planes_buffer
# layout); `_dls_planes_only` marks a tensor whose fp32 bytes ARE those planes (the producer
# wrote nothing else) — only a planes-reading GEMM may consume it. OPTIONS.planes = False
# disables them.


def _planes_of(t):
    return getattr(t, "_dls_planes", None)


def _tag_planes(t, planes, only: bool):
    t._dls_planes = planes
    t._dls_planes_only = only
    return t


def _require_fp32(t, who: str):
    if getattr(t, "_dls_planes_only", False):
        raise RuntimeError(f"{who}: a planes-only activation reached an op that reads fp32 values")


class DeferredBN:
    """A BatchNorm(+ReLU) output whose apply pass is deferred to its one consumer, a 3x3 stride-1
    conv that applies it while staging its input (ops.hip.conv_halo_bn_fwd, csrc/conv_halo.hip
    BNF): the normalised activation is never read back from HBM. The BN hands autograd the
    planes-only alias of `yp` (batch_norm planes=3); in training the fused conv also writes the
    planes and ReLU bits (its weight gradient and the BN backward read them). A consumer that
    cannot fuse — or anything that needs the values first — calls `materialize()`, which runs
    the ordinary apply pass into the same buffers. Bits are identical either way."""

    __slots__ = ("x", "coef", "relu", "valid_rows", "yp", "mask", "write_out", "pending")

    def __init__(self, x, coef, relu, valid_rows, yp, mask, write_out):
        self.x, self.coef, self.relu, self.valid_rows = x, coef, relu, valid_rows
        self.yp, self.mask, self.write_out = yp, mask, write_out
        self.pending = True

    def materialize(self):
        if self.pending:
            from . import hip

            hip.bn_apply_only(self.x, self.coef, self.valid_rows, self.relu, self.yp, self.mask)
            self.pending = False


# downsample BN applies folded into the next BN ("folded") or run as their own pass ("materialized")
res_fold_count = {"folded": 0, "materialized": 0}


class DeferredRes:
    """A BatchNorm output without ReLU whose one reader is the next BatchNorm, as its residual — a
    ResNet downsample shortcut's BN (batch_norm planes=4): the statistics and (scale, shift) are
    computed, the output is never written, and the reader folds the apply into its own
    (hip.bn_fwd res_coef: act(bn2(x) + scale·x_ds + shift), the bits of applying it first). The
    backward needs no output (no ReLU). Anything else that needs the values calls materialize(),
    the ordinary apply pass into the same tensor."""

    __slots__ = ("x", "coef", "valid_rows", "y", "pending")

    def __init__(self, x, coef, valid_rows, y):
        self.x, self.coef, self.valid_rows, self.y = x, coef, valid_rows, y
        self.pending = True

    def materialize(self):
        if self.pending:
            from . import hip

            hip.bn_apply_only(self.x, self.coef, self.valid_rows, False, None, y=self.y)
            self.pending = False
            res_fold_count["materialized"] += 1


# deferred BN backward applies (DeferredBNBwd) taken by a halo weight gradient's loader ("wgrad")
# or run as their own pass ("materialized"): tests, reports
bn_bwd_defer_count = {"wgrad": 0, "materialized": 0}


class DeferredBNBwd:
    """A training BatchNorm's input gradient dX whose apply pass is deferred to the conv that
    produced the BN's input (OPTIONS.bn_bwd_in_wgrad): the BN backward computed only its
    coefficients (a, d, e) and dγ / dβ, and hands autograd the planes-only alias of an unwritten
    `dxp`. That conv's backward runs its halo weight gradient first, in dY mode 2
    (csrc/conv_halo_wgrad.hip), which builds dX = a·(dy·relu') + e·x + d in its loader and stores
    the planes for the dgrad on the way; any other consumer calls `materialize()` — the ordinary
    apply pass into the same planes, with the same bits."""

    __slots__ = ("dy", "x", "mask", "coef", "valid_rows", "dxp", "pending")

    def __init__(self, dy, x, mask, coef, valid_rows, dxp):
        self.dy, self.x, self.mask, self.coef, self.valid_rows, self.dxp = dy, x, mask, coef, valid_rows, dxp
        self.pending = True

    def materialize(self):
        if self.pending:
            from . import hip

            hip.bn_bwd_apply_planes(self.dy, self.x, self.mask, self.coef, self.valid_rows, self.dxp)
            self.pending = False
            bn_bwd_defer_count["materialized"] += 1

    def wgrad_args(self):
        return (self.dy, self.x, self.mask, self.coef, self.valid_rows, self.dxp)


class _Conv(torch.autograd.Function):
    """Conv2d over the client dim. If the input carries more channels than the weight (image
    data stored zero-padded to 8 channels), the weight is zero-padded to match and only the
    real channels' gradient is written back."""

    @staticmethod
    def forward(ctx, x, token, w, gw, stride, pad, b, gb, link=None, stats=None, w_split=None, donor=None,
                sgd=None):
        be = _be(x)
        ci = w.shape[-1]
        # (the fused SGD step: plane wgrads of unpadded, bias-free fp32 convs only)
        ctx.sgd = sgd if (sgd is not None and be is not ref and x.dtype == torch.float32 and gw is not None
                          and b is None and x.shape[-1] == ci and w_split is not None) else None
        if x.shape[-1] > ci:
            w = torch.nn.functional.pad(w, (0, x.shape[-1] - ci))
            w_split = None  # (the padded copy has no planes)
        if be is ref or x.dtype != torch.float32:
            w_split = None
        # split-plane GEMMs: x's planes (from the producing BN) + the weight planes
        xp = _planes_of(x)
        use_pl = (xp is not None and w_split is not None and x.is_contiguous()
                  and be.conv_planes_ok(x.shape[-1], w.shape[1]) and be.planes_fit(x[0].numel()))
        if getattr(x, "_dls_planes_only", False) and not use_pl:
            raise RuntimeError("conv2d: planes-only input but the split-plane GEMM cannot run here")
        pl = {"x_planes": xp} if use_pl else {}
        ctx.xp = xp if use_pl else None
        if stats is not None:
            stats.dy_planes_ok = use_pl and b is None
        K, B, H, W = x.shape[:4]
        KH = w.shape[2]
        OH, OW = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - w.shape[3]) // stride + 1
        y_numel = B * OH * OW * w.shape[1]
        # per-client windows past 2 GiB run batch-chunked (ops.hip): no epilogue statistics there
        big = be is not ref and max(x[0].numel(), y_numel) * x.element_size() >= (1 << 31)
        if stats is not None:
            stats.dy_planes_ok = stats.dy_planes_ok and be.planes_fit(y_numel)
        want_stats = stats is not None and be is not ref and x.dtype == torch.float32 and not big
        y = None
        ctx.bn_src = None
        defer = getattr(x, "_dls_bn_defer", None)
        if defer is not None and defer.pending:
            # a deferred BN input (DeferredBN): apply it in this conv's halo loader if it can
            if (use_pl and stride == 1 and pad == 1 and KH == 3 and w.shape[3] == 3 and b is None
                    and be.halo_bn_ok(x.shape, w)):
                part = (torch.empty((K, be.conv_stats_parts(B * OH * OW), 2, w.shape[1]), dtype=torch.float32,
                                    device=x.device) if want_stats else None)
                # the weight gradient applies the BN in its own loader too (halo wgrad x mode 2): then
                # the normalised planes are never written, only the ReLU bits the BN backward reads
                bn_wgrad = (defer.write_out and gw is not None and OPTIONS.halo_wgrad
                            and x.shape[-1] == ci and be.halo_wgrad_ok(x.shape, w.shape[1]))
                y = be.conv_halo_bn_fwd(defer.x.view(x.shape), defer.coef, defer.relu, defer.valid_rows, w, w_split,
                                        stats=part, stats_valid=stats.valid if want_stats else None,
                                        yp=defer.yp if defer.write_out and not bn_wgrad else None,
                                        mask=defer.mask if defer.write_out else None)
                if y is not None:
                    defer.pending = False
                    if want_stats:
                        stats.part = part
                    if bn_wgrad:
                        ctx.bn_src = (defer.x.view(x.shape), defer.coef, defer.relu, defer.valid_rows)
            defer.materialize()
        if y is not None:
            pass
        elif want_stats:
            stats.part = torch.empty((K, be.conv_stats_parts(B * OH * OW), 2, w.shape[1]), dtype=torch.float32,
                                     device=x.device)
            y = be.conv_fwd(x, w, stride, pad, bias=b, stats=stats.part, stats_valid=stats.valid,
                            **({"w_split": w_split} if w_split is not None else {}), **pl)
        elif w_split is not None:
            y = be.conv_fwd(x, w, stride, pad, bias=b, w_split=w_split, **pl)
        else:
            y = be.conv_fwd(x, w, stride, pad, bias=b)
        ctx.w_split = w_split
        # the consuming BN will hand the backward dY as planes only: a dY without them (a tensor
        # rebuilt on the way, which drops the _dls_planes attributes) must fail, not be read as fp32
        ctx.expect_dy_planes = stats is not None and stats.dy_planes_ok
        ctx.x_planes_only = bool(getattr(x, "_dls_planes_only", False))
        bnb = getattr(x, "_dls_bnb", None) if OPTIONS.bn_bwd_parts else None
        # (the dgrad writes the partials only in one launch: a dY or dX window past 2 GiB runs
        # batch-chunked, e.g. a 64 -> 256 1x1 conv whose output alone crosses it)
        if bnb is not None and not (be is not ref and donor is None and x.shape[-1] == ci and not big
                                    and be.bn_bwd_parts_ok(x.shape, stride, x.dtype)):
            bnb = None
        ctx.bnb = bnb
        ctx.halo_wgrad = OPTIONS.halo_wgrad  # (read once: the backward follows the forward's decision)
        # (valid samples: the BatchNorm around this conv zeroes the rows past them, so the halo wgrad
        # skips those images' tiles)
        ctx.valid = stats.valid if (stats is not None and OPTIONS.skip_invalid) else None
        ctx.dgrad_wt = be is not ref
        ctx.save_for_backward(x, w)
        ctx.gw, ctx.gb, ctx.stride, ctx.pad, ctx.ci = gw, gb, stride, pad, ci
        ctx.link = link
        ctx.donor = donor
        if link is not None:
            link.receiver_stride = stride
        return y

    @staticmethod
    def _wgrad(ctx, dy, x, w, dyp, be, bbd=None, sgd_ok=True) -> bool:
        """The weight gradient (or the SGD step fused into it). `bbd` (DeferredBNBwd): only the halo
        kernel's BN-backward dY mode — returns False, launching nothing, when it cannot serve;
        `sgd_ok` False: store dW (the flat step covers the weight)."""
        if bbd is not None:
            if not (ctx.stride == 1 and ctx.pad == 1 and w.shape[2] == 3 and w.shape[3] == 3):
                return False
            sgd = ctx.sgd if sgd_ok else None
            if ctx.bn_src is not None:
                xr, coef, relu, vrows = ctx.bn_src
                ok = be.halo_wgrad(dy, xr, ctx.gw, bn=(coef, relu, vrows), valid=ctx.valid, sgd=sgd,
                                   bn_bwd=bbd.wgrad_args())
            else:
                ok = be.halo_wgrad(dy, x, ctx.gw, x_planes=ctx.xp, valid=ctx.valid, sgd=sgd, bn_bwd=bbd.wgrad_args())
            if ok and sgd is not None:
                sgd[0].done.add(sgd[1])
            return bool(ok)
        padded = w.shape[-1] > ctx.ci
        K = x.shape[0]
        sgd = ctx.sgd if not padded else None
        stepped = False
        gw = torch.empty((K,) + tuple(w.shape[1:]), dtype=torch.float32, device=dy.device) if padded else ctx.gw
        if be is ref:
            gw.copy_(ref.conv_wgrad(dy.float(), x.float(), (K,) + tuple(w.shape[1:]), ctx.stride, ctx.pad))
            if ctx.gb is not None:
                ctx.gb.copy_(dy.float().sum(dim=(1, 2, 3)))
        elif ctx.bn_src is not None:
            # x's planes were never written: the halo wgrad applies the BN to the raw tensor
            xr, coef, relu, vrows = ctx.bn_src
            if not be.halo_wgrad(dy, xr, gw, dy_planes=dyp, bn=(coef, relu, vrows), valid=ctx.valid,
                                 sgd=sgd):
                raise RuntimeError("conv2d backward: the halo wgrad refused a shape its forward accepted")
            stepped = sgd is not None
        elif (ctx.halo_wgrad and ctx.stride == 1 and ctx.pad == 1 and w.shape[2] == 3 and w.shape[3] == 3
              and not padded and be.halo_wgrad(dy, x, gw, dy_planes=dyp, x_planes=ctx.xp, valid=ctx.valid,
                                               sgd=sgd)):
            stepped = sgd is not None
        elif dyp is not None:
            stepped = be.conv_wgrad(dy, x, gw, ctx.stride, ctx.pad, dy_planes=dyp, x_planes=ctx.xp, sgd=sgd)
        else:
            if ctx.x_planes_only:
                raise RuntimeError("conv2d backward: fp32 dY with a planes-only input")
            be.conv_wgrad(dy, x, gw, ctx.stride, ctx.pad)
            if ctx.gb is not None:
                be.bias_grad(dy, ctx.gb)
        if padded:
            ctx.gw.copy_(gw[..., : ctx.ci])
        if stepped:
            sgd[0].done.add(sgd[1])  # (this weight's optimiser step ran in its wgrad)
        return True

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        be = _be(dy)
        dy = dy.contiguous()
        dx = None
        link = ctx.link
        acc = link.grad if link is not None else None
        acc_mask = None
        if isinstance(acc, MaskedGrad):
            if be is not ref and dy.dtype == torch.float32 and ctx.needs_input_grad[0] and not link.compact:
                acc, acc_mask = acc.dy.contiguous(), acc.mask  # (gated in the dgrad epilogue)
            else:
                acc = acc.dense()
        acc_compact = False
        if link is not None:
            if acc is not None and link.compact:
                if link.compact == ctx.stride and ctx.stride > 1 and be is not ref and ctx.needs_input_grad[0]:
                    acc_compact = True
                else:  # (a receiver that cannot take the stride grid: expand it)
                    full = torch.zeros(x.shape, dtype=acc.dtype, device=acc.device)
                    full[:, :, :: link.compact, :: link.compact] = acc
                    acc = full
            link.grad = None
            link.compact = 0
            if acc is None:
                link.receiver_done = True  # (a late donor hands its dX to autograd instead)
        dyp = _planes_of(dy)
        wgrad_done = False
        wt_pre = None
        bbd = getattr(dy, "_dls_bnbwd", None)
        if bbd is not None and bbd.pending:
            # dY is a deferred BN input gradient (DeferredBNBwd): the halo weight gradient applies
            # the BN backward in its loader and writes dY's planes, so it runs before the dgrad
            if ctx.gw is not None and be is not ref and ctx.halo_wgrad and w.shape[-1] == ctx.ci:
                sgd_ok = True
                if ctx.sgd is not None and ctx.needs_input_grad[0]:
                    # its SGD epilogue rewrites the weight planes the dgrad reads: the dgrad's
                    # transposed copy is built first, or the flat step takes this weight
                    wt_pre = (be.dgrad_wt_prebuild(dy.shape, w, ctx.w_split, x.shape[2:4], ctx.stride, ctx.pad)
                              if ctx.dgrad_wt and ctx.w_split is not None and not acc_compact and ctx.donor is None
                              else None)
                    sgd_ok = wt_pre is not None
                wgrad_done = _Conv._wgrad(ctx, dy, x, w, dyp, be, bbd, sgd_ok=sgd_ok)
            if wgrad_done:
                bbd.pending = False
                bn_bwd_defer_count["wgrad"] += 1
            else:
                bbd.materialize()
        if dyp is not None and ctx.xp is None:
            raise RuntimeError("conv2d backward: dY planes without the input's planes")
        if dyp is None:
            if ctx.expect_dy_planes:
                raise RuntimeError("conv2d backward: the BN wrote dY as planes only, but they did not arrive")
            _require_fp32(dy, "conv2d backward")
        donor = ctx.donor
        compact = (donor is not None and not donor.receiver_done and be is not ref and dy.dtype == torch.float32
                   and ctx.stride > 1 and ctx.pad == 0 and w.shape[2] == 1 and w.shape[3] == 1 and acc is None
                   and w.shape[-1] == ctx.ci and donor.receiver_stride == ctx.stride)
        if ctx.needs_input_grad[0] and compact:
            # 1x1 stride-s downsample shortcut: dX is non-zero only on the stride grid, where it is
            # the stride-1 1x1 dgrad of dY — computed compactly and handed to the block's first conv
            dx = be.conv_dgrad(dy, w, dy.shape[2:4], 1, 0, w_split=ctx.w_split,
                               **({"dy_planes": dyp} if dyp is not None else {}))
        elif ctx.needs_input_grad[0]:
            if acc_compact:
                dx = be.conv_dgrad(dy, w, x.shape[2:4], ctx.stride, ctx.pad, acc=acc, w_split=ctx.w_split,
                                   acc_compact=True, **({"dy_planes": dyp} if dyp is not None else {}))
            else:
                kw = {}
                bnb = ctx.bnb
                if bnb is not None:
                    K, B, H, W, Ci = x.shape
                    part = torch.empty((K, be.conv_stats_parts(B * H * W), 2, Ci), dtype=torch.float32,
                                       device=dy.device)
                    kw["bnb"] = bnb.args(part)
                if dyp is not None:
                    kw["dy_planes"] = dyp
                if ctx.w_split is not None:
                    kw["w_split"] = ctx.w_split
                if acc_mask is not None:
                    kw["acc_mask"] = acc_mask
                if ctx.dgrad_wt:
                    kw["wt"] = True
                if wt_pre is not None:
                    kw["wt_buf"] = wt_pre
                dx = be.conv_dgrad(dy, w, x.shape[2:4], ctx.stride, ctx.pad, acc=acc, **kw)
                if bnb is not None:
                    bnb.part, bnb.key = part, (dx.data_ptr(), dx._version)
            if dx.shape[-1] > ctx.ci:
                dx = dx[..., : ctx.ci]
        elif acc is not None:
            dx = acc if acc_mask is None else MaskedGrad(acc, acc_mask).dense()
        if ctx.gw is not None and not wgrad_done:
            _Conv._wgrad(ctx, dy, x, w, dyp, be)
        if donor is not None and dx is not None and not donor.receiver_done:
            donor.grad = dx  # added by the block's first conv in its dgrad epilogue
            donor.compact = ctx.stride if compact else 0
            dx = None
        return dx, None, None, None, None, None, None, None, None, None, None, None, None


def conv2d(x, token, w, gw, stride=1, pad=0, b=None, gb=None, link: ResidualLink | None = None,
           stats: BNStats | None = None, w_split: torch.Tensor | None = None, donor: ResidualLink | None = None,
           sgd=None):
    """`link`: this conv's input gets a second gradient through the link (identity shortcut of a
    residual BN, or a downsample conv given the same link as `donor`), added in the dgrad epilogue.
    `donor`: this conv's input gradient is deposited in the link instead of returned. `stats`: the output feeds a
    BatchNorm given the same holder (its statistics come from this conv's epilogue)."""
    if link is not None:
        assert w.shape[-1] == x.shape[-1], "a residual link needs an unpadded conv"
    return _Conv.apply(x, token, w, gw, stride, pad, b, gb, link, stats, w_split, donor, sgd)


# --------------------------------------------------------------------------- linear
class _Linear(torch.autograd.Function):
    """y = x Wᵀ + b with optional epilogue fusions (Transformer FFN / residual branches):
    relu      — ReLU in the GEMM epilogue (no separate activation pass);
    premasked — the ReLU gradient is applied by the consumer (the next linear's gate_input),
                so this backward takes dy as d(pre-activation) directly;
    gate_input— x is a ReLU output: dX leaves through ReLU' (zeroed where x <= 0) in the dgrad
                epilogue, one pass instead of a separate threshold-backward;
    residual  — y += residual in the epilogue (its gradient is dy, passed straight through);
    drop_p    — dropout of the GEMM output (after the ReLU, before the residual add) in the
                epilogue, mask from `drop_seeds` [K] (ops dropout_apply rule); the backward masks
                the GEMM branch's gradient once (premasked outputs leave that to the consumer);
    gate_scale— the 1/(1-p) of the producer's dropout, applied with the gate_input ReLU'.
    Split planes (fp32 native, with the weight's planes `w_split`; csrc/conv_pl.hip):
    x_planes  — x's planes (a LayerNorm / planes-writing linear output): the forward GEMM and
                the weight gradient read them;
    out_planes— the epilogue also writes y's planes (tagged `_dls_planes`) for the next linear;
    dx_planes — the dgrad epilogue also writes dX's planes (for the producer's backward);
    a dy arriving with planes, or masked here by the dropout backward (which then writes them),
    feeds the dgrad and the weight gradient as planes. x and y keep their leading shape."""

    @staticmethod
    def forward(ctx, x, token, w, b, gw, gb, residual=None, relu=False, premasked=False, gate_input=False,
                drop_p=0.0, drop_seeds=None, gate_scale=1.0, w_split=None, x_planes=None, out_planes=False,
                dx_planes=False, res_link=None, acc_link=None, sgd=None):
        be = _be(x)
        ctx.res_link, ctx.acc_link = res_link, acc_link
        shp = x.shape
        x = x.reshape(shp[0], -1, shp[-1])
        ctx.res_shape = residual.shape if residual is not None else None
        if residual is not None:
            residual = residual.reshape(shp[0], x.shape[1], -1).contiguous()
        native = be is not ref and x.dtype == torch.float32 and w_split is not None and OPTIONS.planes
        if not native:
            w_split = x_planes = None
            out_planes = dx_planes = False
        if not OPTIONS.tfm_planes:
            out_planes = dx_planes = False
        ws = {"w_split": w_split} if w_split is not None else {}
        xp = {"x_planes": x_planes} if x_planes is not None else {}
        y = be.linear_fwd(x, w, b, relu=relu, acc=residual, drop_p=drop_p, drop_seeds=drop_seeds, **ws, **xp,
                          **({"out_planes": True} if out_planes else {}))
        yp = None
        if out_planes:
            y, yp = y
        ctx.ws = ws
        mask_dy = relu and not premasked
        ctx.save_for_backward(x, w, y if mask_dy else None, drop_seeds if drop_p else None)
        ctx.x_planes = x_planes
        ctx.gw, ctx.gb = gw, gb
        ctx.mask_dy, ctx.gate_input, ctx.has_res = mask_dy, gate_input, residual is not None
        ctx.drop_p, ctx.premasked, ctx.gate_scale = drop_p, premasked, gate_scale
        ctx.native, ctx.dx_planes, ctx.shape = native, dx_planes, shp
        ctx.drop_planes = bool(OPTIONS.tfm_planes)
        ctx.sgd = sgd if (native and gw is not None) else None  # (the plane weight gradient may step W)
        yo = y.view(*shp[:-1], y.shape[-1])
        if yp is not None:
            _tag_planes(yo, yp.view((shp[0], 2) + tuple(yo.shape[1:])), False)
        return yo

    @staticmethod
    def backward(ctx, dy):
        x, w, y, seeds = ctx.saved_tensors
        be = _be(dy)
        K, N, Fi = x.shape
        dyp = _planes_of(dy) if ctx.native else None
        dy = dy.reshape(K, N, -1)
        if dyp is None:
            dy = dy.contiguous()
        _require_fp32(dy, "linear backward")
        Fo = dy.shape[-1]
        dres = dy.reshape(ctx.res_shape) if ctx.has_res else None
        if dres is not None and ctx.res_link is not None and not ctx.res_link.receiver_done:
            ctx.res_link.grad = dres.contiguous()  # added by the residual input's other reader's dgrad
            dres = None
        acc = None
        if ctx.acc_link is not None:  # (a residual branch's gradient of x, deposited by its linear)
            acc = ctx.acc_link.grad
            ctx.acc_link.grad = None
            ctx.acc_link.receiver_done = True
        bias_done = False  # (the bias gradient already written by the dropout backward)
        if ctx.mask_dy:
            # y > 0 iff the unit was kept AND its pre-activation was positive
            dy = dy * (y > 0).to(dy.dtype)
            dyp = None
            if ctx.drop_p:
                dy = dy * (1.0 / (1.0 - ctx.drop_p))
        elif ctx.drop_p and not ctx.premasked:
            # the GEMM branch's gradient, with its planes for the dgrad / wgrad GEMMs
            if ctx.native and ctx.drop_planes:
                # (the bias gradient comes from the dropout pass's column sums: dY is written
                # only as planes, and no separate column-sum pass reads it)
                cs = ctx.gb is not None and ctx.gw is not None and Fo % 2 == 0
                # planes only when both GEMMs that read dY take the plane path (else they read fp32 dY)
                pl_only = (ctx.x_planes is not None and be.planes_ok(Fo, Fi) and Fo % 8 == 0
                           and ctx.ws.get("w_split") is not None)
                dy, dyp = be.dropout_apply(dy, seeds, ctx.drop_p,
                                           planes=2 if (ctx.gb is None or (cs and pl_only)) else 1,
                                           colsum=ctx.gb if cs else None)
                bias_done = cs
            else:
                dy, dyp = be.dropout_apply(dy, seeds, ctx.drop_p), None
        if dyp is not None:
            dyp = dyp.reshape(K, 2, N, Fo)
        gate = x.contiguous() if ctx.gate_input else None
        dx = None
        if ctx.needs_input_grad[0]:
            kw = dict(ctx.ws)
            if dyp is not None:
                kw["dy_planes"] = dyp
            if ctx.dx_planes:
                kw["out_planes"] = True
            if acc is not None and be is not ref:
                kw["acc"] = acc.reshape(K, N, Fi)
            dx = be.linear_dgrad(dy, w, gate=gate, gate_scale=ctx.gate_scale, **kw)
            dxp = None
            if ctx.dx_planes:
                dx, dxp = dx
            if acc is not None and be is ref:
                dx = dx + acc.reshape(dx.shape)
            dx = dx.view(ctx.shape)
            if dxp is not None:
                _tag_planes(dx, dxp.view((K, 2) + tuple(ctx.shape[1:])), False)
        if ctx.gw is not None:
            if be is ref:
                dw, db = ref.linear_wgrad(dy.float(), x.float(), ctx.gb is not None)
                ctx.gw.copy_(dw)
                if ctx.gb is not None:
                    ctx.gb.copy_(db)
            else:
                pl = {"dy_planes": dyp, "x_planes": ctx.x_planes} if (dyp is not None and ctx.x_planes is not None) else {}
                if pl and ctx.sgd is not None:
                    pl["sgd"] = ctx.sgd
                if be.linear_wgrad(dy, x, ctx.gw, None if bias_done else ctx.gb, **pl):
                    ctx.sgd[0].done.add(ctx.sgd[1])  # (W stepped in its weight-gradient kernel)
        if dx is None and acc is not None:
            dx = acc.reshape(ctx.shape)
        return (dx, None, None, None, None, None, dres, None, None, None, None, None, None, None, None, None, None, None,
                None, None)


def linear(x, token, w, b, gw, gb, residual=None, relu=False, premasked=False, gate_input=False,
           drop_p: float = 0.0, drop_seeds=None, gate_scale: float = 1.0, w_split=None, out_planes: bool = False,
           dx_planes: bool = False, res_link: ResidualLink | None = None, acc_link: ResidualLink | None = None,
           sgd=None):
    """x [K, ..., Fi] -> [K, ..., Fo]. Epilogue fusions and split planes: see _Linear
    (relu / premasked / gate_input / residual / dropout / out_planes / dx_planes). `w_split`: the
    weight's pre-split bf16 planes (BoundParams.ws) for the fp32 GEMMs; x's planes, when it
    carries them (`_dls_planes`), are read by the plane GEMMs. `res_link` (with `residual`): the
    residual's gradient is deposited in the link instead of returned; `acc_link`: this linear's
    dgrad adds the link's gradient to dX in its epilogue — give both to the two readers of one
    tensor (the residual add and the next linear) and autograd never adds their gradients in a
    separate pass. The depositing linear must be later in the forward (its backward runs first);
    otherwise the receiver marks the link done and the gradient goes back to autograd."""
    assert not (relu and residual is not None), "ReLU and residual epilogues are not combined"
    return _Linear.apply(x, token, w, b, gw, gb, residual, relu, premasked, gate_input, drop_p, drop_seeds,
                         gate_scale, w_split, _planes_of(x), out_planes, dx_planes, res_link, acc_link, sgd)


class _LinearSharedInput(torch.autograd.Function):
    """y[k] = x W_kᵀ for ONE input x [N, Fi] shared by K weight rows: a single GEMM against the
    concatenated weights [K·Fo, Fi] (GCN first layer: node features are common to all clients)."""

    @staticmethod
    def forward(ctx, x, token, w, gw):
        be = _be(x)
        K, Fo, Fi = w.shape
        wcat = w.reshape(1, K * Fo, Fi).contiguous()
        y = be.linear_fwd(x.unsqueeze(0).contiguous(), wcat, None)  # [1, N, K*Fo]
        ctx.save_for_backward(x)
        ctx.gw, ctx.K, ctx.Fo = gw, K, Fo
        return y[0].view(-1, K, Fo).permute(1, 0, 2).contiguous()

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        if ctx.gw is not None:
            be = _be(dy)
            K, Fo = ctx.K, ctx.Fo
            dyc = dy.permute(1, 0, 2).reshape(1, -1, K * Fo).contiguous()
            Fi = x.shape[-1]
            if be is ref:
                dw, _ = ref.linear_wgrad(dyc.float(), x.unsqueeze(0).float(), False)
            else:
                dw = torch.empty((1, K * Fo, Fi), dtype=torch.float32, device=dy.device)
                be.linear_wgrad(dyc, x.unsqueeze(0).contiguous(), dw, None)
            ctx.gw.copy_(dw.view(K, Fo, Fi))
        return None, None, None, None


def linear_shared_input(x, token, w, gw):
    return _LinearSharedInput.apply(x, token, w, gw)


# ------------------------------------------------------------------------ batchnorm
class _BN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, token, gamma, beta, ggamma, gbeta, valid_rows, relu, residual, link=None, stats=None,
                planes=0):
        be = _be(x)
        K = x.shape[0]
        C = x.shape[-1]
        _require_fp32(x, "batch_norm")
        if residual is not None:
            _require_fp32(residual, "batch_norm residual")
        x3 = x.reshape(K, -1, C)
        r3 = residual.reshape(K, -1, C) if residual is not None else None
        mask = None
        yp = None
        bnb = None
        res_coef = None
        fold = getattr(residual, "_dls_res_fold", None) if residual is not None else None
        if fold is not None and fold.pending:
            # a downsample BN's apply folded into this one (DeferredRes), or materialised first
            if (be is not ref and x.dtype == torch.float32 and fold.valid_rows is valid_rows
                    and fold.x.shape == x3.shape and x3.is_contiguous()):
                r3, res_coef = fold.x, fold.coef
                fold.pending = False
                res_fold_count["folded"] += 1
            else:
                fold.materialize()
        fold_out = None
        if be is ref:
            y, mean, rstd = be.bn_fwd(x3, gamma, beta, valid_rows, relu, r3)
        else:  # native: 1-bit ReLU mask so the backward need not re-read y
            pre = stats.part if stats is not None else None
            planes = planes if (OPTIONS.planes and x.dtype == torch.float32 and x.is_contiguous()
                                and be.planes_fit(x[0].numel())) else 0
            # (inference passes — evaluation, GTG utilities — write no ReLU mask: no backward reads
            # it. Autograd is off inside Function.forward, so ask which inputs need a gradient)
            wm = any(ctx.needs_input_grad)
            C8 = C % 8 == 0
            if planes == 3 and not (OPTIONS.bn_fused_halo and residual is None and C8 and x3.is_contiguous()):
                planes = 2  # (no deferral: apply now, planes only)
            if planes == 4 and not (OPTIONS.bn_res_fold and residual is None and not relu and x3.is_contiguous()):
                planes = 0  # (no fold: apply now, fp32)
            if planes == 4:
                # the reader (the next BN, as its residual) applies it (DeferredRes)
                coef, mean, rstd = be.bn_coef(x3, gamma, beta, valid_rows, pre_stats=pre)
                y = torch.empty((K, x3.shape[1], C), dtype=x.dtype, device=x.device)
                fold_out = DeferredRes(x3, coef, valid_rows, y)
                defer = None
                planes = 0
            elif planes == 3:
                # deferred apply (DeferredBN): statistics + coefficients now; the consuming 3x3 conv
                # applies them in its halo loader, or materialises the planes / ReLU bits first
                coef, mean, rstd = be.bn_coef(x3, gamma, beta, valid_rows, pre_stats=pre)
                y, yp = be.planes_buffer((K, x3.shape[1], C), x.device)
                mask = torch.empty((K, x3.shape[1], C // 8), dtype=torch.uint8, device=x.device) if (wm and relu) else None
                defer = DeferredBN(x3, coef, relu, valid_rows, yp, mask, write_out=wm)
            else:
                defer = None
                out = be.bn_fwd(x3, gamma, beta, valid_rows, relu, r3, with_mask=wm, pre_stats=pre, planes=planes,
                                res_coef=res_coef)
                y, mean, rstd = out[:3]
                mask = out[3] if wm else None
                if planes:
                    yp = out[-1]
            if stats is not None:
                stats.part = None
            if (wm and OPTIONS.bn_bwd_parts and x.dtype == torch.float32 and x3.is_contiguous()
                    and (mask is not None or not relu)):
                vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
                bnb = BNBwdLink(x3, mask, mean, rstd, vr)
        # (y itself is only read by the backward when there is no ReLU mask)
        ctx.save_for_backward(x3, y if mask is None else None, mean, rstd, gamma)
        ctx.relu_mask = mask
        ctx.valid_rows, ctx.relu, ctx.has_res = valid_rows, relu, residual is not None
        ctx.link = link
        ctx.stats = stats
        ctx.ggamma, ctx.gbeta, ctx.shape = ggamma, gbeta, x.shape
        ctx.bnb = bnb
        ctx.planes_on = OPTIONS.planes  # (the backward's dX-planes decision follows the forward's)
        ctx.bwd_in_wgrad = OPTIONS.bn_bwd_in_wgrad
        yo = y.reshape(x.shape)
        if yp is not None:
            _tag_planes(yo, yp.view((K, 2) + tuple(x.shape[1:])), planes >= 2)
        ctx.defer = None
        if be is not ref and planes == 3:
            yo._dls_bn_defer = ctx.defer = defer
        if fold_out is not None:
            yo._dls_res_fold = fold_out
        if bnb is not None:
            yo._dls_bnb = bnb
        return yo

    @staticmethod
    def backward(ctx, dy):
        x3, y, mean, rstd, gamma = ctx.saved_tensors
        be = _be(dy)
        K, R, C = x3.shape
        if ctx.defer is not None:  # (a consumer that never ran: the ReLU bits must exist now)
            ctx.defer.materialize()
            ctx.defer = None
        dy3 = dy.reshape(K, R, C).contiguous()
        if be is ref:
            dx, dgamma, dbeta, dpre = ref.bn_bwd(dy3, x3, y, mean, rstd, gamma, ctx.valid_rows, ctx.relu)
            if ctx.ggamma is not None:
                ctx.ggamma.copy_(dgamma)
                ctx.gbeta.copy_(dbeta)
        else:
            _require_fp32(dy, "batch_norm backward")
            # the producing conv reads dX as split planes: write only those
            dxm = 2 if (ctx.stats is not None and ctx.stats.dy_planes_ok and ctx.planes_on) else 0
            # partial sums from the consuming conv's dgrad epilogue, if dy is exactly its output
            pre = None
            bnb = ctx.bnb
            if bnb is not None:
                if bnb.part is not None and bnb.key == (dy3.data_ptr(), dy3._version):
                    pre = bnb.part
                bn_bwd_parts_count["used" if pre is not None else "none" if bnb.part is None else "fallback"] += 1
                bnb.part = bnb.key = None
            # identity shortcut (ResidualLink): its gradient dy·relu' goes to the block's first conv
            # as factors (MaskedGrad) — the backward writes no dpre tensor
            masked = (ctx.has_res and ctx.link is not None and ctx.relu and ctx.relu_mask is not None
                      and C % 8 == 0)
            if (dxm == 2 and ctx.bwd_in_wgrad and not (ctx.has_res and not masked) and C % 64 == 0
                    and (ctx.relu_mask is not None or not ctx.relu) and x3.is_contiguous()):
                # coefficients only: the producing conv's halo weight gradient applies them in its
                # dY loader and writes dX's planes (DeferredBNBwd), or materialize() does
                coef = torch.empty((K, C, 3), dtype=torch.float32, device=dy3.device)
                be.bn_bwd(dy3, x3, y, mean, rstd, gamma, ctx.valid_rows, ctx.relu, ctx.ggamma, ctx.gbeta, False,
                          relu_mask=ctx.relu_mask, pre_part=pre, coef_out=coef)
                dx, dxp = be.planes_buffer((K, R, C), dy3.device)
                if masked:
                    ctx.link.grad = MaskedGrad(dy3.view(ctx.shape), ctx.relu_mask)
                dxo = dx.reshape(ctx.shape)
                _tag_planes(dxo, dxp.view((K, 2) + tuple(ctx.shape[1:])), True)
                dxo._dls_bnbwd = DeferredBNBwd(dy3, x3, ctx.relu_mask if ctx.relu else None, coef, ctx.valid_rows,
                                               dxp)
                return dxo, None, None, None, None, None, None, None, None, None, None, None
            out = be.bn_bwd(dy3, x3, y, mean, rstd, gamma, ctx.valid_rows, ctx.relu,
                            ctx.ggamma, ctx.gbeta, ctx.has_res and not masked, relu_mask=ctx.relu_mask,
                            dx_planes=dxm, pre_part=pre)
            dx, dpre = out[0], out[1]
            if masked:
                ctx.link.grad = MaskedGrad(dy3.view(ctx.shape), ctx.relu_mask)
            if dxm:
                dxo = dx.reshape(ctx.shape)
                _tag_planes(dxo, out[2].view((K, 2) + tuple(ctx.shape[1:])), True)
                dres = dpre.reshape(ctx.shape) if (ctx.has_res and not masked) else None
                if dres is not None and ctx.link is not None:
                    ctx.link.grad = dres
                    dres = None
                return dxo, None, None, None, None, None, None, None, dres, None, None, None
            if masked:
                return dx.reshape(ctx.shape), None, None, None, None, None, None, None, None, None, None, None
        dres = dpre.reshape(ctx.shape) if ctx.has_res else None
        if dres is not None and ctx.link is not None:
            ctx.link.grad = dres  # delivered by the block's first conv (ResidualLink)
            dres = None
        dxo = dx.reshape(ctx.shape)
        if be is not ref:
            dxo._dls_owned = True  # (freshly written, read by nothing else: a consumer may reuse it in place)
        return dxo, None, None, None, None, None, None, None, dres, None, None, None


def batch_norm(x, token, gamma, beta, ggamma, gbeta, valid_rows=None, relu=False, residual=None,
               link: ResidualLink | None = None, stats: BNStats | None = None, planes: int = 0):
    """`planes` (fp32 native): 1 = the output also carries its split planes (`_dls_planes`) for
    the conv(s) that read it, 2 = the output is ONLY planes — for outputs read by nothing but
    split-plane convs (e.g. a ResNet block's inner BN), 3 = as 2 with the apply pass deferred to
    the ONE conv that reads it (DeferredBN: a 3x3 stride-1 halo conv applies it while staging);
    4 (no ReLU): the output's one reader is the next BatchNorm, as its residual, which folds this
    apply into its own (DeferredRes: a ResNet downsample shortcut)."""
    return _BN.apply(x, token, gamma, beta, ggamma, gbeta, valid_rows, relu, residual, link, stats, planes)


# ------------------------------------------------------------------------ layernorm
class _LN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, token, gamma, beta, ggamma, gbeta, planes=False):
        be = _be(x)
        yp = None
        if (planes and OPTIONS.planes and be is not ref and x.dtype == torch.float32
                and be.planes_fit(x[0].numel())):
            y, mean, rstd, yp = be.ln_fwd(x, gamma, beta, planes=True)
        else:
            y, mean, rstd = be.ln_fwd(x, gamma, beta)
        ctx.save_for_backward(x, mean, rstd, gamma)
        ctx.ggamma, ctx.gbeta = ggamma, gbeta
        if yp is not None:
            _tag_planes(y, yp, False)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, gamma = ctx.saved_tensors
        be = _be(dy)
        dx, dgamma, dbeta = be.ln_bwd(dy.contiguous(), x, mean, rstd, gamma)
        if ctx.ggamma is not None:
            ctx.ggamma.copy_(dgamma)
            ctx.gbeta.copy_(dbeta)
        return dx, None, None, None, None, None, None


def layer_norm(x, token, gamma, beta, ggamma, gbeta, planes: bool = False):
    """`planes` (fp32 native): the output also carries its split planes (`_dls_planes`) for the
    split-plane linears that read it (Fn.linear)."""
    return _LN.apply(x, token, gamma, beta, ggamma, gbeta, planes)


# -------------------------------------------------------------------------- pooling
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        be = _be(x)
        y, idx = be.maxpool_fwd(x, k, s, pad)
        ctx.save_for_backward(idx)
        ctx.k, ctx.s, ctx.pad, ctx.xshape = k, s, pad, x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        be = _be(dy)
        dx = be.maxpool_bwd(dy.contiguous(), idx, ctx.xshape, ctx.k, ctx.s, ctx.pad)
        return dx, None, None, None


def max_pool2d(x, k, s=None, pad=0):
    return _MaxPool.apply(x, k, s or k, pad)


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s):
        ctx.k, ctx.s, ctx.xshape = k, s, x.shape
        return _be(x).avgpool_fwd(x, k, s)

    @staticmethod
    def backward(ctx, dy):
        return _be(dy).avgpool_bwd(dy.contiguous(), ctx.xshape, ctx.k, ctx.s), None, None


def avg_pool2d(x, k, s=None):
    return _AvgPool.apply(x, k, s or k)


class _GAP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.xshape = x.shape
        return _be(x).gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return _be(dy).gap_bwd(dy.contiguous(), ctx.xshape)


def global_avg_pool(x):
    return _GAP.apply(x)


# -------------------------------------------------------------------- cross entropy
class _CE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, valid):
        loss, correct, dlogits = _be(logits).ce_fwd_bwd(logits, labels, valid)
        ctx.save_for_backward(dlogits)
        ctx.mark_non_differentiable(correct)
        return loss, correct

    @staticmethod
    def backward(ctx, dloss, dcorrect):
        (dlogits,) = ctx.saved_tensors
        if dloss is None:
            return None, None, None
        g = dlogits * dloss.to(dlogits.dtype)[:, None, None]
        return g, None, None


def cross_entropy(logits, labels, valid=None):
    """Per-client mean CE [K] and correct counts [K] (fused fwd+bwd kernel)."""
    return _CE.apply(logits, labels, valid)


# ------------------------------------------------------------------------ embedding
class _Emb(torch.autograd.Function):
    """Embedding lookup × scale (+ positional encoding) in one kernel (Transformer input:
    emb·√d + PE, reference TransformerClassificationModel)."""

    @staticmethod
    def forward(ctx, tokens, token, table, gtable, scale=1.0, pe=None):
        ctx.save_for_backward(tokens)
        ctx.gtable, ctx.vocab, ctx.scale = gtable, table.shape[1], scale
        return _be(table).embedding_fwd(tokens, table, scale, pe)

    @staticmethod
    def backward(ctx, dy):
        (tokens,) = ctx.saved_tensors
        if ctx.gtable is not None:
            be = _be(dy)
            if be is ref:
                ctx.gtable.copy_(ref.embedding_bwd(dy, tokens, ctx.vocab, ctx.scale))
            else:
                be.embedding_bwd(dy.contiguous(), tokens, ctx.gtable, ctx.scale)
        return None, None, None, None, None, None


def embedding(tokens, token, table, gtable, scale: float = 1.0, pe=None):
    return _Emb.apply(tokens, token, table, gtable, scale, pe)


class _SeqMean(torch.autograd.Function):
    """Masked mean over the sequence axis (the classifier's pooling of valid tokens)."""

    @staticmethod
    def forward(ctx, x, lengths):
        ctx.save_for_backward(lengths)
        ctx.L = x.shape[-2]
        return _be(x).seq_mean_fwd(x, lengths)

    @staticmethod
    def backward(ctx, dy):
        (lengths,) = ctx.saved_tensors
        return _be(dy).seq_mean_bwd(dy.contiguous(), lengths, ctx.L), None


def seq_mean(x, lengths):
    return _SeqMean.apply(x, lengths)


# ------------------------------------------------------------------------ attention
class _Attn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, key_valid, drop_p=0.0, drop_seeds=None):
        dr = {"drop_p": drop_p, "drop_seeds": drop_seeds} if drop_p else {}
        o, lse = _be(q).attn_fwd(q, k, v, key_valid, **dr)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.key_valid, ctx.dr = key_valid, dr
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = _be(do).attn_bwd(do.contiguous(), q, k, v, o, lse, ctx.key_valid, **ctx.dr)
        return dq, dk, dv, None, None, None


def attention(q, k, v, key_valid=None, drop_p: float = 0.0, drop_seeds=None):
    """Softmax attention over [K, B, H, L, dh]; `drop_p` / `drop_seeds` [K]: dropout on the
    attention probabilities (hash mask per client, head, query, key — ops/ref.py attn_drop_scale)."""
    return _Attn.apply(q, k, v, key_valid, drop_p, drop_seeds)


class _AttnPacked(torch.autograd.Function):
    """Attention on the QKV projection's own output rows qkv [K, B, L, 3·D] → o [K, B, L, D]
    (the out projection's input layout); backward returns dqkv in the QKV layout. On the GPU the
    MFMA kernels read / write the heads in place (no permute copies either way)."""

    @staticmethod
    def forward(ctx, qkv, key_valid, H, drop_p=0.0, drop_seeds=None):
        be = _be(qkv)
        K, B, L, D3 = qkv.shape
        D = D3 // 3
        dr = {"drop_p": drop_p, "drop_seeds": drop_seeds} if drop_p else {}
        if be is ref:
            t = qkv.reshape(K, B, L, 3, H, D // H).permute(3, 0, 1, 4, 2, 5)
            o, lse = ref.attn_fwd(t[0], t[1], t[2], key_valid, **dr)
            o = o.permute(0, 1, 3, 2, 4).reshape(K, B, L, D)
        else:
            o, lse = be.attn_fwd_packed(qkv, H, key_valid, **dr)
        ctx.save_for_backward(qkv, o, lse)
        ctx.key_valid, ctx.H, ctx.dr = key_valid, H, dr
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        be = _be(do)
        H = ctx.H
        K, B, L, D3 = qkv.shape
        D = D3 // 3
        if be is ref:
            t = qkv.reshape(K, B, L, 3, H, D // H).permute(3, 0, 1, 4, 2, 5)
            op = o.reshape(K, B, L, H, D // H).permute(0, 1, 3, 2, 4)
            dop = do.reshape(K, B, L, H, D // H).permute(0, 1, 3, 2, 4)
            dq, dk, dv = ref.attn_bwd(dop, t[0], t[1], t[2], op, lse, ctx.key_valid, **ctx.dr)
            dqkv = torch.stack([dq, dk, dv]).permute(1, 2, 4, 0, 3, 5).reshape(K, B, L, D3)
        else:
            dqkv = be.attn_bwd_packed(do.contiguous(), qkv, o, lse, H, ctx.key_valid, **ctx.dr)
        return dqkv, None, None, None, None


def attention_packed(qkv, key_valid, H: int, drop_p: float = 0.0, drop_seeds=None):
    """Attention over the QKV projection's packed rows (no permute copies; MFMA kernels)."""
    return _AttnPacked.apply(qkv, key_valid, H, drop_p, drop_seeds)


def packed_attention_ok(t: torch.Tensor, L: int, DH: int) -> bool:
    """Whether the packed (copy-free) attention path runs for this device / shape."""
    if not backend.using_hip(t):
        return True
    from . import hip

    return hip.attn_packed_supported(L, DH)


# ---------------------------------------------------------------------------- spmm
class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rowptr, col, val, rowptr_t, col_t, val_t):
        ctx.save_for_backward(rowptr_t, col_t, val_t)
        return _be(x).spmm(rowptr, col, val, x)

    @staticmethod
    def backward(ctx, dy):
        rowptr_t, col_t, val_t = ctx.saved_tensors
        return _be(dy).spmm(rowptr_t, col_t, val_t, dy.contiguous()), None, None, None, None, None, None


def spmm(x, graph):
    """A @ x for a shared normalised adjacency `graph` (CSR + its transpose)."""
    return _SpMM.apply(x, graph.rowptr, graph.col, graph.val, graph.rowptr_t, graph.col_t, graph.val_t)


# ---------------------------------------------------------------------- dense block
dense_grad_reuse = collections.Counter()  # (tests: how often _DenseBlock.backward reused dF_out in place)


class DenseLayerParams:
    """One DenseNet layer's parameter views: BN (γ, β and their grads) + 3x3 conv (w, grad)."""

    __slots__ = ("gamma", "beta", "ggamma", "gbeta", "w", "gw")

    def __init__(self, gamma, beta, ggamma, gbeta, w, gw):
        self.gamma, self.beta, self.ggamma, self.gbeta, self.w, self.gw = gamma, beta, ggamma, gbeta, w, gw


class _DenseBlock(torch.autograd.Function):
    """A whole DenseNet block (L × [BN-ReLU-Conv3x3, concat]) over ONE preallocated feature
    buffer F [K, B, H, W, c0 + L·g]: layer i's BN reads the channel prefix F[..., :c_i] in place
    (channel-strided kernels) and its conv writes the g new channels straight into
    F[..., c_i : c_i + g] through the epilogue's row stride — no per-layer `torch.cat` (which
    re-copies the growing prefix every layer: Σ c_i channel-copies per block). The backward walks
    the layers in reverse over one gradient buffer dF: layer i's conv dgrad reads its slice of dF
    in place and the BN backward ADDS its input gradient into dF[..., :c_i].
    Reference: torchvision-style `_DenseLayer` + `torch.cat` (the cyy_torch_vision densenet40,
    SURVEY §2.7), BN with batch statistics (`util/model.py:23`)."""

    @staticmethod
    def forward(ctx, x, token, layers, growth, valid_rows, training=True):
        be = _be(x)
        K, B, H, W, c0 = x.shape
        L = len(layers)
        Ct = c0 + L * growth
        F = torch.empty((K, B, H, W, Ct), dtype=x.dtype, device=x.device)
        F[..., :c0].copy_(x)
        native = be is not ref
        saved = []
        halo = native and x.dtype == torch.float32 and OPTIONS.dense_bn_halo
        # Per-channel batch statistics are the same for every later layer that normalises a
        # channel (only γ/β differ), so with the fused growth convs they can be summed ONCE per
        # channel (OPTIONS.dense_stats_cache): the block input's in one pass, each new slice's from
        # its conv's epilogue partials — running fp64 sums S [K, 2, Ct] that the coefficient kernel
        # reads for the prefix — instead of a statistics pass over the whole growing prefix in every
        # layer (O(L²) → O(L) bytes).
        cache = halo and OPTIONS.dense_stats_cache and all(
            be.halo_bn_dense_ok(F[..., : c0 + i * growth], lp.w) for i, lp in enumerate(layers))
        R = B * H * W
        if cache:
            S = torch.zeros((K, 2, Ct), dtype=torch.float64, device=x.device)
            x3 = F[..., :c0].reshape(K, R, c0)
            if 2 * c0 <= 1024:  # (the fixed-order fp64 kernel's column limit)
                be.chan_sums_f64(x3, valid_rows, S[:, :, :c0])
            else:
                if valid_rows is not None:
                    keep = (torch.arange(R, device=x.device).view(1, R) < valid_rows.view(K, 1)).unsqueeze(-1)
                    x3 = torch.where(keep, x3, torch.zeros((), dtype=x3.dtype, device=x.device))
                S[:, 0, :c0] = x3.sum(dim=1, dtype=torch.float64)
                S[:, 1, :c0] = (x3.double() * x3.double()).sum(dim=1)
            samples = valid_rows // (H * W) if valid_rows is not None else None
        for i, lp in enumerate(layers):
            ci = c0 + i * growth
            xi = F[..., :ci].reshape(K, -1, ci)
            halo_i = native and halo and be.halo_bn_dense_ok(F[..., :ci], lp.w)
            if halo_i:
                # BN + ReLU applied in the growth conv's halo loader (csrc/conv_halo.hip BNM 2): the
                # prefix is read in place once per 32-channel chunk for all nine taps; the normalised
                # activation is written only in training (the weight gradient and BN backward read it)
                part = None
                if cache:
                    coef, mean, rstd = be.bn_coef_sums(S, ci, lp.gamma, lp.beta, R, valid_rows)
                    part = torch.empty((K, be.conv_stats_parts(R), 2, growth), dtype=torch.float32, device=x.device)
                else:
                    coef, mean, rstd = be.bn_coef(xi, lp.gamma, lp.beta, valid_rows)
                # the normalised activation is stored for the backward only if a reader needs it: the
                # fused dgrad and the recomputing weight gradient rebuild it from x and coef
                need_y = training and not (
                    OPTIONS.dense_y_recompute and OPTIONS.dense_dgrad_fused and OPTIONS.dense_wgrad_halo
                    and be.dense_recompute_ok(B, H, W, ci, growth, lp.ggamma is not None))
                y = torch.empty((K, B * H * W, ci), dtype=x.dtype, device=x.device) if need_y else None
                # ReLU bits for the backward where whole bytes fit (ci % 8 == 0; otherwise it gates on y)
                # — not with the fused dgrad, which recomputes the gate from x and coef
                mask = (torch.empty((K, B * H * W, ci // 8), dtype=torch.uint8, device=x.device)
                        if training and ci % 8 == 0 and not OPTIONS.dense_dgrad_fused else None)
                ok = be.conv_halo_bn_dense_fwd(F[..., :ci], coef, True, valid_rows, lp.w, F[..., ci : ci + growth],
                                               stats=part, stats_valid=samples if cache else None, ny=y, mask=mask)
                assert ok, "dense halo conv refused a shape halo_bn_dense_ok accepted"
                if cache:
                    be.part_sum_f64(part, S[:, :, ci : ci + growth])
            elif native:
                y, mean, rstd, mask = be.bn_fwd(xi, lp.gamma, lp.beta, valid_rows, True, None, with_mask=True)
                be.conv_fwd(y.view(K, B, H, W, ci), lp.w, 1, 1, out=F[..., ci : ci + growth])
            else:
                y, mean, rstd = ref.bn_fwd(xi, lp.gamma, lp.beta, valid_rows, True, None)
                mask = None
                F[..., ci : ci + growth].copy_(ref.conv_fwd(y.view(K, B, H, W, ci), lp.w, 1, 1))
            # (the halo path's BN (scale, shift) also rides along: the fused dgrad recomputes the
            # ReLU gate from x with it instead of reading the bits / y)
            saved.append((y, mean, rstd, mask, coef if native and halo_i else None))
        ctx.save_for_backward(F)
        ctx.saved = saved
        ctx.wgrad_halo = OPTIONS.dense_wgrad_halo  # (the backward follows the forward's options)
        ctx.dgrad_fused = OPTIONS.dense_dgrad_fused
        ctx.layers, ctx.growth, ctx.valid_rows, ctx.c0 = layers, growth, valid_rows, c0
        return F

    @staticmethod
    def backward(ctx, dF_out):
        (F,) = ctx.saved_tensors
        be = _be(dF_out)
        native = be is not ref
        K, B, H, W, Ct = F.shape
        g, c0 = ctx.growth, ctx.c0
        # the block's gradient buffer: the incoming gradient itself when it is a BatchNorm backward's
        # fresh output (the transition / final BN: dF_out's only reader is this backward), else a copy
        if native and getattr(dF_out, "_dls_owned", False) and dF_out.is_contiguous():
            dF = dF_out
            dense_grad_reuse["reused"] += 1
        else:
            dF = dF_out.contiguous().clone() if native else dF_out.float().clone()
            dense_grad_reuse["cloned"] += 1
        wgrad_halo = native and F.dtype == torch.float32 and ctx.wgrad_halo
        # growth-conv input gradient + BN backward in one recomputing kernel pair (dX̂ never stored)
        dense_dgrad = native and F.dtype == torch.float32 and ctx.dgrad_fused
        for i in range(len(ctx.layers) - 1, -1, -1):
            lp = ctx.layers[i]
            y, mean, rstd, mask, bn_sc = ctx.saved[i]
            ci = c0 + i * g
            d_out = dF[..., ci : ci + g]
            yv = y.view(K, B, H, W, ci) if y is not None else None
            xi = F[..., :ci].reshape(K, -1, ci)
            if native:
                if y is None:  # (the forward stored no normalised activation: recompute it from x)
                    assert bn_sc is not None and wgrad_halo and dense_dgrad
                    if lp.gw is not None:
                        ok = be.dense_wgrad(d_out, None, lp.gw, x=F[..., :ci], bn_coef=bn_sc, valid_rows=ctx.valid_rows)
                        assert ok, "dense_wgrad refused a shape dense_recompute_ok accepted"
                elif lp.gw is not None and not (wgrad_halo and be.dense_wgrad(d_out, y, lp.gw)):
                    be.conv_wgrad(d_out, yv, lp.gw, 1, 1)
                if y is None:
                    ok = be.dense_dgrad_bn(d_out, lp.w, F[..., :ci], dF[..., :ci], None, None, mean, rstd, lp.gamma,
                                           ctx.valid_rows, lp.ggamma, lp.gbeta, bn_coef=bn_sc)
                    assert ok, "dense_dgrad_bn refused a shape dense_recompute_ok accepted"
                    continue
                if (dense_dgrad and lp.ggamma is not None
                        and be.dense_dgrad_bn(d_out, lp.w, F[..., :ci], dF[..., :ci], y, mask, mean, rstd, lp.gamma,
                                              ctx.valid_rows, lp.ggamma, lp.gbeta, bn_coef=bn_sc)):
                    continue
                # (BN partials from this dgrad's epilogue measured slower here: 14.57 vs 14.36 s per
                # 100-client round — the strided x / gate reads cost more than the pass they replace)
                dy = be.conv_dgrad(d_out, lp.w, (H, W), 1, 1)
                be.bn_bwd(dy.view(K, -1, ci), xi, y, mean, rstd, lp.gamma, ctx.valid_rows, True, lp.ggamma, lp.gbeta,
                          False, relu_mask=mask, dx_out=dF[..., :ci].reshape(K, -1, ci))
            else:
                d_out = d_out.contiguous()
                if lp.gw is not None:
                    lp.gw.copy_(ref.conv_wgrad(d_out.float(), yv.float(), (K,) + tuple(lp.w.shape[1:]), 1, 1))
                dy = ref.conv_dgrad(d_out, lp.w.to(d_out.dtype), (H, W), 1, 1)
                dx, dgamma, dbeta, _ = ref.bn_bwd(dy.view(K, -1, ci), xi, y, mean, rstd, lp.gamma, ctx.valid_rows, True)
                if lp.ggamma is not None:
                    lp.ggamma.copy_(dgamma)
                    lp.gbeta.copy_(dbeta)
                dF[..., :ci] += dx.view(K, B, H, W, ci).to(dF.dtype)
        ctx.saved = None
        return dF[..., :c0].contiguous().to(dF_out.dtype), None, None, None, None, None


def dense_block(x, token, layers: list[DenseLayerParams], growth: int, valid_rows=None, training: bool = True):
    """All layers of a DenseNet block in one buffer (see _DenseBlock). `training=False`: no
    backward will run, so the normalised activations are not kept."""
    return _DenseBlock.apply(x, token, layers, growth, valid_rows, training)
