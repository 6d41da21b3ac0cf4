"""Host wrappers of the gfx950 kernels (`_dls_hip`), same API as `ops.ref`.

Importing this module on a machine with a GPU but without the built extension raises — the
GPU path never silently falls back to PyTorch. Shape/stride contracts are asserted here
before any launch (a mis-shaped launch on the box can fault the GPU).
"""

from __future__ import annotations

import collections
import importlib
import os
import threading

import torch

from ..options import OPTIONS
from . import ref

try:
    _C = importlib.import_module("distributed_learning_simulator_amd._dls_hip")
except ImportError as e:  # pragma: no cover - exercised only on a GPU box without a build
    raise ImportError(
        "HIP extension _dls_hip is not built; run `python -m distributed_learning_simulator_amd.ops.build` "
        f"(original error: {e})"
    ) from e


def _check_provenance() -> None:
    """The loaded binary must have been linked from the csrc/ sources in this tree (its
    compiled-in content hash, ops/build.source_hash): a stale or foreign .so fails loudly."""
    from . import build as _build

    built, here = _C.src_hash(), _build.source_hash()
    if built != here and os.environ.get("DLS_SKIP_SRC_HASH") != "1":
        raise ImportError(f"_dls_hip was built from different sources (binary {built}, tree {here}); "
                          "rebuild with `python -m distributed_learning_simulator_amd.ops.build`")


_check_provenance()

BF16 = torch.bfloat16
F32 = torch.float32
NULL = 0
_DTYPES = (BF16, F32)


def _f32(t: torch.Tensor) -> int:
    """Kernel element-type flag of an activation tensor: bf16 (fast mode) or fp32 (reference
    precision: the GEMMs then run as split-bf16 MFMA, csrc/conv_f32.hip)."""
    assert t.dtype in _DTYPES, f"unsupported activation dtype {t.dtype}"
    return int(t.dtype == F32)


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


_tls = threading.local()  # per thread: concurrent training tasks build launches in parallel


def _p(t) -> int:
    """Device pointer of t. The tensor is kept referenced until well after the launch that
    consumes the pointer: an inline temporary (`_p(x.to(...))`) would otherwise be freed
    while the argument list is still being built and a second temporary in the same call
    could be allocated at the same address. After the launch, the caching allocator's
    stream ordering makes reuse safe. (The keep-alive ring is per thread, so another task
    thread's launches cannot push this launch's temporaries out early.)"""
    if t is None:
        return 0
    ring = getattr(_tls, "keepalive", None)
    if ring is None:
        ring = _tls.keepalive = collections.deque(maxlen=48)  # > pointer args of any one launch
    ring.append(t)
    return t.data_ptr()


def _client_view(w: torch.Tensor, K: int):
    """(client stride, rep) of a [Kw, ...] parameter view with contiguous inner dims."""
    Kw = w.shape[0]
    inner = w[0]
    assert inner.is_contiguous(), "parameter inner dims must be contiguous"
    assert K % Kw == 0, (K, Kw)
    return (w.stride(0) if Kw > 1 else 0), K // Kw


def _check(t: torch.Tensor, dtype=None, contiguous=True, name="tensor"):
    assert t.is_cuda, f"{name} must be on the GPU"
    if dtype is not None:
        assert t.dtype == dtype, f"{name}: expected {dtype}, got {t.dtype}"
    if contiguous:
        assert t.is_contiguous(), f"{name} must be contiguous"


def _pix_stride(t: torch.Tensor):
    """(t, pixel/row stride) of a [K, ..., C] tensor. A channel slice of a wider contiguous
    buffer (DenseNet's block buffer F[..., a:b]) keeps one uniform stride between consecutive
    pixels: it is passed to the kernels as is (stride ld ≥ C, client stride t.stride(0));
    anything else is made contiguous (ld = C)."""
    C = t.shape[-1]
    if t.is_contiguous():
        return t, C
    if t.stride(-1) != 1 or t.dim() < 3:
        return t.contiguous(), C
    ld = t.stride(-2)
    expect = ld
    for d in range(t.dim() - 2, 0, -1):
        if t.shape[d] != 1 and t.stride(d) != expect:
            return t.contiguous(), C
        expect *= t.shape[d]
    return t, ld


_ws_cache: dict = {}
# Buffers a growing cache replaced. A captured step graph (engine/trainer.py keeps up to
# OPTIONS.max_graphs, keyed by cohort size) holds the pointer it was captured with: when a later
# warm-up of a larger graph grows the cache, the older graph must still find its buffer mapped on
# replay, so superseded buffers stay referenced here (they grow a handful of times per process).
_retired: list = []


def _grown(cache: dict, key, numel: int, device) -> torch.Tensor:
    """cache[key], replaced by a ≥ numel-float buffer when too small (the old one is retired, not
    freed). Per (device, stream) keys: sub-cohorts on concurrent streams never share one."""
    t = cache.get(key)
    if t is None or t.numel() < numel:
        if t is not None:
            _retired.append(t)
        t = torch.empty(max(numel, 1 << 16), dtype=torch.float32, device=device)
        cache[key] = t
    return t


def _workspace(numel: int, device) -> torch.Tensor:
    key = (device, torch.cuda.current_stream().cuda_stream if torch.cuda.is_available() else 0)
    return _grown(_ws_cache, key, numel, device)


# ----------------------------------------------------------------------------- conv
# NT-GEMM tile configuration: -1 = per-shape heuristic (csrc/conv_nt.hip); the kernel
# microbenchmark (bench/kernel_bench.py) sets explicit variant ids to sweep them.
nt_variant = -1
tn_variant = -1  # weight-gradient (TN) tile configuration, same convention
nt_f32_variant = -1  # the same for the fp32 (split-bf16) kernels of csrc/conv_f32.hip
tn_f32_variant = -1
# large-tile LDS-DMA kernel (csrc/conv_gl.hip) for fwd / dgrad: -1 = shape heuristic (or env
# DLS_CONV_GL), 0 = never, 1 = whenever the shape is supported (tests, A/B benchmarks)
gl_mode = -1


def _gl(K: int, M: int, N: int, C: int, taps: int) -> bool:
    mode = gl_mode if nt_variant < 0 else 0  # an explicit NT variant (sweeps) bypasses it
    return bool(_C.conv_gl_wanted(K, M, N, C, taps, mode))


def conv_stats_parts(M: int) -> int:
    """Partial-sum rows per client of the conv-epilogue BN statistics (one per 32 GEMM rows)."""
    return (M + 31) // 32


# launches that took the split-plane GEMM path (fwd / dgrad / wgrad), for tests and reports
planes_launches = collections.Counter()


def planes_ok(C: int, N: int, ld: int | None = None) -> bool:
    """Shape contract of the pre-split-operand GEMMs (csrc/conv_pl.hip): a K tile of 32 never
    straddles a tap (C % 32), contiguous planes, 16-B output columns (N % 8)."""
    return C % 32 == 0 and N % 8 == 0 and (ld is None or ld == C)


WINDOW = 1 << 31  # the GEMM loaders address one client's operand window with 32-bit byte offsets


def planes_fit(numel_per_client: int) -> bool:
    """A [K, 2, n] plane buffer fits the kernels' per-client window (hi plane + lo plane)."""
    return numel_per_client * 4 < WINDOW


def _batch_chunks(B: int, bytes_per_sample: int) -> list[tuple[int, int]]:
    """Split a per-client batch so each chunk's operand window stays under 2 GiB (ADVICE r2:
    the launchers used to abort on larger windows, e.g. ResNet-50 at 224² with batch ≥ 640)."""
    per = max(1, (WINDOW - 1) // max(1, bytes_per_sample))
    return [(b, min(B, b + per)) for b in range(0, B, per)]


def conv_planes_ok(C: int, Co: int, ldx: int | None = None) -> bool:
    """A conv with C input / Co output channels can run all three GEMMs on split planes:
    forward (A = x planes, C % 32), dgrad (A = dY planes, Co % 32; output Ci % 8), wgrad."""
    return planes_ok(C, Co, ldx) and planes_ok(Co, C)


def split_planes(x, out=None):
    """[K, 2, *x.shape[1:]] bf16 (hi, lo) planes of a contiguous fp32 activation x:
    hi = bf16(x), lo = bf16(x − hi) (RNE), the operand form of the conv_pl.hip GEMMs."""
    assert x.dtype == F32 and x.is_contiguous()
    K = x.shape[0]
    if out is None:
        out = torch.empty((K, 2) + tuple(x.shape[1:]), dtype=BF16, device=x.device)
    assert out.shape == (K, 2) + tuple(x.shape[1:]) and out.dtype == BF16 and out.is_contiguous()
    split_rows(x.view(K, -1), out.view(K, 2, -1))
    return out


def _planes_args(planes, t):
    """(hi-plane pointer, client stride, hi→lo distance) of [K, 2, ...] planes of tensor t."""
    assert planes.dtype == BF16 and planes.is_contiguous(), "planes must be contiguous bf16"
    assert planes.shape == (t.shape[0], 2) + tuple(t.shape[1:]), (planes.shape, t.shape)
    assert planes.stride(1) * 4 < 2 ** 31, "per-client plane window over 2 GiB"
    return _p(planes), planes.stride(0), planes.stride(1)


def conv_fwd(x, w, stride: int, pad: int, bias=None, relu=False, out=None, stats=None, stats_valid=None,
             w_split=None, x_planes=None):
    """`x` may be a channel slice of a wider buffer, `out` (optional) a channel slice to write
    into (DenseNet block buffer): both are read / written in place through channel strides.
    `stats` (fp32 only): a [K, conv_stats_parts(M), 2, Co] fp32 buffer the epilogue fills with the
    BN partial sums Σy, Σy² over the rows of the first `stats_valid[k]` samples (bn_fwd(pre_stats=))."""
    K, B, H, W, C = x.shape
    Kw, Co, KH, KW, Ci = w.shape
    OHs, OWs = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    per_sample = max(H * W * (x.stride(-2) if x.dim() == 5 else C), OHs * OWs * Co) * x.element_size()
    if B * per_sample >= WINDOW and stats is None and x_planes is None:
        chunks = _batch_chunks(B, per_sample)
        if out is None:
            out = torch.empty((K, B, OHs, OWs, Co), dtype=x.dtype, device=x.device)
        for b0, b1 in chunks:
            conv_fwd(x[:, b0:b1], w, stride, pad, bias=bias, relu=relu, out=out[:, b0:b1], w_split=w_split)
        return out
    x, ldx = _pix_stride(x)
    f32 = _f32(x)
    _check(x, x.dtype, contiguous=False, name="x")
    _check(w, x.dtype, contiguous=False, name="w")
    assert Ci == C, (Ci, C)
    w_cs, rep = _client_view(w, K)
    OH = (H + 2 * pad - KH) // stride + 1
    OW = (W + 2 * pad - KW) // stride + 1
    if out is None:
        y, ldy = torch.empty((K, B, OH, OW, Co), dtype=x.dtype, device=x.device), Co
    else:
        assert out.shape == (K, B, OH, OW, Co) and out.dtype == x.dtype
        y, ldy = _pix_stride(out)
        assert y.data_ptr() == out.data_ptr(), "out must be a row-strided view"
    b_cs = 0
    if bias is not None:
        assert bias.dtype == x.dtype
        b_cs, _ = _client_view(bias, K)
    M = B * OH * OW
    if stats is not None:
        assert f32 and stats.dtype == torch.float32 and stats.is_contiguous()
        assert stats.shape == (K, conv_stats_parts(M), 2, Co), stats.shape
        if stats_valid is not None:
            stats_valid = stats_valid.to(torch.int32).contiguous()
            assert stats_valid.shape == (K,)
    if not f32 and ldx == C and ldy == Co and _gl(K, M, Co, C, KH * KW):
        _C.conv_gl_fwd(_p(x), _p(w), _p(y), _p(bias), B * H * W * C, M * Co, w_cs, b_cs, K, rep, B, H, W, C, OH, OW,
                       KH, KW, stride, pad, Co, int(relu), _s())
        return y
    ws_p, ws_cs, ws_plane = _wsplit_args(w_split if f32 else None, w)
    xp, x_cs, x_lo = _p(x), x.stride(0), 0
    if x_planes is not None and ws_p and planes_ok(C, Co, ldx):
        xp, x_cs, x_lo = _planes_args(x_planes, x)  # LDS-DMA GEMM on pre-split operands
        planes_launches["fwd"] += 1
    _C.conv_nt(xp, _p(w), _p(y), _p(bias), x_cs, y.stride(0), w_cs, b_cs, B, H, W, C, OH, OW, KH, KW, stride,
               pad, 1, M, Co, KH * KW * Ci, rep, int(relu), K, 0, nt_f32_variant if f32 else nt_variant, NULL, NULL, f32,
               _s(), ldx, ldy, _p(stats), _p(stats_valid), NULL, 0.0, 0.0, ws_p, ws_cs, ws_plane, x_lo, NULL, 0, 0)
    return y


def bn_bwd_parts_ok(dx_shape, stride: int, dtype) -> bool:
    """A dgrad of this shape can write the BN-backward partials of its dX (conv_dgrad(bnb=)):
    fp32, stride 1, 4-channel columns, one launch (no batch chunks)."""
    K, B, H, W, Ci = dx_shape
    return dtype == F32 and stride == 1 and Ci % 4 == 0 and B * H * W * Ci * 4 < WINDOW


def _wt_dgrad_ok(Co, Ci, KH, KW, H, W, stride, pad, planes: bool, ws_p) -> bool:
    # (halo shapes only — H, W >= 8: at 4 x 4 the implicit-GEMM k-major tiles win, and the
    # transposition of 512 x 512 weight rows costs more than it saves: bench/epilogue_bench.py l4)
    return bool(planes and ws_p and stride == 1 and pad == 1 and KH == 3 and KW == 3 and Co % 32 == 0
                and Ci % 32 == 0 and nt_f32_variant < 0 and min(H, W) >= 8)


def dgrad_wt_prebuild(dy_shape, w, w_split, in_hw, stride: int, pad: int):
    """The transposed, flipped weight planes a planes dgrad of this shape would build
    (conv_dgrad(wt=True)), built NOW — before a weight-gradient launch with the SGD epilogue
    rewrites the weight planes — for conv_dgrad(wt_buf=). None: that dgrad would not use them."""
    K, B, OH, OW, Co = dy_shape
    Kw, Co2, KH, KW, Ci = w.shape
    ws_p, ws_cs, ws_plane = _wsplit_args(w_split, w)
    if not (w.dtype == F32 and planes_ok(Co, Ci, Co)
            and _wt_dgrad_ok(Co, Ci, KH, KW, int(in_hw[0]), int(in_hw[1]), stride, pad, True, ws_p)):
        return None
    wt_buf = torch.empty(Kw * 2 * 9 * Ci * Co, dtype=BF16, device=w.device)
    _C.wt_planes(ws_p, ws_cs, ws_plane, _p(wt_buf), Kw, Co, Ci, _s())
    return wt_buf


def conv_dgrad(dy, w, in_hw, stride: int, pad: int, acc=None, w_split=None, dy_planes=None, acc_compact=False,
               bnb=None, acc_mask=None, wt: bool = False, wt_buf=None):
    """dX (+ `acc`, a second gradient of the same input added in the epilogue: the identity
    residual branch of a ResNet block, so autograd never materialises the sum separately).
    `dy` may be a channel slice of a wider buffer (DenseNet block-buffer gradient).
    `acc_compact` (fp32, stride > 1): `acc` holds only the stride grid (pixels (s·i, s·j)) as a
    dense [K, B, ceil(H/s), ceil(W/s), Ci] tensor — a 1x1 stride-s shortcut's input gradient —
    added by the parity class (0, 0) launch alone.
    `bnb` (bn_bwd_parts_ok shapes): (part [K, conv_stats_parts(B·H·W), 2, Ci] fp32 out, x, mask,
    mean, rstd, valid_rows, y) of the BatchNorm whose dY this dX is — the epilogue writes that BN's
    backward partial sums Σĝ, Σĝ·x̂ (bn_bwd(pre_part=)). x [K, R, Ci] may be a channel prefix of a
    wider buffer (row stride ld); the ReLU gate is the bit mask, else y > 0 (y contiguous), else
    none; mask / valid_rows / y may be None.
    `acc_mask` (fp32, with `acc`, not compact): ReLU bits [K, B·H·W, Ci / 8] gating `acc` — the
    identity shortcut's gradient dy·relu' read from the block output's gradient, never stored.
    `wt` (fp32 planes, 3x3 stride-1 pad-1): run the dgrad on the forward tiles with transposed,
    flipped weight planes (built into a scratch buffer right before the launch, or `wt_buf` from
    dgrad_wt_prebuild)."""
    K, B, OH, OW, Co = dy.shape
    Kw, Co2, KH, KW, Ci = w.shape
    H, W = int(in_hw[0]), int(in_hw[1])
    per_sample = max(OH * OW * Co, H * W * Ci) * dy.element_size()
    if acc_compact:
        assert stride > 1 and acc is not None and _f32(dy), "compact acc: fp32 strided dgrad only"
        assert acc.shape == (K, B, (H + stride - 1) // stride, (W + stride - 1) // stride, Ci), acc.shape
        assert acc.dtype == dy.dtype and acc.is_contiguous()
    bnb_args = (NULL, NULL, 0, NULL, NULL, NULL, NULL, NULL)
    if bnb is not None:
        part, bx, bmask, bmean, brstd, bvalid, by = bnb
        R = B * H * W
        assert bn_bwd_parts_ok((K, B, H, W, Ci), stride, dy.dtype) and not acc_compact
        assert part.shape == (K, conv_stats_parts(R), 2, Ci) and part.dtype == F32 and part.is_contiguous()
        bx, bxld = _pix_stride(bx.reshape(K, R, -1) if bx.is_contiguous() else bx)
        assert bx.dtype == F32 and bx.shape[-1] == Ci and bx.stride(0) == R * bxld and bxld % 4 == 0
        assert bmean.shape == (K, Ci) and brstd.shape == (K, Ci) and bmean.is_contiguous() and brstd.is_contiguous()
        if bmask is not None:
            assert bmask.dtype == torch.uint8 and bmask.is_contiguous() and bmask.numel() == K * R * Ci // 8
        if by is not None:
            assert by.dtype == F32 and by.is_contiguous() and by.numel() == K * R * Ci
        if bvalid is not None:
            assert bvalid.dtype == torch.int32 and bvalid.shape == (K,) and bvalid.is_contiguous()
        bnb_args = (_p(part), _p(bx), bxld, _p(by), _p(bmask), _p(bmean), _p(brstd), _p(bvalid))
    if acc_mask is not None:
        assert acc is not None and not acc_compact and _f32(dy), "acc_mask: fp32 dgrad with a full-size acc"
        assert acc_mask.dtype == torch.uint8 and acc_mask.is_contiguous() and Ci % 8 == 0
        assert acc_mask.numel() == K * B * H * W * Ci // 8, acc_mask.shape
    if B * per_sample >= WINDOW and dy_planes is None:
        assert bnb is None
        if acc_mask is not None:  # (chunked launches: the gated acc built once)
            from .functional import MaskedGrad

            acc, acc_mask = MaskedGrad(acc, acc_mask).dense(), None
        if acc_compact:  # (chunked launches take the full-size acc)
            full = torch.zeros((K, B, H, W, Ci), dtype=dy.dtype, device=dy.device)
            full[:, :, ::stride, ::stride] = acc
            acc, acc_compact = full, False
        dx = torch.empty((K, B, H, W, Ci), dtype=dy.dtype, device=dy.device)
        for b0, b1 in _batch_chunks(B, per_sample):
            dx[:, b0:b1] = conv_dgrad(dy[:, b0:b1], w, in_hw, stride, pad,
                                      acc=None if acc is None else acc[:, b0:b1].contiguous(), w_split=w_split)
        return dx
    dy, ld_dy = _pix_stride(dy)
    f32 = _f32(dy)
    _check(w, dy.dtype, contiguous=False, name="w")
    assert Co2 == Co
    w_cs, rep = _client_view(w, K)
    dx = torch.empty((K, B, H, W, Ci), dtype=dy.dtype, device=dy.device)
    if acc is not None and not acc_compact:
        # (stride > 1: every parity-class launch adds acc at the pixels it writes)
        assert acc.shape == dx.shape and acc.dtype == dy.dtype and acc.is_contiguous(), acc.shape
    if (not f32 and not acc_compact and ld_dy == Co and (stride == 1 or (gl_mode == 1 and acc is None))
            and _gl(K, B * H * W, Ci, Co, KH * KW)):
        # (strided dgrad splits into stride² short-K parity classes: conv_nt's smaller tiles win
        # there, l3a dgrad 447 vs 396 TFLOP/s). Large tiles want a k-contiguous B: one flip+transpose pass over the weight rows
        # (weights are small next to the activations), then stride² parity-class launches
        wt = torch.empty((Kw, Ci, KH, KW, Co), dtype=BF16, device=dy.device)
        _C.conv_weight_flip_t(_p(w), _p(wt), w.stride(0), Kw, Co, KH, KW, Ci, _s())
        _C.conv_gl_dgrad(_p(dy), _p(wt), _p(dx), _p(acc), K, rep, B, OH, OW, Co, H, W, Ci, KH, KW, stride, pad, _s())
        return dx
    # B operand read straight from the forward weight (flip + transpose in the loader);
    # stride > 1 splits into stride² dense parity-class GEMMs (csrc/conv_nt.hip: conv_dgrad)
    ws_p, ws_cs, ws_plane = _wsplit_args(w_split if f32 else None, w)
    dyp, dy_cs, dy_lo = _p(dy), dy.stride(0), 0
    if dy_planes is not None and ws_p and planes_ok(Co, Ci, ld_dy):
        dyp, dy_cs, dy_lo = _planes_args(dy_planes, dy)
        planes_launches["dgrad"] += 1
    wt_ready = wt_buf is not None
    if (wt or wt_ready) and _wt_dgrad_ok(Co, Ci, KH, KW, H, W, stride, pad, bool(dy_lo), ws_p):
        if wt_buf is None:
            wt_buf = torch.empty(Kw * 2 * 9 * Ci * Co, dtype=BF16, device=dy.device)
        planes_launches["dgrad_wt"] += 1
    else:
        assert not wt_ready, "conv_dgrad: a prebuilt wt_buf for a dgrad that does not take it"
        wt_buf = None
    _C.conv_dgrad(dyp, _p(w), _p(dx), _p(acc), w_cs, K, rep, B, OH, OW, Co, H, W, Ci, KH, KW, stride, pad,
                  nt_f32_variant if f32 else nt_variant, f32, _s(), ld_dy, dy_cs, ws_p, ws_cs, ws_plane, dy_lo,
                  int(bool(acc_compact)), *bnb_args, _p(wt_buf), _p(acc_mask), int(wt_ready))
    return dx


# fp32 weight gradients: split-K partial slabs folded in split order (bitwise-reproducible, no
# atomics) — OPTIONS.deterministic = False restores fp32 atomics into pre-zeroed rows (A/B)
_part_cache: dict = {}


def _tn_part(numel: int, device) -> torch.Tensor:
    """Split-K slab buffer of the deterministic wgrad fold, per (device, stream); grown, never
    shrunk, so a captured graph keeps a stable pointer after the warm-up step sized it."""
    return _grown(_part_cache, (device, torch.cuda.current_stream().cuda_stream), numel, device)


def _sgd_arg(sgd):
    """The SGD epilogue of one conv_tn / halo_wgrad launch (engine.params.FusedSGD ref: (handle,
    name, element offset)), passed with that launch: it steps the weight rows instead of storing
    dW. None: dW is stored."""
    if sgd is None:
        return None
    f, _, off = sgd
    wd, mom, damp, nest = f.hyper
    assert f.theta.stride(1) == 1 and f.mom.stride(0) == f.theta.stride(0) and f.split.is_contiguous()
    return (_p(f.theta) + off * 4, _p(f.mom) + off * 4, _p(f.split) + off * 2, f.theta.stride(0), f.split.stride(0),
            f.split.stride(1), _p(f.lr), _p(f.active), _p(f.first), float(wd), float(mom), float(damp), int(nest))


def _tn_launch(dy, x, gw, dy_cs, x_cs, B, H, W, C, OH, OW, KH, KW, stride, pad, M, Co, R, K, f32, ldy, ldx,
               dy_planes=None, x_planes=None, sgd=None):
    """conv_tn with the split-K policy: slabs + ordered fold (fp32, deterministic) or atomics."""
    planes = f32 and dy_planes is not None and x_planes is not None
    tv = (_C.conv_tn_pl_variant() if planes else tn_f32_variant) if f32 else tn_variant
    dyp, xp, dy_lo, x_lo = _p(dy), _p(x), 0, 0
    if planes:
        dyp, dy_cs, dy_lo = _planes_args(dy_planes, dy)
        xp, x_cs, x_lo = _planes_args(x_planes, x)
        planes_launches["wgrad"] += 1
    splitk = _C.conv_tn_splitk(K, Co, R, M, C, tv, f32, ldy, ldx, int(planes))
    part = NULL
    if splitk > 1:
        if f32 and (OPTIONS.deterministic or planes):
            part = _p(_tn_part(splitk * K * Co * R, gw.device))
        else:
            gw.zero_()
    if sgd is not None:
        assert planes, "the SGD epilogue needs the plane TN kernels"
    _C.conv_tn(dyp, xp, _p(gw), dy_cs, x_cs, gw.stride(0), B, H, W, C, OH, OW, KH, KW, stride, pad, M, Co, R, K, tv,
               f32, _s(), ldy, ldx, part, dy_lo, x_lo, _sgd_arg(sgd))


def conv_wgrad(dy, x, gw, stride: int, pad: int, dy_planes=None, x_planes=None, sgd=None) -> bool:
    """dW of a conv into the fp32 gradient rows gw [K, Co, KH, KW, Ci]. `dy_planes` /
    `x_planes` (fp32 only, both or neither): pre-split operands (split_planes), read by the
    LDS-DMA GEMM of csrc/conv_pl.hip when the shape allows (planes_ok). `sgd` (a FusedSGD ref,
    plane path only): the kernel steps the weights instead of storing dW — returns True then."""
    K, B, OH, OW, Co = dy.shape
    _, _, H, W, C = x.shape
    per_sample = max(OH * OW * Co, H * W * C) * dy.element_size()
    if B * per_sample >= WINDOW and dy_planes is None:
        # Σ over batch chunks of the chunk weight gradients (fp32, chunk order fixed)
        chunks = _batch_chunks(B, per_sample)
        tmp = torch.empty_like(gw) if len(chunks) > 1 else gw
        for i, (b0, b1) in enumerate(chunks):
            conv_wgrad(dy[:, b0:b1], x[:, b0:b1], gw if i == 0 else tmp, stride, pad)
            if i:
                gw.add_(tmp)
        return
    dy, ldy = _pix_stride(dy)
    x, ldx = _pix_stride(x)
    f32 = _f32(dy)
    _check(x, dy.dtype, contiguous=False, name="x")
    assert gw.dtype == torch.float32 and gw.shape[0] == K and gw[0].is_contiguous()
    _, Co2, KH, KW, Ci = gw.shape
    assert Co2 == Co and Ci == C
    M = B * OH * OW
    R = KH * KW * C
    use_pl = (dy_planes is not None and x_planes is not None and f32 and C % 8 == 0 and Co % 8 == 0
              and ldy == Co and ldx == C)
    _tn_launch(dy, x, gw, dy.stride(0), x.stride(0), B, H, W, C, OH, OW, KH, KW, stride, pad, M, Co, R, K, f32,
               ldy, ldx, dy_planes if use_pl else None, x_planes if use_pl else None,
               sgd if use_pl else None)
    return bool(use_pl and sgd is not None)


def halo_wgrad_ok(x_shape, Co: int) -> bool:
    """conv_halo_wgrad.hip serves the 3x3 / stride-1 / pad-1 weight gradient of an input
    [K, B, H, W, C] with Co output channels (64-channel blocks; 32², 16², 8² images)."""
    K, B, H, W, C = x_shape
    return bool(_C.halo_wgrad_supported(B, H, W, C, Co))


def halo_wgrad(dy, x, gw, dy_planes=None, x_planes=None, bn=None, valid=None, sgd=None, bn_bwd=None) -> bool:
    """3x3 / stride-1 / pad-1 weight gradient on the LDS-halo kernel (csrc/conv_halo_wgrad.hip)
    into the gradient rows gw [K, N, 3, 3, C]. dy [K, B, H, W, N] fp32 (contiguous) or its split
    planes `dy_planes` [K, 2, ...]; x [K, B, H, W, C]: its planes `x_planes`, or — `bn` = (coef
    [K, C, 2], relu, valid_rows) — the RAW input of a BatchNorm(+ReLU) that the loader applies
    (the operand bits of bn_apply's planes), or plain fp32. `valid` [K] (samples): the images past
    it carry zero dY and X (BatchNorm outputs) and are skipped. False: shape not served. `sgd` (a
    FusedSGD ref): the kernel (or its fold) steps the weights instead of storing dW.
    `bn_bwd` = (dy_out, x_bn, mask, coef [K, N, 3], valid_rows, dxp [K, 2, R, N]): dY is the input
    gradient of a BatchNorm(+ReLU) — `dy_out` its output gradient (fp32, dy's shape), `x_bn` its
    raw input, `mask` the ReLU bits (or None), `coef` bn_bwd(stage=1)'s coefficients — applied in the
    loader (bn_bwd_apply's bits), and the kernel also writes dY's split planes into `dxp` for the
    dgrad (`dy` / `dy_planes` are then the planes-only alias and ignored)."""
    K, B, H, W, N = dy.shape
    C = x.shape[-1]
    if x.shape != (K, B, H, W, C) or dy.dtype != F32 or x.dtype != F32 or not halo_wgrad_ok(x.shape, N):
        return False
    assert gw.shape == (K, N, 3, 3, C) and gw.dtype == F32 and gw[0].is_contiguous(), gw.shape
    if gw.data_ptr() % 16 or gw.stride(0) % 4:
        return False
    bnb = None
    if bn_bwd is not None:
        dyo, xb, mk, cf, vr, dxp = bn_bwd
        R = B * H * W
        if not (dyo.is_contiguous() and xb.is_contiguous() and dyo.numel() == K * R * N and xb.numel() == K * R * N
                and dyo.dtype == F32 and xb.dtype == F32):
            return False
        assert cf.shape == (K, N, 3) and cf.dtype == F32 and cf.is_contiguous(), cf.shape
        assert dxp.shape == (K, 2, R, N) and dxp.dtype == BF16 and dxp.is_contiguous(), dxp.shape
        if mk is not None:
            assert mk.dtype == torch.uint8 and mk.is_contiguous() and mk.numel() == K * R * N // 8
        if vr is not None:
            vr = vr.to(torch.int32).contiguous()
            assert vr.shape == (K,)
        bnb = (_p(xb), _p(mk), _p(cf), _p(vr), _p(dxp))
        dyp, dy_cs, dy_lo, dm = _p(dyo), R * N, 0, 2
    elif dy_planes is not None:
        dyp, dy_cs, dy_lo = _planes_args(dy_planes, dy)
        dm = 0
    else:
        if not dy.is_contiguous():
            return False
        dyp, dy_cs, dy_lo, dm = _p(dy), dy.stride(0), 0, 1
    coef, relu, valid_rows_p = NULL, 0, NULL
    if x_planes is not None and bn is None:
        xp, x_cs, x_lo = _planes_args(x_planes, x)
        xm = 0
    else:
        if not x.is_contiguous():
            return False
        xp, x_cs, x_lo, xm = _p(x), x.stride(0), 0, 1
        if bn is not None:
            c, r, v = bn
            assert c.shape == (K, C, 2) and c.dtype == F32 and c.is_contiguous(), c.shape
            coef, relu, xm = _p(c), int(bool(r)), 2
            if v is not None:
                v = v.to(torch.int32).contiguous()
                assert v.shape == (K,)
                valid_rows_p = _p(v)
    n = _C.halo_wgrad_part_floats(K, B, H, W, C, N)
    part = _p(_tn_part(n, dy.device)) if n else NULL
    vimg = NULL
    if valid is not None:
        valid = valid.to(torch.int32).contiguous()
        assert valid.shape == (K,)
        vimg = _p(valid)
    ok = _C.halo_wgrad(dyp, dy_cs, dy_lo, N, xp, x_cs, x_lo, C, coef, relu, valid_rows_p, _p(gw), gw.stride(0), part,
                       K, B, H, W, C, N, xm, dm, _s(), vimg, _sgd_arg(sgd), bnb)
    if ok:
        planes_launches["wgrad_halo"] += 1
    return bool(ok)


def _col_sum(x, out, K: int, rows: int, C: int):
    """out[k, c] = Σ_rows x[k, row, c] (fp32, into a strided gradient view): partials folded in
    order when deterministic, else fp32 atomics into the zeroed view."""
    if OPTIONS.deterministic:
        ws = _tn_part(_C.col_sum_workspace_floats(K, rows, C), x.device)
        _C.col_sum(_p(x), _p(out), out.stride(0), K, rows, C, _f32(x), _s(), _p(ws))
    else:
        out.zero_()
        _C.col_sum(_p(x), _p(out), out.stride(0), K, rows, C, _f32(x), _s(), NULL)


def bias_grad(dy, gb):
    """gb[k, c] = Σ_{b,h,w} dy[k, b, h, w, c] (conv bias gradient)."""
    K = dy.shape[0]
    C = dy.shape[-1]
    rows = dy.numel() // (K * C)
    _col_sum(dy.contiguous(), gb, K, rows, C)


# --------------------------------------------------------------------------- linear
def _out_planes(y):
    """(pointer, client stride, hi→lo distance) of fresh [K, 2, ...] planes for an fp32 output y."""
    yp = torch.empty((y.shape[0], 2) + tuple(y.shape[1:]), dtype=BF16, device=y.device)
    return yp, _p(yp), yp.stride(0), yp.stride(1)


def linear_fwd(x, w, b=None, relu=False, acc=None, drop_p: float = 0.0, drop_seeds=None, w_split=None,
               x_planes=None, out_planes: bool = False):
    """y = x Wᵀ + b, optionally ReLU'd, dropped out (`drop_p`, per-client-row `drop_seeds`
    [K] int32: the epilogue mask of `dropout_apply`) and/or + `acc` (a residual branch), in the
    epilogue. `x_planes` [K, 2, N, Fi] (fp32, with `w_split`): x's split planes — the LDS-DMA
    plane GEMM (csrc/conv_pl.hip) when the shape allows (planes_ok). `out_planes` (fp32): the
    epilogue also writes y's split planes; returns (y, planes [K, 2, N, Fo]) then."""
    K, N, Fi = x.shape
    x = x.contiguous()
    f32 = _f32(x)
    Kw, Fo, Fi2 = w.shape
    assert Fi2 == Fi and w.dtype == x.dtype
    w_cs, rep = _client_view(w, K)
    b_cs = _client_view(b, K)[0] if b is not None else 0
    y = torch.empty((K, N, Fo), dtype=x.dtype, device=x.device)
    if acc is not None:
        assert acc.shape == y.shape and acc.dtype == x.dtype and acc.is_contiguous()
    ws_p, ws_cs, ws_plane = _wsplit_args(w_split if f32 else None, w)
    xp, x_cs, x_lo = _p(x), N * Fi, 0
    if x_planes is not None and f32 and ws_p and planes_ok(Fi, Fo):
        xp, x_cs, x_lo = _planes_args(x_planes.reshape((K, 2) + tuple(x.shape[1:])), x)
        planes_launches["linear_fwd"] += 1
    yp, ypp, yp_cs, yp_lo = _out_planes(y) if (out_planes and f32) else (None, NULL, 0, 0)
    _C.conv_nt(xp, _p(w), _p(y), _p(b), x_cs, N * Fo, w_cs, b_cs, 1, N, 1, Fi, N, 1, 1, 1, 1, 0, 1, N, Fo, Fi, rep,
               int(relu), K, 0, nt_f32_variant if f32 else nt_variant, _p(acc), NULL, f32, _s(), 0, 0, NULL, NULL,
               _p(_drop_seeds(drop_seeds, K, drop_p)), float(drop_p), 0.0, ws_p, ws_cs, ws_plane, x_lo,
               ypp, yp_cs, yp_lo)
    return (y, yp) if out_planes else y


def linear_dgrad(dy, w, gate=None, gate_scale: float = 1.0, w_split=None, dy_planes=None, out_planes: bool = False,
                 acc=None):
    """dX = dY W, zeroed where `gate` <= 0 when given (gate = the ReLU output this layer read:
    the gradient then leaves already through the ReLU), times `gate_scale` (the 1/(1-p) of a
    dropout folded into that ReLU output). `dy_planes` [K, 2, N, Fo] (fp32, with `w_split`): dY's
    split planes — the LDS-DMA plane GEMM with the k-major weight; `out_planes`: the epilogue also
    writes dX's planes (returns (dx, planes)). `acc` [K, N, Fi] (contiguous): a second gradient of
    X added in the epilogue (a residual branch's, ops.functional.ResidualLink)."""
    K, N, Fo = dy.shape
    dy = dy.contiguous()
    f32 = _f32(dy)
    Kw, Fo2, Fi = w.shape
    assert w.dtype == dy.dtype
    w_cs, rep = _client_view(w, K)
    dx = torch.empty((K, N, Fi), dtype=dy.dtype, device=dy.device)
    if gate is not None:
        assert gate.shape == dx.shape and gate.dtype == dy.dtype and gate.is_contiguous()
    if acc is not None:
        assert acc.shape == dx.shape and acc.dtype == dy.dtype and acc.is_contiguous()
    # dX = dY W: B[n=fi][k=fo] = W[fo][fi] is k-major in W's own layout
    ws_p, ws_cs, ws_plane = _wsplit_args(w_split if f32 else None, w)
    dyp, dy_cs, dy_lo = _p(dy), N * Fo, 0
    if dy_planes is not None and f32 and ws_p and planes_ok(Fo, Fi):
        dyp, dy_cs, dy_lo = _planes_args(dy_planes.reshape((K, 2) + tuple(dy.shape[1:])), dy)
        planes_launches["linear_dgrad"] += 1
    xp_, ypp, yp_cs, yp_lo = _out_planes(dx) if (out_planes and f32) else (None, NULL, 0, 0)
    _C.conv_nt(dyp, _p(w), _p(dx), NULL, dy_cs, N * Fi, w_cs, 0, 1, N, 1, Fo, N, 1, 1, 1,
               1, 0, 1, N, Fi, Fo, rep, 0, K, 1, nt_f32_variant if f32 else nt_variant, _p(acc), _p(gate), f32, _s(),
               0, 0, NULL, NULL, NULL, 0.0, float(gate_scale), ws_p, ws_cs, ws_plane, dy_lo, ypp, yp_cs, yp_lo)
    return (dx, xp_) if out_planes else dx


def _drop_seeds(seeds, K: int, p: float):
    if not p:
        return None
    assert seeds is not None and seeds.dtype == torch.int32 and seeds.numel() == K and seeds.is_contiguous()
    return seeds


def dropout_apply(x, seeds, p: float, planes: int = 0, colsum=None):
    """out = keep ? x / (1-p) : 0 over x [K, rows, N] — the GEMM epilogue's dropout mask (the
    backward of a dropout fused into a linear's output). `planes` (fp32, N even): 1 = also
    write out's split planes [K, 2, *x.shape[1:]], 2 = write ONLY the planes (out is their
    fp32-typed alias, planes_buffer); returns (out, planes) then. `colsum` [K, N] (with planes):
    also written with out's column sums (the consuming linear's bias gradient, fixed order)."""
    K = x.shape[0]
    N = x.shape[-1]
    x = x.contiguous()
    rows = x.numel() // (K * N)
    if planes and _f32(x) and N % 2 == 0:
        if planes == 2:
            out, yp = planes_buffer(tuple(x.shape), x.device)
        else:
            out = torch.empty_like(x)
            yp = torch.empty((K, 2) + tuple(x.shape[1:]), dtype=BF16, device=x.device)
        cs_args = (NULL, 0, NULL)
        if colsum is not None:
            assert colsum.shape == (K, N) and colsum.dtype == F32 and colsum.stride(1) == 1
            ws = _tn_part(_C.dropout_planes_ws_floats(K, rows, N), x.device)
            cs_args = (_p(colsum), colsum.stride(0), _p(ws))
        _C.dropout_planes(_p(x), _p(out) if planes == 1 else NULL, _p(yp), K, rows, N, _p(_drop_seeds(seeds, K, p)),
                          float(p), 1.0 / (1.0 - p), _s(), *cs_args)
        return out, yp
    assert colsum is None, "dropout_apply(colsum=) needs the planes path (fp32, even N)"
    out = torch.empty_like(x)
    _C.dropout_apply(_p(x), _p(out), K, rows, N, N, _p(_drop_seeds(seeds, K, p)), float(p), 1.0 / (1.0 - p),
                     _f32(x), _s())
    return (out, None) if planes else out


def linear_wgrad(dy, x, gw, gb=None, dy_planes=None, x_planes=None, sgd=None) -> bool:
    """dW = dYᵀ X into gw [K, Fo, Fi] (+ the bias gradient Σ dY into gb). `dy_planes` /
    `x_planes` [K, 2, N, ·] (fp32, both or neither): the LDS-DMA plane wgrad (csrc/conv_pl.hip).
    `sgd` (a FusedSGD ref, plane path only): the kernel steps W instead of storing dW — returns
    True then (the bias gradient is still stored)."""
    K, N, Fo = dy.shape
    Fi = x.shape[-1]
    dy = dy.contiguous()
    x = x.contiguous()
    f32 = _f32(dy)
    assert x.dtype == dy.dtype
    assert gw.shape == (K, Fo, Fi) and gw[0].is_contiguous()
    use_pl = dy_planes is not None and x_planes is not None and f32 and Fi % 8 == 0 and Fo % 8 == 0
    dyp = dy_planes.reshape((K, 2) + tuple(dy.shape[1:])) if use_pl else None
    xp = x_planes.reshape((K, 2) + tuple(x.shape[1:])) if use_pl else None
    _tn_launch(dy, x, gw, N * Fo, N * Fi, 1, N, 1, Fi, N, 1, 1, 1, 1, 0, N, Fo, Fi, K, f32, 0, 0, dyp, xp,
               sgd if use_pl else None)
    if gb is not None:
        _col_sum(dy, gb, K, N, Fo)
    return bool(use_pl and sgd is not None)


# ------------------------------------------------------------------------ batchnorm
def planes_buffer(shape, device):
    """(fp32 tensor of `shape`, its bytes as [K, 2, *shape[1:]] bf16 split planes): client k's
    hi plane then lo plane occupy exactly the bytes of its fp32 row, so a producer that writes
    only the planes can hand autograd the fp32-typed alias (consumers read `_dls_planes`)."""
    buf = torch.empty(shape, dtype=F32, device=device)
    K = shape[0]
    return buf, buf.view(K, -1).view(BF16).view((K, 2) + tuple(shape[1:]))


def bn_fwd(x, gamma, beta, valid_rows=None, relu=False, residual=None, eps=1e-5, with_mask=False, pre_stats=None,
           planes: int = 0, res_coef=None):
    """Returns (y, mean, rstd); with_mask=True (ReLU, C % 8 == 0) also returns the 1-bit ReLU
    mask [K, R, C/8] uint8 that bn_bwd can read instead of y. `x` (and `residual`) may be
    channel slices of a wider buffer ([K, R, C] at row stride ld); y is contiguous.
    `pre_stats`: [K, parts, 2, C] Σx / Σx² partials written by the producing conv's epilogue
    (conv_fwd(stats=)) — the statistics pass over x is skipped.
    `planes` (fp32): 1 = also write y's split planes, 2 = write only the planes (y is then their
    fp32-typed alias, see planes_buffer); the planes [K, 2, R, C] are returned last.
    `res_coef` [K, C, 2] (fp32, with `residual`): the residual is the RAW input of a second
    BatchNorm without ReLU (same valid rows) whose (scale, shift) pairs bn_coef computed — its
    apply is folded into this one (y = act(bn(x) + scale·res + shift), the bits of applying it
    first)."""
    K, R, C = x.shape
    x, ldx = _pix_stride(x)
    assert x.stride(0) == R * ldx, "client stride of a strided BN input must be R*ld"
    g_cs, rep = _client_view(gamma, K)
    yp = None
    if planes and x.dtype == F32:
        if planes == 2:
            y, yp = planes_buffer((K, R, C), x.device)
        else:
            y = torch.empty((K, R, C), dtype=x.dtype, device=x.device)
            yp = torch.empty((K, 2, R, C), dtype=BF16, device=x.device)
    else:
        planes = 0
        y = torch.empty((K, R, C), dtype=x.dtype, device=x.device)
    mean = torch.empty((K, C), dtype=torch.float32, device=x.device)
    rstd = torch.empty((K, C), dtype=torch.float32, device=x.device)
    ws = _workspace(_C.bn_workspace_floats(K, R, C), x.device)
    if residual is not None:
        residual = residual.contiguous() if ldx == C else residual
        assert _pix_stride(residual)[1] == ldx and residual.stride() == x.stride()
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    if pre_stats is not None:
        assert pre_stats.dtype == torch.float32 and pre_stats.is_contiguous()
        assert pre_stats.shape[0] == K and pre_stats.shape[2:] == (2, C), pre_stats.shape
    mask = None
    if with_mask and relu and C % 8 == 0 and ldx % 8 == 0:
        mask = torch.empty((K, R, C // 8), dtype=torch.uint8, device=x.device)
    assert gamma.dtype == x.dtype and (residual is None or residual.dtype == x.dtype)
    if res_coef is not None:
        assert residual is not None and x.dtype == F32 and res_coef.shape == (K, C, 2) and res_coef.is_contiguous()
    _C.bn_fwd(_p(x), _p(gamma), _p(beta), _p(residual), _p(y), _p(mean), _p(rstd), _p(vr), g_cs, K, R, C, int(relu),
              eps, rep, _p(ws), _p(mask), _f32(x), _s(), ldx, _p(pre_stats),
              0 if pre_stats is None else pre_stats.shape[1], _p(yp), int(planes != 2), NULL, 1, _p(res_coef))
    out = (y, mean, rstd, mask) if with_mask else (y, mean, rstd)
    return out + (yp,) if planes else out


def bn_coef(x, gamma, beta, valid_rows=None, eps=1e-5, pre_stats=None):
    """BatchNorm statistics → per-(client, channel) (scale, shift) pairs [K, C, 2] fp32, with
    nothing applied: the consumer conv applies them while staging its input (conv_halo_bn_fwd).
    Same statistics / coefficient kernels (and bits) as bn_fwd."""
    K, R, C = x.shape
    assert x.dtype == F32
    x, ldx = _pix_stride(x)  # (a channel prefix of DenseNet's block buffer is read in place)
    assert x.stride(0) == R * ldx, "client stride of a strided BN input must be R*ld"
    g_cs, rep = _client_view(gamma, K)
    mean = torch.empty((K, C), dtype=torch.float32, device=x.device)
    rstd = torch.empty((K, C), dtype=torch.float32, device=x.device)
    coef = torch.empty((K, C, 2), dtype=torch.float32, device=x.device)
    ws = _workspace(_C.bn_workspace_floats(K, R, C), x.device)
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    if pre_stats is not None:
        assert pre_stats.dtype == torch.float32 and pre_stats.is_contiguous()
        assert pre_stats.shape[0] == K and pre_stats.shape[2:] == (2, C), pre_stats.shape
    _C.bn_fwd(_p(x), _p(gamma), _p(beta), NULL, NULL, _p(mean), _p(rstd), _p(vr), g_cs, K, R, C, 0, eps, rep, _p(ws),
              NULL, 1, _s(), ldx, _p(pre_stats),
              0 if pre_stats is None else pre_stats.shape[1], NULL, 1, _p(coef), 0, NULL)
    return coef, mean, rstd


def bn_coef_sums(sums, C: int, gamma, beta, R: int, valid_rows=None, eps=1e-5):
    """bn_coef from running fp64 per-channel sums `sums` [K, 2, ld] (Σx, Σx² over the valid rows)
    for the first C channels, with no pass over x (DenseNet block: the statistics of a channel are
    summed once, from the epilogue of the conv that produced it)."""
    K = sums.shape[0]
    assert sums.dtype == torch.float64 and sums.is_contiguous() and sums.shape[1] == 2 and C <= sums.shape[2]
    g_cs, rep = _client_view(gamma, K)
    mean = torch.empty((K, C), dtype=torch.float32, device=sums.device)
    rstd = torch.empty((K, C), dtype=torch.float32, device=sums.device)
    coef = torch.empty((K, C, 2), dtype=torch.float32, device=sums.device)
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    _C.bn_coef_sums(_p(sums), sums.stride(0), sums.shape[2], _p(gamma), _p(beta), _p(vr), g_cs, K, R, C, eps, rep,
                    _p(mean), _p(rstd), _p(coef), _s())
    return coef, mean, rstd


def part_sum_f64(part, out):
    """out[k, j, c] = Σ_p part[k, p, j, c] in fp64, fixed order (DenseNet running channel sums):
    `part` [K, parts, 2, g] fp32 conv-epilogue partials, `out` an fp64 [K, 2, g] view with unit
    channel stride (a channel slice of the block's [K, 2, Ct] sums)."""
    K, nparts, two, g = part.shape
    assert two == 2 and part.dtype == F32 and part.is_contiguous() and 2 * g <= 1024
    assert out.dtype == torch.float64 and out.shape == (K, 2, g) and out.stride(2) == 1
    _C.part_sum_f64(_p(part), K, nparts, g, _p(out), out.stride(0), out.stride(1), _s())


def chan_sums_f64(x, valid_rows, out):
    """out[k, 0, c] = Σ x[k, r, c], out[k, 1, c] = Σ x[k, r, c]² over r < valid_rows[k] (all rows
    if None), in fp64 with a fixed order (DenseNet block input's running sums). `x` [K, R, C] fp32
    with unit channel stride (a channel prefix of a wider buffer is fine); `out` an fp64 [K, 2, C]
    view with unit channel stride."""
    K, R, C = x.shape
    x, ldx = _pix_stride(x)
    assert x.dtype == F32 and x.stride(0) == R * ldx and 2 * C <= 1024
    assert out.dtype == torch.float64 and out.shape == (K, 2, C) and out.stride(2) == 1
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    ws = torch.empty(max(1, K * _C.chan_sums_f64_ws(R, C)), dtype=torch.float64, device=x.device)
    _C.chan_sums_f64(_p(x), x.stride(0), ldx, K, R, C, _p(vr), _p(ws), _p(out), out.stride(0), out.stride(1), _s())


def halo_bn_ok(shape, w) -> bool:
    """conv_halo_bn_fwd serves a [K, B, H, W, C] fp32 input and a 3x3 weight of this shape."""
    K, B, H, W, C = shape
    return (w.dim() == 5 and w.shape[2] == 3 and w.shape[3] == 3 and w.shape[4] == C
            and bool(_C.conv_halo_bn_supported(B, H, W, C, w.shape[1])))


def bn_apply_only(x, coef, valid_rows, relu: bool, yp, mask=None, y=None):
    """Materialise a deferred BN: relu?(coef-scaled x) → split planes yp [K, 2, R, C] (+ ReLU bits)
    and / or the fp32 output `y` [K, R, C] (bn_fwd's bits either way)."""
    K, R, C = x.shape
    assert x.dtype == F32 and x.is_contiguous() and coef.shape == (K, C, 2)
    assert yp is None or (yp.shape == (K, 2, R, C) and yp.dtype == BF16 and yp.is_contiguous())
    assert y is None or (y.shape == (K, R, C) and y.dtype == F32 and y.is_contiguous())
    if mask is not None:
        assert mask.shape == (K, R, C // 8) and C % 8 == 0
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    _C.bn_apply_only(_p(x), _p(coef), _p(vr), K, R, C, int(relu), _p(yp), _p(mask), _s(), _p(y))


def conv_halo_bn_fwd(x, coef, relu: bool, valid_rows, w, w_split, stats=None, stats_valid=None, yp=None, mask=None):
    """3x3 / stride-1 / pad-1 fp32 conv of relu?(BN(x)) with the BN applied in the halo loader
    (csrc/conv_halo.hip BNF): x [K, B, H, W, C] is the RAW previous conv output, `coef` [K, C, 2]
    its BN (scale, shift) pairs (bn_coef), `valid_rows` [K] the BN's valid rows (zero past them).
    `yp` [K, 2, B·H·W, C] / `mask` [K, B·H·W, C/8] (training): the normalised activation's split
    planes and ReLU bits are written as well (the conv's weight gradient and the BN's backward
    read them). Returns y [K, B, H, W, N], or None where no halo kernel serves the shape."""
    K, B, H, W, C = x.shape
    Kw, N, KH, KW, Ci = w.shape
    if not (x.dtype == F32 and x.is_contiguous() and KH == 3 and KW == 3 and Ci == C and w_split is not None):
        return None
    assert coef.shape == (K, C, 2) and coef.dtype == F32 and coef.is_contiguous()
    w_cs, rep = _client_view(w, K)
    ws_p, ws_cs, ws_plane = _wsplit_args(w_split, w)
    y = torch.empty((K, B, H, W, N), dtype=F32, device=x.device)
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    if stats is not None:
        assert stats.shape == (K, conv_stats_parts(B * H * W), 2, N) and stats.is_contiguous()
        if stats_valid is not None:
            stats_valid = stats_valid.to(torch.int32).contiguous()
    if yp is not None:
        assert yp.shape == (K, 2, B * H * W, C) and yp.dtype == BF16 and yp.is_contiguous()
    if mask is not None:
        assert mask.shape == (K, B * H * W, C // 8) and mask.dtype == torch.uint8 and mask.is_contiguous()
    ok = _C.conv_halo_bn_fwd(_p(x), x.stride(0), _p(coef), int(relu), _p(vr), ws_p, ws_cs, ws_plane, rep, _p(y),
                             y.stride(0), K, B, H, W, C, N, _p(stats), _p(stats_valid), _s(), _p(yp), _p(mask))
    if ok:
        planes_launches["fwd_bn_fused"] += 1
    return y if ok else None


_dw_part_cache: dict = {}


def dense_wgrad(dy, y, gw, x=None, bn_coef=None, valid_rows=None) -> bool:
    """DenseNet growth-conv weight gradient on the LDS-halo kernel (csrc/conv_dense_wgrad.hip):
    dy [K, B, H, W, N] the block gradient's growth channels (a pixel-strided view, read in place),
    y [K, B·H·W, C] the normalised prefix (contiguous), gw [K, N, 3, 3, C] the gradient rows
    (written). With `bn_coef` [K, C, 2] (the forward's BN scale / shift) the normalised prefix is
    recomputed while staged from `x` [K, B, H, W, C] (the block buffer's raw prefix, read in place)
    — bitwise the y the forward would have stored (rows past `valid_rows` zero) — and y is unused.
    False: shape not served (nothing ran)."""
    K, B, H, W, N = dy.shape
    if bn_coef is not None:
        C = x.shape[-1]
        xs, ldx = _pix_stride(x)
        if (x.dtype != F32 or xs.data_ptr() != x.data_ptr() or ldx % 4 or x.stride(0) != B * H * W * ldx
                or bn_coef.shape != (K, C, 2) or not bn_coef.is_contiguous()):
            return False
        src, src_cs = x, x.stride(0)
    else:
        if (y.dim() != 3 or dy.dtype != F32 or y.dtype != F32 or not y.is_contiguous()
                or y.shape[:2] != (K, B * H * W)):
            return False
        C = y.shape[2]
        src, src_cs, ldx = y, y.stride(0), 0
    if dy.dtype != F32 or not _C.dense_wgrad_supported(B, H, W, C, N):
        return False
    d, ldy = _pix_stride(dy)
    if d.data_ptr() != dy.data_ptr() or ldy % 4 or dy.stride(0) != B * H * W * ldy:
        return False
    assert gw.shape == (K, N, 3, 3, C) and gw.dtype == F32 and gw[0].is_contiguous(), gw.shape
    vr = valid_rows.to(torch.int32).contiguous() if (valid_rows is not None and bn_coef is not None) else None
    n = _C.dense_wgrad_part_floats(K, B, H, W, C)
    part = _grown(_dw_part_cache, (dy.device, torch.cuda.current_stream().cuda_stream), n, dy.device)
    ok = _C.dense_wgrad(_p(d), dy.stride(0), ldy, _p(src), src_cs, _p(gw), gw.stride(0), _p(part), K, B, H, W, C, N,
                        _s(), _p(bn_coef), ldx, _p(vr))
    if ok:
        planes_launches["wgrad_dense_halo"] += 1
    return bool(ok)


def dense_recompute_ok(B: int, H: int, W: int, C: int, N: int, bn_trained: bool) -> bool:
    """Both DenseNet backward kernels serve this layer from the raw prefix + the forward's BN
    (scale, shift) (dense_wgrad(bn_coef=), dense_dgrad_bn(bn_coef=)), so the forward need not
    store the normalised activation."""
    return bool(bn_trained and _C.dense_wgrad_supported(B, H, W, C, N) and _C.dense_dgrad_supported(B, H, W, C, N))


def dense_dgrad_bn(dy, w, x, dx, y, mask, mean, rstd, gamma, valid_rows, ggamma, gbeta, bn_coef=None) -> bool:
    """DenseNet layer backward after its weight gradient, fused (csrc/conv_dense_dgrad.hip): the
    growth conv's input gradient dX̂ = conv3x3ᵀ(dy) is recomputed per tile instead of stored, the
    BN backward sums come from its first pass and `dx += ` the BN input gradient from its second.
    dy [K, B, H, W, N] the block gradient's growth channels, x / dx [K, B, H, W, C] the block
    buffer's prefix and its gradient (pixel-strided views of F / dF, same strides), y [K, B·H·W, C]
    the normalised activation (ReLU gate when `mask` is None), mask [K, B·H·W, C/8] uint8 or None,
    mean / rstd [K, C], gamma [Kw, C], ggamma / gbeta the γ / β gradient rows (written).
    `bn_coef` [K, C, 2]: the forward's BN (scale, shift) — the ReLU gate is then recomputed from x
    (bitwise the forward's decision) and neither y nor mask is read.
    False: shape not served (nothing ran)."""
    K, B, H, W, N = dy.shape
    C = x.shape[-1]
    if dy.dtype != F32 or x.dtype != F32 or w.dtype != F32 or not _C.dense_dgrad_supported(B, H, W, C, N):
        return False
    d, ldy = _pix_stride(dy)
    xs, ldx = _pix_stride(x)
    dxs, lddx = _pix_stride(dx)
    if (d.data_ptr() != dy.data_ptr() or xs.data_ptr() != x.data_ptr() or dxs.data_ptr() != dx.data_ptr()
            or ldx != lddx or x.stride() != dx.stride() or ldy % 4 or ldx % 4):
        return False
    R = B * H * W
    if dy.stride(0) != R * ldy or x.stride(0) != R * ldx:
        return False
    assert w.shape[1:] == (N, 3, 3, C) and w[0].is_contiguous(), w.shape
    w_cs, rep = _client_view(w, K)
    g_cs, grep = _client_view(gamma, K)
    assert grep == 1 or gamma.shape[0] == 1
    assert mean.shape == (K, C) and rstd.shape == (K, C) and mean.is_contiguous() and rstd.is_contiguous()
    if mask is not None:
        assert mask.dtype == torch.uint8 and mask.is_contiguous() and mask.numel() == K * R * C // 8
    if y is not None:
        assert y.dtype == F32 and y.is_contiguous() and y.numel() == K * R * C
    if bn_coef is not None:
        assert bn_coef.shape == (K, C, 2) and bn_coef.dtype == F32 and bn_coef.is_contiguous()
        y = mask = None
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    dg_cs = ggamma.stride(0) if ggamma is not None else 0
    ws = _workspace(_C.dense_dgrad_ws_floats(K, B, H, C), dy.device)
    ok = _C.dense_dgrad_bn(_p(d), dy.stride(0), ldy, _p(w), w_cs, rep, _p(x), _p(dx), x.stride(0), ldx, _p(mask),
                           _p(y), _p(mean), _p(rstd), _p(vr), _p(gamma), g_cs, _p(ggamma), _p(gbeta), dg_cs, _p(ws), K,
                           B, H, W, C, N, _s(), _p(bn_coef))
    if ok:
        planes_launches["dgrad_dense_bn"] += 1
    return bool(ok)


def _c32(c: int) -> int:
    return (c + 31) // 32 * 32


def halo_bn_dense_ok(x, w) -> bool:
    """conv_halo_bn_dense_fwd serves this DenseNet layer: x the channel prefix [K, B, H, W, c]
    of the block buffer (fp32, uniform pixel stride), w [Kw, N ≤ 32, 3, 3, c]."""
    K, B, H, W, C = x.shape
    if x.dtype != F32 or w.dtype != F32 or w.dim() != 5 or tuple(w.shape[2:]) != (3, 3, C) or C % 4:
        return False
    xs, ldx = _pix_stride(x)
    if xs.data_ptr() != x.data_ptr() or ldx % 8 or x.stride(0) != B * H * W * ldx:
        return False
    return bool(_C.conv_halo_bn_dense_supported(B, H, W, _c32(C), w.shape[1]))


def dense_weight_planes(w) -> torch.Tensor:
    """[Kw, 2, N, 3, 3, C32] split planes of a growth conv's weight zero-padded to 32-channel
    chunks (the halo kernel stages whole chunks; tap rows then start 64-B aligned)."""
    Kw, N, KH, KW, C = w.shape
    C32 = _c32(C)
    assert w.dtype == F32 and w[0].is_contiguous()
    out = torch.empty((Kw, 2, N, KH, KW, C32), dtype=BF16, device=w.device)
    _C.split_rows_padded(_p(w), w.stride(0) if Kw > 1 else 0, Kw, N * KH * KW, C, C32, _p(out), _s())
    return out


def conv_halo_bn_dense_fwd(x, coef, relu: bool, valid_rows, w, out, w_planes=None, stats=None, stats_valid=None,
                           ny=None, mask=None) -> bool:
    """DenseNet growth conv out = conv3x3(relu?(BN(x))) with the BN applied in the halo loader
    (csrc/conv_halo.hip BNM 2): x [K, B, H, W, c] the block buffer's channel prefix read in place,
    coef [K, c, 2] its (scale, shift) pairs (bn_coef), out [K, B, H, W, N] the buffer's new
    channels (written in place). `ny` [K, B·H·W, c] fp32 (training): the normalised activation
    (what bn_fwd would have returned as y) for the weight gradient and the BN backward. No
    normalised copy of the prefix is written otherwise. `mask` [K, B·H·W, c/8] uint8 (with `ny`,
    c % 8 == 0): its ReLU bits, which bn_bwd reads instead of ny. False: shape not served."""
    K, B, H, W, C = x.shape
    Kw, N = w.shape[0], w.shape[1]
    C32 = _c32(C)
    xs, ldx = _pix_stride(x)
    assert xs.data_ptr() == x.data_ptr(), "x must be a pixel-strided view"
    y, ldy = _pix_stride(out)
    assert y.data_ptr() == out.data_ptr() and out.shape == (K, B, H, W, N), "out must be a pixel-strided view"
    assert coef.shape == (K, C, 2) and coef.dtype == F32
    cp = coef
    if C32 != C:
        cp = torch.zeros((K, C32, 2), dtype=F32, device=x.device)
        cp[:, :C].copy_(coef)
    cp = cp.contiguous()
    if w_planes is None:
        w_planes = dense_weight_planes(w)
    assert w_planes.shape == (Kw, 2, N, 3, 3, C32) and w_planes.dtype == BF16 and w_planes.is_contiguous()
    rep = K // Kw
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    if stats is not None:
        assert stats.shape == (K, conv_stats_parts(B * H * W), 2, N) and stats.is_contiguous()
        if stats_valid is not None:
            stats_valid = stats_valid.to(torch.int32).contiguous()
    if ny is not None:
        assert ny.shape == (K, B * H * W, C) and ny.dtype == F32 and ny.is_contiguous()
    if mask is not None:
        assert ny is not None and C % 8 == 0 and mask.shape == (K, B * H * W, C // 8) and mask.dtype == torch.uint8
        assert mask.is_contiguous()
    ok = _C.conv_halo_bn_dense_fwd(_p(xs), xs.stride(0), ldx, C, _p(cp), int(relu), _p(vr), _p(w_planes),
                                   w_planes.stride(0) if Kw > 1 else 0, w_planes.stride(1), rep, _p(y), y.stride(0),
                                   ldy, K, B, H, W, C32, N, _p(stats), _p(stats_valid), _p(ny),
                                   ny.stride(0) if ny is not None else 0, C, _p(mask), _s())
    if ok:
        planes_launches["fwd_bn_dense"] += 1
    return bool(ok)


def bn_bwd(dy, x, y, mean, rstd, gamma, valid_rows, relu, ggamma, gbeta, need_dpre, relu_mask=None, dx_out=None,
           dx_planes: int = 0, pre_part=None, coef_out=None):
    """`dx_out`: a channel slice of a wider gradient buffer (same strides as `x`) that dX is ADDED
    into (DenseNet block-buffer gradient); otherwise dX is returned contiguous. `dx_planes`
    (fp32, contiguous, no dx_out): 1 = also write dX's split planes, 2 = only the planes (dX is
    their fp32-typed alias); the planes [K, 2, R, C] are then returned as a third value.
    `pre_part`: [K, parts, 2, C] Σĝ / Σĝ·x̂ partials written by the dgrad that produced dy
    (conv_dgrad(bnb=)) — the reduction pass over dy and x is skipped.
    `coef_out` [K, C, 3] fp32: compute the backward coefficients (a, d, e) and dγ / dβ only, into
    it — no dX is written (bn_bwd_apply_planes or a loader applies them later); returns None."""
    K, R, C = x.shape
    x, ldx = _pix_stride(x)
    assert x.stride(0) == R * ldx
    dy = dy.contiguous()
    g_cs, rep = _client_view(gamma, K)
    # the kernels index γ by client k with stride g_cs: shared (Kw=1 → stride 0) or per client
    assert rep == 1 or gamma.shape[0] == 1, "bn_bwd supports per-client or fully shared γ"
    if dx_out is not None:
        assert dx_out.shape == (K, R, C) and dx_out.stride() == x.stride() and dx_out.dtype == x.dtype
        dx = dx_out
    else:
        assert ldx == C, "strided x needs a strided dx_out"
    dxp = None
    if dx_planes and dx_out is None and x.dtype == F32:
        if dx_planes == 2:
            dx, dxp = planes_buffer((K, R, C), x.device)
        else:
            dx = torch.empty((K, R, C), dtype=x.dtype, device=x.device)
            dxp = torch.empty((K, 2, R, C), dtype=BF16, device=x.device)
    else:
        dx_planes = 0
        if dx_out is None:
            dx = torch.empty((K, R, C), dtype=x.dtype, device=x.device)
    dpre = torch.empty((K, R, C), dtype=x.dtype, device=x.device) if need_dpre else None
    ws = _workspace(_C.bn_workspace_floats(K, R, C), x.device)
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    dg_cs = ggamma.stride(0) if ggamma is not None else 0
    assert dy.dtype == x.dtype == gamma.dtype
    if pre_part is not None:
        assert pre_part.dtype == F32 and pre_part.is_contiguous() and pre_part.shape == (K, (R + 31) // 32, 2, C)
    if coef_out is not None:
        assert coef_out.shape == (K, C, 3) and coef_out.dtype == F32 and coef_out.is_contiguous()
        assert dx_out is None and not need_dpre
    _C.bn_bwd(_p(dy), _p(x), _p(y), _p(mean), _p(rstd), _p(gamma), _p(vr), g_cs, K, R, C, int(relu), _p(dx), _p(dpre),
              _p(ggamma), _p(gbeta), dg_cs, _p(ws), _p(relu_mask), _f32(x), _s(), ldx,
              int(dx_out is not None), _p(dxp), int(dx_planes != 2), _p(pre_part),
              0 if pre_part is None else pre_part.shape[1], _p(coef_out), 1 if coef_out is not None else 0)
    if coef_out is not None:
        return None
    if dx_planes:
        return dx, dpre, dxp
    return dx, dpre


def bn_bwd_apply_planes(dy, x, relu_mask, coef, valid_rows, dxp) -> None:
    """The apply stage of a BN backward whose coefficients bn_bwd(coef_out=) computed: dX's split
    planes into `dxp` [K, 2, R, C] (dy, x [K, R, C] fp32 contiguous; `relu_mask` the ReLU bits or
    None for no gate) — bn_bwd's own apply pass, for a consumer that cannot apply it itself."""
    K, R, C = x.shape
    assert dy.shape == x.shape and dy.is_contiguous() and x.is_contiguous() and dy.dtype == F32 == x.dtype
    assert coef.shape == (K, C, 3) and dxp.shape == (K, 2, R, C) and dxp.is_contiguous()
    ws = _workspace(_C.bn_workspace_floats(K, R, C), x.device)
    vr = valid_rows.to(torch.int32).contiguous() if valid_rows is not None else None
    _C.bn_bwd(_p(dy), _p(x), NULL, NULL, NULL, NULL, _p(vr), 0, K, R, C, int(relu_mask is not None), _p(dxp), NULL,
              NULL, NULL, 0, _p(ws), _p(relu_mask), 1, _s(), C, 0, _p(dxp), 0, NULL, 0, _p(coef), 2)


# ------------------------------------------------------------------------ layernorm
def ln_fwd(x, gamma, beta, eps=1e-5, planes: bool = False):
    """`planes` (fp32): also write y's split planes [K, 2, *x.shape[1:]] (returned fourth) for
    the split-plane linears that read y."""
    K = x.shape[0]
    C = x.shape[-1]
    x = x.contiguous()
    g_cs, rep = _client_view(gamma, K)
    rpc = x.numel() // (K * C)
    y = torch.empty_like(x)
    mean = torch.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    assert gamma.dtype == x.dtype
    yp = torch.empty((K, 2) + tuple(x.shape[1:]), dtype=BF16, device=x.device) if planes and x.dtype == F32 else None
    _C.ln_fwd(_p(x), _p(gamma), _p(beta), _p(y), _p(mean), _p(rstd), g_cs, K, rpc, C, eps, rep, _f32(x), _s(), _p(yp))
    if planes:
        return y, mean, rstd, yp
    return y, mean, rstd


def ln_bwd(dy, x, mean, rstd, gamma):
    K = x.shape[0]
    C = x.shape[-1]
    assert C <= 1024
    g_cs, rep = _client_view(gamma, K)
    rpc = x.numel() // (K * C)
    dx = torch.empty_like(x)
    if OPTIONS.deterministic:
        dgamma = torch.empty((K, C), dtype=torch.float32, device=x.device)
        dbeta = torch.empty((K, C), dtype=torch.float32, device=x.device)
        ws = _p(_tn_part(_C.ln_workspace_floats(K, rpc, C), x.device))
    else:
        dgamma = torch.zeros((K, C), dtype=torch.float32, device=x.device)
        dbeta = torch.zeros((K, C), dtype=torch.float32, device=x.device)
        ws = NULL
    _C.ln_bwd(_p(dy.contiguous()), _p(x), _p(mean), _p(rstd), _p(gamma), g_cs, K, rpc, C, _p(dx), _p(dgamma),
              _p(dbeta), C, _f32(x), _s(), ws)
    return dx, dgamma, dbeta


# -------------------------------------------------------------------------- pooling
def _pool_fwd(x, k, s, pad, mode):
    K, B, H, W, C = x.shape
    x = x.contiguous()
    OH = (H + 2 * pad - k) // s + 1
    OW = (W + 2 * pad - k) // s + 1
    y = torch.empty((K, B, OH, OW, C), dtype=x.dtype, device=x.device)
    idx = torch.empty((K, B, OH, OW, C), dtype=torch.int32, device=x.device) if mode == 0 else None
    _C.pool_fwd(_p(x), _p(y), _p(idx), K, B, H, W, C, OH, OW, k, s, pad, mode, _f32(x), _s())
    return y, idx


def maxpool_fwd(x, k, s, pad=0):
    return _pool_fwd(x, k, s, pad, 0)


def maxpool_bwd(dy, idx, x_shape, k, s, pad=0):
    K, B, H, W, C = x_shape
    _, _, OH, OW, _ = dy.shape
    dx = torch.empty(x_shape, dtype=dy.dtype, device=dy.device)
    _C.pool_bwd(_p(dy.contiguous()), _p(idx), _p(dx), K, B, H, W, C, OH, OW, k, s, pad, 0, _f32(dy), _s())
    return dx


def avgpool_fwd(x, k, s):
    return _pool_fwd(x, k, s, 0, 1)[0]


def avgpool_bwd(dy, x_shape, k, s):
    K, B, H, W, C = x_shape
    _, _, OH, OW, _ = dy.shape
    dx = torch.empty(x_shape, dtype=dy.dtype, device=dy.device)
    _C.pool_bwd(_p(dy.contiguous()), NULL, _p(dx), K, B, H, W, C, OH, OW, k, s, 0, 1, _f32(dy), _s())
    return dx


def gap_fwd(x):
    K, B, H, W, C = x.shape
    x = x.contiguous()
    y = torch.empty((K, B, C), dtype=x.dtype, device=x.device)
    _C.gap_fwd(_p(x), _p(y), K * B, H * W, C, _f32(x), _s())
    return y


def gap_bwd(dy, x_shape):
    K, B, H, W, C = x_shape
    dx = torch.empty(x_shape, dtype=dy.dtype, device=dy.device)
    _C.gap_bwd(_p(dy.contiguous()), _p(dx), K * B, H * W, C, _f32(dy), _s())
    return dx


# -------------------------------------------------------------------- cross entropy
def ce_fwd_bwd(logits, labels, valid=None):
    K, B, NC = logits.shape
    logits = logits.contiguous()
    lab = labels.to(torch.int32).contiguous()
    v = valid.to(torch.int32).contiguous() if valid is not None else None
    loss = torch.empty(K, dtype=torch.float32, device=logits.device)
    correct = torch.empty(K, dtype=torch.float32, device=logits.device)
    dlogits = torch.empty_like(logits)
    rowbuf = torch.empty((2, K, B), dtype=torch.float32, device=logits.device) if OPTIONS.deterministic else None
    _C.ce_fwd_bwd(_p(logits), _p(lab), _p(v), _p(loss), _p(correct), _p(dlogits), K, B, NC, _f32(logits), _s(),
                  _p(rowbuf))
    return loss, correct, dlogits


# ------------------------------------------------------------------------ embedding
def embedding_fwd(tokens, table, scale: float = 1.0, pe=None):
    """table[tokens] · scale (+ pe[position]) in one pass; pe [L, D] fp32 (L = tokens.shape[-1])."""
    K = tokens.shape[0]
    tok = tokens.to(torch.int32).contiguous()
    t_cs, rep = _client_view(table, K)
    D = table.shape[-1]
    n_tok = tok.numel() // K
    out = torch.empty((*tokens.shape, D), dtype=table.dtype, device=table.device)
    L = tokens.shape[-1]
    if pe is not None:
        pe = pe.to(device=table.device, dtype=torch.float32).contiguous()
        assert pe.shape == (L, D)
    _C.embedding_fwd(_p(tok), _p(table), _p(out), K, n_tok, D, t_cs, rep, _f32(table), _s(), float(scale), _p(pe), L)
    return out


def embedding_bwd(dy, tokens, gtable, scale: float = 1.0):
    K = tokens.shape[0]
    tok = tokens.to(torch.int32).contiguous()
    D = dy.shape[-1]
    gtable.zero_()
    if OPTIONS.deterministic:
        # rows grouped by (client, token) with a stable sort; each group summed in sequence order,
        # in fixed 64-row chunks joined in chunk order (a padding token's thousands of rows per
        # client are summed by many waves, not one)
        V = gtable.shape[1]
        keys = (tok.view(K, -1) + torch.arange(K, device=tok.device, dtype=torch.int32)[:, None] * V).reshape(-1)
        sk, order = torch.sort(keys, stable=True)
        n = keys.numel()
        part = torch.empty(_C.embedding_bwd_part_floats(n, D), dtype=torch.float32, device=dy.device)
        _C.embedding_bwd_sorted(_p(sk.contiguous()), _p(order.to(torch.int32).contiguous()), _p(dy.contiguous()),
                                _p(gtable), n, D, V, gtable.stride(0), _f32(dy), _s(), float(scale), _p(part))
        return
    _C.embedding_bwd(_p(tok), _p(dy.contiguous()), _p(gtable), K, tok.numel() // K, D, gtable.stride(0), _f32(dy), _s(),
                     float(scale))


def seq_mean_fwd(x, lengths):
    """x [..., L, D] → masked mean over L with per-sequence lengths [...]."""
    *lead, L, D = x.shape
    x = x.contiguous()
    S = x.numel() // (L * D)
    ln = lengths.to(torch.int32).reshape(-1).contiguous()
    y = torch.empty((*lead, D), dtype=x.dtype, device=x.device)
    _C.seq_mean_fwd(_p(x), _p(ln), _p(y), S, L, D, _f32(x), _s())
    return y


def seq_mean_bwd(dy, lengths, L: int):
    *lead, D = dy.shape
    S = dy.numel() // D
    ln = lengths.to(torch.int32).reshape(-1).contiguous()
    dx = torch.empty((*lead, L, D), dtype=dy.dtype, device=dy.device)
    _C.seq_mean_bwd(_p(dy.contiguous()), _p(ln), _p(dx), S, L, D, _f32(dy), _s())
    return dx


# ------------------------------------------------------------------------ attention
def _attn_shape(q):
    *lead, L, DH = q.shape
    KB = int(q.shape[0] * q.shape[1])
    H = int(q.shape[2])
    return KB * H, H, L, DH


def _key_valid(key_valid, q):
    if key_valid is None:
        return None
    return key_valid.to(device=q.device, dtype=torch.int32).reshape(-1).contiguous()


def _attn_drop(drop_p: float, drop_seeds, K: int, t):
    if not drop_p:
        return NULL, 0.0
    assert drop_seeds is not None and drop_seeds.numel() == K
    return _p(drop_seeds.to(device=t.device, dtype=torch.int32).contiguous()), float(drop_p)


def attn_fwd(q, k, v, key_valid=None, drop_p: float = 0.0, drop_seeds=None):
    """q,k,v [K,B,Hh,L,dh] bf16 → (o [K,B,Hh,L,dh] bf16, lse [K,B,Hh,L] fp32); flash-style
    kernel (csrc/attention.hip), never materialising the L×L scores. drop_p / drop_seeds [K]:
    dropout on the attention probabilities (MFMA kernels)."""
    q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
    _check(q, q.dtype, name="q")
    assert k.dtype == v.dtype == q.dtype
    KBH, H, L, DH = _attn_shape(q)
    if not _C.attn_supported(L, DH):
        raise NotImplementedError(f"attention kernel: unsupported L={L} dh={DH}")
    kv = _key_valid(key_valid, q)
    o = torch.empty_like(q)
    lse = torch.empty(q.shape[:-1], dtype=torch.float32, device=q.device)
    sp, dp_ = _attn_drop(drop_p, drop_seeds, q.shape[0], q)
    ok = _C.attn_fwd(_p(q), _p(k), _p(v), _p(kv), _p(o), _p(lse), KBH, H, L, DH, _f32(q), _s(), 0, 0, sp,
                     KBH // q.shape[0], dp_)
    if not ok:
        raise NotImplementedError(f"attention kernel: L={L} dh={DH} drop_p={drop_p} not supported")
    return o, lse


def attn_bwd(do, q, k, v, o, lse, key_valid=None, drop_p: float = 0.0, drop_seeds=None):
    do, q, k, v, o = do.contiguous(), q.contiguous(), k.contiguous(), v.contiguous(), o.contiguous()
    KBH, H, L, DH = _attn_shape(q)
    kv = _key_valid(key_valid, q)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    delta = torch.empty(q.shape[:-1], dtype=torch.float32, device=q.device)
    sp, dp_ = _attn_drop(drop_p, drop_seeds, q.shape[0], q)
    ok = _C.attn_bwd(_p(do), _p(q), _p(k), _p(v), _p(o), _p(lse.contiguous()), _p(kv), _p(dq), _p(dk), _p(dv),
                     _p(delta), KBH, H, L, DH, _f32(q), _s(), 0, 0, sp, KBH // q.shape[0], dp_)
    if not ok:
        raise NotImplementedError(f"attention kernel: L={L} dh={DH} drop_p={drop_p} not supported")
    return dq, dk, dv


def attn_packed_supported(L: int, DH: int) -> bool:
    return bool(_C.attn_packed_supported(L, DH))


def attn_fwd_packed(qkv, H: int, key_valid=None, drop_p: float = 0.0, drop_seeds=None):
    """Attention straight from the QKV projection's output rows qkv [K, B, L, 3·D] (q | k | v
    column blocks, heads of dh = D/H inside each): returns o [K, B, L, D] — the out projection's
    input layout — and lse [K, B, H, L]. No permute / contiguous copies."""
    K, B, L, D3 = qkv.shape
    D = D3 // 3
    DH = D // H
    qkv = qkv.contiguous()
    assert qkv.dtype in _DTYPES and attn_packed_supported(L, DH)
    kv = _key_valid(key_valid, qkv)
    o = torch.empty((K, B, L, D), dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty((K, B, H, L), dtype=torch.float32, device=qkv.device)
    base = _p(qkv)
    es = qkv.element_size()
    sp, dp_ = _attn_drop(drop_p, drop_seeds, K, qkv)
    ok = _C.attn_fwd(base, base + D * es, base + 2 * D * es, _p(kv), _p(o), _p(lse), K * B * H, H, L, DH,
                     _f32(qkv), _s(), D3, D, sp, B * H, dp_)
    assert ok
    return o, lse


def attn_bwd_packed(do, qkv, o, lse, H: int, key_valid=None, drop_p: float = 0.0, drop_seeds=None):
    """dqkv [K, B, L, 3·D] (the QKV projection's gradient layout) from do / o [K, B, L, D]."""
    K, B, L, D3 = qkv.shape
    D = D3 // 3
    DH = D // H
    do, o, qkv = do.contiguous(), o.contiguous(), qkv.contiguous()
    kv = _key_valid(key_valid, qkv)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty((K, B, H, L), dtype=torch.float32, device=qkv.device)
    b, g, es = _p(qkv), _p(dqkv), qkv.element_size()
    sp, dp_ = _attn_drop(drop_p, drop_seeds, K, qkv)
    ok = _C.attn_bwd(_p(do), b, b + D * es, b + 2 * D * es, _p(o), _p(lse.contiguous()), _p(kv), g, g + D * es,
                     g + 2 * D * es, _p(delta), K * B * H, H, L, DH, _f32(qkv), _s(), D3, D, sp, B * H, dp_)
    assert ok
    return dqkv


# -------------------------------------------------------------- synthetic data
def synth_images(idx, npix: int, C: int, Cout: int, source32, proto32, salt: int, sqrt6: float, noise: float):
    """Procedural synthetic images (data/datasets.py generator, bit-identical) -> fp32 [n, npix/C*Cout]."""
    n = idx.numel()
    assert idx.dtype == torch.int64 and source32.dtype == torch.int32 and proto32.dtype == torch.float32
    out = torch.empty((n, npix // C * Cout), dtype=torch.float32, device=idx.device)
    _C.synth_images(_p(idx), n, npix, C, Cout, _p(source32), _p(proto32), int(salt) & 0xFFFFFFFFFFFFFFFF,
                    float(sqrt6), float(noise), _p(out), _s())
    return out


# ------------------------------------------------------------- compressed payloads
def _payload_args(p):
    m = p.meta
    return (_p(m.seg_ids), _p(m.seg_off), _p(m.seg_numel), _p(p.bits), _p(p.lo), _p(p.scale), _p(p.seg_byte_off),
            _p(p.row_off))


def quant_pack(p, x, seeds):
    """csrc/compress.hip: codes of rows x [K, P] fp32 into p.codes (see ops/compress.py)."""
    K, P = x.shape
    assert x.dtype == torch.float32 and x.stride(1) == 1 and P == p.meta.P and K == p.K
    sd = _seeds_dev(seeds) if seeds is not None else None
    m = p.meta
    _C.quant_pack(_p(x), x.stride(0), _p(m.seg_ids), _p(m.seg_off), _p(m.seg_numel), _p(p.bits), _p(p.lo),
                  _p(p.scale), _p(p.seg_byte_off), _p(p.row_off), K, m.nseg, P, int(seeds is not None), _p(sd),
                  _p(p.codes), _s())


def quant_unpack(p, out):
    _C.quant_unpack(_p(p.codes), *_payload_args(p), p.K, p.meta.nseg, p.meta.P, _p(out), out.stride(0), _s())


def quant_unpack_acc(p, w, acc):
    assert w.dtype == torch.float64 and w.numel() == p.K and acc.is_contiguous()
    _C.quant_unpack_acc(_p(p.codes), *_payload_args(p), p.K, p.meta.nseg, p.meta.P, _p(w), _p(acc), _s())


# ---------------------------------------------------------------------- GNN sampling
def _hmix_int(h: int) -> int:
    h &= 0x7FFFFFFF
    h ^= h >> 16
    h = (h * 0x45D9F3B) & 0x7FFFFFFF
    h ^= h >> 16
    h = (h * 0x45D9F3B) & 0x7FFFFFFF
    return h ^ (h >> 16)


def neighbor_sample(rowptr32, col32, owner32, is_val_u8, nodes, clients, fanout: int, seed: int):
    """csrc/graph.hip: per frontier row the `fanout` (<= 32) hash-smallest in-neighbours ->
    (neighbour ids, frontier row) of the kept samples, row-major (data/graph.py rule)."""
    assert 0 < fanout <= 32
    n = nodes.numel()
    nodes = nodes.long().contiguous()
    clients = clients.long().contiguous()
    assert rowptr32.dtype == col32.dtype == owner32.dtype == torch.int32 and is_val_u8.dtype == torch.uint8
    assert nodes.device == rowptr32.device and clients.shape == nodes.shape
    out = torch.empty((n, fanout), dtype=torch.int32, device=nodes.device)
    cnt = torch.empty(n, dtype=torch.int32, device=nodes.device)
    _C.neighbor_sample(_p(rowptr32), _p(col32), _p(owner32), _p(is_val_u8), _p(nodes), _p(clients), n, fanout,
                       _hmix_int(seed), _p(out), _p(cnt), _s())
    keep = out >= 0
    rows = torch.arange(n, device=nodes.device).unsqueeze(1).expand(n, fanout)
    return out[keep].long(), rows[keep]


# ----------------------------------------------------------------------------- SpMM
def spmm(rowptr, col, val, x):
    """CSR (shared graph, fp32 values) times per-client dense x [K,Nx,F] → [K,N,F] (x's dtype)."""
    x = x.contiguous()
    f32 = _f32(x)
    K, Nx, F = x.shape
    N = rowptr.numel() - 1
    y = torch.empty((K, N, F), dtype=x.dtype, device=x.device)
    rp = rowptr.to(torch.int32).contiguous()
    cl = col.to(torch.int32).contiguous()
    vl = val.to(torch.float32).contiguous()
    _C.spmm(_p(rp), _p(cl), _p(vl), _p(x), _p(y), K, N, Nx, F, Nx * F, N * F, f32, _s())
    return y


# ---------------------------------------------------------------- optimiser / FL math
def _row_args(theta):
    assert theta.dtype == torch.float32 and theta.stride(1) == 1
    K, P = theta.shape
    assert P % 16 == 0, "flat buffers are padded to 16 elements"
    return K, P, theta.stride(0)


def sgd_step(theta, grad, mom, lr, active, weight_decay, momentum, dampening, nesterov, first_step, shadow=None,
             split=None):
    """`split` [K, 2, P] bf16: the rows' (hi, lo) weight planes, rewritten with the new θ (the
    fp32 convolutions read them instead of splitting the weights in every workgroup)."""
    K, P, ld = _row_args(theta)
    assert grad.stride(0) == ld and mom.stride(0) == ld
    if shadow is not None:
        assert shadow.stride(0) == ld and shadow.dtype == BF16
    if split is not None:
        assert split.shape == (K, 2, P) and split.is_contiguous() and split.dtype == BF16 and ld == P
    _C.sgd_step(_p(theta), _p(grad), _p(mom), _p(shadow), _p(split), _p(lr.float().contiguous()),
                _p(active.to(torch.uint8).contiguous()), _p(first_step.to(torch.uint8).contiguous()), K, P, ld,
                float(weight_decay), float(momentum), float(dampening), int(nesterov), _s())


def sgd_step_seg(theta, grad, mom, lr, active, weight_decay, momentum, dampening, nesterov, first_step, split,
                 seg_table):
    """sgd_step over the spans of `seg_table` [n, 2] int64 (first float4 of the row, count): the
    parameters whose wgrad kernels did not already step them (engine.params.FusedSGD)."""
    K, P, ld = _row_args(theta)
    assert grad.stride(0) == ld and mom.stride(0) == ld
    assert split.shape == (K, 2, P) and split.is_contiguous() and split.dtype == BF16 and ld == P
    assert seg_table.dtype == torch.int64 and seg_table.is_contiguous() and seg_table.shape[1] == 2
    _C.sgd_step_seg(_p(theta), _p(grad), _p(mom), _p(split), _p(lr.float().contiguous()),
                    _p(active.to(torch.uint8).contiguous()), _p(first_step.to(torch.uint8).contiguous()), K, ld,
                    float(weight_decay), float(momentum), float(dampening), int(nesterov), _p(seg_table),
                    seg_table.shape[0], _s())


def adam_step(theta, grad, m, v, lr, active, step, beta1, beta2, eps, weight_decay, shadow=None):
    K, P, ld = _row_args(theta)
    _C.adam_step(_p(theta), _p(grad), _p(m), _p(v), _p(shadow), _p(lr.float().contiguous()),
                 _p(active.to(torch.uint8).contiguous()), _p(step.float().contiguous()), K, P, ld, beta1, beta2, eps,
                 weight_decay, _s())


def split_rows(theta, split):
    """split[k] = (bf16 hi, bf16 lo) planes of theta[k] (x = hi + lo, RNE hi)."""
    K, P, ld = _row_args(theta)
    assert split.shape == (K, 2, P) and split.is_contiguous() and split.dtype == BF16 and ld == P
    _C.split_rows(_p(theta), _p(split), K, P, ld, _s())


def _wsplit_args(w_split, w):
    """(pointer, client stride, hi→lo plane distance) of a weight's pre-split planes: `w_split`
    is the hi-plane view of the weight inside a [K, 2, P] split buffer, same shape as `w`."""
    if w_split is None:
        return NULL, 0, 0
    assert w_split.dtype == BF16 and w_split.shape == w.shape, (w_split.shape, w.shape)
    base = w_split._base if w_split._base is not None else w_split
    assert base.dim() == 3 and base.shape[1] == 2, "w_split must view a [K, 2, P] split buffer"
    return _p(w_split), w_split.stride(0), base.stride(1)


def broadcast_rows(theta_rows, src, shadow_rows=None):
    K, P, ld = _row_args(theta_rows)
    src = src.float().contiguous()
    assert src.numel() == P
    _C.broadcast_rows(_p(theta_rows), _p(shadow_rows), _p(src), K, P, ld, _s())


def delta_rows(theta_rows, base, out=None):
    K, P, ld = _row_args(theta_rows)
    if out is None:
        out = torch.empty_like(theta_rows)
    assert out.stride(0) == ld or out.data_ptr() == theta_rows.data_ptr()
    _C.delta_rows(_p(theta_rows), _p(base.float().contiguous()), _p(out), K, P, ld, _s())
    return out


def weighted_sum(x, w, out=None):
    """out (fp64 [P], zeros if None) += Σ_k w_k x[k, :] — fp64 accumulation, fp64 result."""
    K, P, ld = _row_args(x)
    if out is None:
        out = torch.zeros(P, dtype=torch.float64, device=x.device)
    assert out.dtype == torch.float64 and out.is_contiguous() and out.numel() == P
    _C.weighted_sum(_p(x), _p(w.double().contiguous()), _p(out), K, P, ld, _s())
    return out


def mix_rows(x, w, out_dtype=BF16):
    """[M, P] = W[M, K] · x[K, P]: subset models for Shapley utilities, emitted in the eval
    compute dtype (bf16 or fp32) by one native pass that reads each x row once per 32 models;
    K > 256 is split into 256-row chunks (fp32 partial sums, one rounding at the end)."""
    K, P, ld = _row_args(x)
    M = w.shape[0]
    assert w.shape == (M, K) and out_dtype in _DTYPES
    w = w.float().to(x.device).contiguous()
    if K > 256:
        acc = None
        for k0 in range(0, K, 256):
            part = mix_rows(x[k0:k0 + 256], w[:, k0:k0 + 256].contiguous(), F32)
            acc = part if acc is None else acc.add_(part)
        return acc.to(out_dtype)
    out = torch.empty((M, P), dtype=out_dtype, device=x.device)
    if M:
        _C.mix_rows(_p(x), _p(w), _p(out), K, M, P, ld, P, int(out_dtype == F32), _s())
    return out


def masked_weighted_sum(x, mask, w, num=None, den=None):
    """(num, den) fp64 [P] += (Σ_k w_k m_k x_k, Σ_k w_k m_k)."""
    K, P, ld = _row_args(x)
    mask = mask.to(torch.uint8)
    assert mask.is_contiguous() and mask.shape == (K, P) and ld == P
    num = torch.zeros(P, dtype=torch.float64, device=x.device) if num is None else num
    den = torch.zeros(P, dtype=torch.float64, device=x.device) if den is None else den
    assert num.dtype == den.dtype == torch.float64
    _C.masked_weighted_sum(_p(x), _p(mask), _p(w.double().contiguous()), _p(num), _p(den), K, P, ld, _s())
    return num, den


def _seeds_dev(seeds) -> torch.Tensor:
    return torch.tensor([s & 0xFFFFFFFF for s in seeds], dtype=torch.int64).to(torch.int32).to("cuda")


def dropout_mask(shape, p, seeds):
    K, P = shape
    assert len(seeds) == K
    m = torch.empty(shape, dtype=torch.uint8, device="cuda")
    sd = _seeds_dev(seeds)
    _C.dropout_mask(_p(m), K, P, float(p), _p(sd), _s())
    return m.bool()


def block_sq_norms(x, block_offsets, block_ids):
    K, P, ld = _row_args(x)
    nb = int(block_offsets.numel()) - 1
    out = torch.empty((K, nb), dtype=torch.float32, device=x.device)
    _C.block_sq_norms(_p(x), _p(block_ids.to(torch.int32).contiguous()), _p(out), K, P, ld, nb, _s())
    return out


def stochastic_qdq(x, seg_ids, nseg, seeds, levels):
    K, P, ld = _row_args(x)
    assert len(seeds) == K
    mn = torch.full((K, nseg), float("inf"), dtype=torch.float32, device=x.device)
    mx = torch.full((K, nseg), float("-inf"), dtype=torch.float32, device=x.device)
    seg = seg_ids.to(torch.int32).contiguous()
    out = x.contiguous().clone()
    ld = out.stride(0)
    sd = _seeds_dev(seeds)
    _C.seg_minmax(_p(out), _p(seg), _p(mn), _p(mx), K, P, ld, nseg, _s())
    # QSGD code (ops.quant.qsgd_range): the kernel's affine form with range [−‖x‖, ‖x‖] and codes
    # 0..2s (scale (2‖x‖)/(2s) = ‖x‖/s exactly)
    from .quant import qsgd_range

    lo, _, qmax = qsgd_range(mn, mx, levels)
    lo = lo.contiguous()
    hi = (-lo).contiguous()
    _C.stochastic_qdq(_p(out), _p(seg), _p(lo), _p(hi), K, P, ld, nseg, _p(sd), qmax, _s())
    return out


def seg_minmax(x, seg_ids, nseg):
    K, P, ld = _row_args(x)
    mn = torch.full((K, nseg), float("inf"), dtype=torch.float32, device=x.device)
    mx = torch.full((K, nseg), float("-inf"), dtype=torch.float32, device=x.device)
    _C.seg_minmax(_p(x), _p(seg_ids.to(torch.int32).contiguous()), _p(mn), _p(mx), K, P, ld, nseg, _s())
    return mn, mx


def seg_sq_sums(x, seg_ids, nseg):
    """Σx² per (row, segment); segments are 16-element aligned layout tensors."""
    K, P, ld = _row_args(x)
    out = torch.empty((K, nseg), dtype=torch.float32, device=x.device)
    _C.block_sq_norms(_p(x), _p(seg_ids.to(torch.int32).contiguous()), _p(out), K, P, ld, nseg, _s())
    return out


def nnadq_qdq(x, seg_ids, lo, scale, levels):
    K, P, ld = _row_args(x)
    out = x.contiguous().clone()
    nseg = lo.shape[1]
    _C.nnadq_qdq(_p(out), _p(seg_ids.to(torch.int32).contiguous()), _p(lo.contiguous()), _p(scale.contiguous()),
                 _p(levels.float().contiguous()), K, P, out.stride(0), nseg, _s())
    return out


def sign_pack(g):
    K, P, ld = _row_args(g)
    out = torch.empty((K, (P + 7) // 8), dtype=torch.uint8, device=g.device)
    _C.sign_pack(_p(g), _p(out), K, P, ld, _s())
    return out


def sign_vote(packed, P, active=None):
    K = packed.shape[0]
    votes = torch.empty(P, dtype=torch.int32, device=packed.device)
    a = active.to(torch.uint8).contiguous() if active is not None else None
    _C.sign_vote(_p(packed.contiguous()), _p(a), _p(votes), K, P, _s())
    return votes


def gather_rows(src, idx):
    """src [N, ...] contiguous (rows a multiple of 16 B), idx int -> [len(idx), ...]"""
    row_bytes = src[0].numel() * src.element_size()
    assert row_bytes % 16 == 0 and src.is_contiguous()
    i32 = idx.reshape(-1).to(torch.int32).contiguous()
    out = torch.empty((i32.numel(), *src.shape[1:]), dtype=src.dtype, device=src.device)
    _C.gather_rows(_p(src), _p(i32), _p(out), i32.numel(), row_bytes, _s())
    return out
