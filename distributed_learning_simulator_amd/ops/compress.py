"""Materialised compressed payloads: the wire buffers quantising endpoints actually send.

Reference `topology/quantized_endpoint.py:29-34,58-68,86-116`: the client endpoint REPLACES the
uploaded tensors with their quantised form and the server dequantises what it receives;
`get_message_size` then counts the quantised tensors. Here the quantiser writes one ragged
uint8 buffer per cohort:
- client k's bytes start at `row_off[k]`;
- tensor s of client k occupies ceil(bits·numel / 8) bytes at `seg_byte_off[k, s]`, with b-bit
  codes packed LSB-first in 8-element groups (csrc/compress.hip);
- per sent tensor there is the fp32 norm (stochastic) or fp32 `lo` and `scale` + one uint8
  bit-width (NNADQ).

Wire bytes per client are the sizes of those buffers (`QuantPayload.row_bytes`), not a formula.
The server either decodes to dense rows or, for FedAvg-style weighted sums, dequantises inside
the fp64 accumulation kernel (`accumulate`: no dense [K, P] materialisation).

Codes:
- stochastic (FedPAQ / fed_obd_sq, QSGD with 255 signed levels = 8 bits, ops.quant): lo = −‖x‖,
  scale = ‖x‖/127, q = clamp(floor((x − lo)/scale + u), 0, 254), with u the shared per-element
  hash uniform (`fl.uniform_rows`; unbiased); per sent tensor only the fp32 norm travels;
- NNADQ (FedOBD): round-to-nearest with the per-tensor adaptive bit-width of `quant.nnadq_bits`.

x̂ = lo + q·scale; the CPU path below writes the identical buffer and decodes to identical bits.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

from . import backend, ref
from .fl import uniform_rows


@dataclass
class LayoutMeta:
    seg_ids: torch.Tensor  # int32 [P] (padding = nseg)
    seg_off: torch.Tensor  # int64 [nseg] flat offsets (16-element aligned)
    seg_numel: torch.Tensor  # int64 [nseg]
    nseg: int
    P: int

    @classmethod
    def of(cls, layout, device) -> "LayoutMeta":
        off = torch.tensor([e.offset for e in layout.entries], dtype=torch.int64, device=device)
        numel = torch.tensor([e.numel for e in layout.entries], dtype=torch.int64, device=device)
        assert layout.padded_size % 8 == 0 and all(e.offset % 8 == 0 for e in layout.entries)
        return cls(layout.segment_ids(device), off, numel, len(layout.entries), layout.padded_size)


@dataclass
class QuantPayload:
    kind: str  # "sq8" | "nnadq"
    codes: torch.Tensor  # uint8 [total bytes]
    row_off: torch.Tensor  # int64 [K + 1]
    seg_byte_off: torch.Tensor  # int64 [K, nseg]
    bits: torch.Tensor  # uint8 [K, nseg] (0: tensor not sent)
    lo: torch.Tensor  # fp32 [K, nseg]
    scale: torch.Tensor  # fp32 [K, nseg]
    meta: LayoutMeta
    row_off_host: list

    @property
    def K(self) -> int:
        return self.bits.shape[0]

    def row_bytes(self) -> list[int]:
        """Per client: code bytes + the metadata tensors of the tensors it sent."""
        per_seg = 9 if self.kind == "nnadq" else 4  # lo, scale, bit-width | the QSGD norm
        sent = (self.bits > 0).sum(1).cpu().tolist()
        off = self.row_off_host
        return [off[k + 1] - off[k] + per_seg * sent[k] for k in range(self.K)]

    def decode(self, out: torch.Tensor | None = None) -> torch.Tensor:
        K, P = self.K, self.meta.P
        if out is None:
            out = torch.empty((K, P), dtype=torch.float32, device=self.codes.device)
        assert out.shape == (K, P) and out.dtype == torch.float32 and out.stride(1) == 1
        if backend.get(out) is ref:
            out.copy_(_unpack_torch(self))
            return out
        from . import hip

        hip.quant_unpack(self, out)
        return out

    def accumulate(self, acc: torch.Tensor, w: torch.Tensor) -> None:
        """acc [P] fp64 += Σ_k w[k]·x̂_k (the server's FedAvg accumulation, fused)."""
        assert acc.dtype == torch.float64 and acc.shape == (self.meta.P,)
        w = w.to(acc.device, torch.float64).contiguous()
        if backend.get(acc) is ref:
            acc += (w[:, None] * _unpack_torch(self).double()).sum(0)
            return
        from . import hip

        hip.quant_unpack_acc(self, w, acc)


# ------------------------------------------------------------------ packing
def _segment_stats(x, meta: LayoutMeta):
    be = backend.get(x)
    if be is not ref:
        mn, mx = be.seg_minmax(x, meta.seg_ids, meta.nseg + 1)
        sq = be.seg_sq_sums(x, meta.seg_ids, meta.nseg + 1)
    else:
        K = x.shape[0]
        idx = meta.seg_ids.long().unsqueeze(0).expand(K, -1)
        mn = torch.full((K, meta.nseg + 1), float("inf"), device=x.device)
        mx = torch.full((K, meta.nseg + 1), float("-inf"), device=x.device)
        mn.scatter_reduce_(1, idx, x.float(), reduce="amin", include_self=True)
        mx.scatter_reduce_(1, idx, x.float(), reduce="amax", include_self=True)
        sq = torch.zeros((K, meta.nseg + 1), device=x.device)
        sq.index_add_(1, meta.seg_ids.long(), x.float() ** 2)
    return mn[:, : meta.nseg], mx[:, : meta.nseg], sq[:, : meta.nseg]


def _offsets(bits: torch.Tensor, meta: LayoutMeta):
    seg_bytes = (bits.long() * meta.seg_numel[None, :] + 7) // 8  # [K, nseg]
    seg_byte_off = torch.cumsum(seg_bytes, 1) - seg_bytes
    row_bytes = seg_bytes.sum(1)
    row_off = torch.zeros(bits.shape[0] + 1, dtype=torch.int64, device=bits.device)
    row_off[1:] = torch.cumsum(row_bytes, 0)
    return seg_byte_off.contiguous(), row_off


def _pack(kind: str, x: torch.Tensor, meta: LayoutMeta, bits, lo, scale, seeds) -> QuantPayload:
    seg_byte_off, row_off = _offsets(bits, meta)
    host = row_off.cpu().tolist()
    codes = torch.zeros(host[-1], dtype=torch.uint8, device=x.device)
    p = QuantPayload(kind, codes, row_off, seg_byte_off, bits.to(torch.uint8).contiguous(), lo.float().contiguous(),
                     scale.float().contiguous(), meta, host)
    if backend.get(x) is ref:
        _pack_torch(p, x, seeds)
    else:
        from . import hip

        hip.quant_pack(p, x, seeds)
    return p


def pack_stochastic(x: torch.Tensor, meta: LayoutMeta, seeds: list[int], seg_mask: torch.Tensor | None = None,
                    levels: int = 255) -> QuantPayload:
    """255-level QSGD stochastic quantisation of rows x [K, P] into an 8-bit payload."""
    from .quant import qsgd_range

    assert levels == 255, "the stochastic payload packs 8-bit codes"
    mn, mx, _ = _segment_stats(x, meta)
    lo, scale, _ = qsgd_range(mn, mx, levels)
    bits = torch.full_like(mn, 8, dtype=torch.uint8)
    if seg_mask is not None:
        bits = torch.where(seg_mask.to(bits.device), bits, torch.zeros_like(bits))
    return _pack("sq8", x, meta, bits, lo, scale, seeds)


def pack_nnadq(x: torch.Tensor, meta: LayoutMeta, weight: float, seg_mask: torch.Tensor | None = None) -> QuantPayload:
    """NNADQ: per-tensor adaptive bit-width (quant.nnadq_bits), round-to-nearest codes."""
    from .quant import nnadq_bits

    mn, mx, sq = _segment_stats(x, meta)
    rms = (sq / meta.seg_numel[None, :].float().clamp(min=1)).sqrt()
    b = nnadq_bits(mn, mx, rms, weight)
    levels = 2 ** b - 1
    lo = torch.where(torch.isfinite(mn), mn, torch.zeros_like(mn))
    scale = ((mx - mn) / levels).clamp(min=1e-30)
    scale = torch.where(torch.isfinite(scale), scale, torch.ones_like(scale))
    bits = b.to(torch.uint8)
    if seg_mask is not None:
        bits = torch.where(seg_mask.to(bits.device), bits, torch.zeros_like(bits))
    return _pack("nnadq", x, meta, bits, lo, scale, None)


# ------------------------------------------------------------------ CPU oracle
def _group_tables(p: QuantPayload):
    """Per flat 8-element group: its tensor, element index and valid count."""
    meta = p.meta
    t = torch.arange(meta.P // 8, device=p.codes.device)
    s = meta.seg_ids.long()[t * 8]
    real = s < meta.nseg
    t, s = t[real], s[real]
    j0 = t * 8 - meta.seg_off[s]
    n = torch.clamp(meta.seg_numel[s] - j0, max=8)
    return t, s, j0, n


def _codes_torch(p: QuantPayload, x: torch.Tensor, seeds) -> torch.Tensor:
    K = x.shape[0]
    sid = p.meta.seg_ids.long().clamp(max=p.meta.nseg - 1)
    lo, sc = p.lo[:, sid], p.scale[:, sid]
    # QSGD codes stop at 2s = 2^b − 2 (255 signed levels); NNADQ uses all 2^b levels
    top = (2 ** p.bits.long()[:, sid] - (2 if p.kind == "sq8" else 1)).float()
    r = (x.float() - lo) / sc
    if p.kind == "sq8":
        q = torch.floor(r + uniform_rows(seeds, x.shape[1], x.device))
    else:
        q = torch.round(r)
    q = torch.minimum(q.clamp(min=0), top)
    return q.long().view(K, -1)


def _pack_torch(p: QuantPayload, x: torch.Tensor, seeds) -> None:
    q = _codes_torch(p, x, seeds)  # [K, P]
    t, s, j0, n = _group_tables(p)
    K = x.shape[0]
    lane = torch.arange(8, device=x.device)
    for k in range(K):
        b = p.bits[k].long()[s]  # [G]
        sel = b > 0
        tt, ss, jj, nn, bb = t[sel], s[sel], j0[sel], n[sel], b[sel]
        codes = q[k].view(-1, 8)[tt]  # [G, 8]
        codes = torch.where(lane[None, :] < nn[:, None], codes, torch.zeros_like(codes))
        word = (codes << (lane[None, :] * bb[:, None])).sum(1)  # disjoint bit fields
        base = p.row_off[k] + p.seg_byte_off[k, ss] + (jj // 8) * bb
        nbytes = (nn * bb + 7) // 8
        for i in range(8):
            m = i < nbytes
            p.codes[base[m] + i] = ((word[m] >> (8 * i)) & 0xFF).to(torch.uint8)


def _unpack_torch(p: QuantPayload) -> torch.Tensor:
    K, P = p.K, p.meta.P
    out = torch.zeros((K, P), dtype=torch.float32, device=p.codes.device)
    t, s, j0, n = _group_tables(p)
    lane = torch.arange(8, device=p.codes.device)
    for k in range(K):
        b = p.bits[k].long()[s]
        sel = b > 0
        tt, ss, jj, nn, bb = t[sel], s[sel], j0[sel], n[sel], b[sel]
        base = p.row_off[k] + p.seg_byte_off[k, ss] + (jj // 8) * bb
        nbytes = (nn * bb + 7) // 8
        word = torch.zeros_like(base)
        for i in range(8):
            m = i < nbytes
            word[m] |= p.codes[base[m] + i].long() << (8 * i)
        q = (word[:, None] >> (lane[None, :] * bb[:, None])) & ((1 << bb[:, None]) - 1)
        v = p.lo[k, ss][:, None] + q.float() * p.scale[k, ss][:, None]
        v = torch.where(lane[None, :] < nn[:, None], v, torch.zeros_like(v))
        out[k].view(-1, 8)[tt] = v
    return out
