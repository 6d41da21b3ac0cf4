"""Materialised compressed payloads (ops/compress.py, csrc/compress.hip): the packed wire
buffers decode to exactly what the in-place quantisers produce, the reported bytes are the
buffers' sizes, unsent tensors cost nothing, the fused dequantise-accumulate equals the dense
weighted sum, and the HIP packer writes the CPU oracle's bytes bit for bit."""

import pytest
import torch

from distributed_learning_simulator_amd.engine.params import ParamLayout
from distributed_learning_simulator_amd.ops import compress, fl, quant


def _layout():
    lay = ParamLayout()
    for name, shape in (("a", (37,)), ("b", (8, 9)), ("c", (3,)), ("d", (130,)), ("e", (16,))):
        lay.add(name, shape)
    return lay


def _rows(lay, K=4, dev="cpu", seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(K, lay.padded_size, generator=g) * torch.linspace(0.01, 3, lay.padded_size)
    x[:, ~lay.valid_mask()] = 0
    return x.to(dev)


def test_stochastic_payload_roundtrip_and_bytes():
    lay = _layout()
    meta = compress.LayoutMeta.of(lay, "cpu")
    x = _rows(lay)
    seeds = fl.row_seeds(7, [3, 1, 9, 4])
    p = compress.pack_stochastic(x, meta, seeds)
    dq_ref, wire_ref = quant.stochastic_quantize(x, lay.segment_ids(), lay.segment_sizes(), seeds)
    torch.testing.assert_close(p.decode(), dq_ref, rtol=0, atol=0)
    n = lay.num_params
    assert p.codes.numel() == 4 * n  # one byte per real element, padding not sent
    assert p.row_bytes() == [n + 4 * len(lay.entries)] * 4 == wire_ref
    # QSGD code: 255 signed levels of the per-tensor max-abs norm, unbiased
    dq = p.decode()
    for e in lay.entries:
        seg = x[:, e.offset : e.offset + e.numel]
        step = seg.abs().amax(1, keepdim=True) / 127
        assert ((dq[:, e.offset : e.offset + e.numel] - seg).abs() <= step * 1.0001 + 1e-30).all()


def test_qsgd_code_unbiased_signed_levels():
    """QSGD form: codes are 255 signed levels of the per-tensor max-abs norm — the
    extremes ±‖x‖ are exact, zero is a level, signs are kept — and E[Q(x)] = x over seeds."""
    lay = _layout()
    x = _rows(lay, K=2, seed=3)
    seg, sizes = lay.segment_ids(), lay.segment_sizes()
    reps = torch.stack([quant.stochastic_quantize(x, seg, sizes, fl.row_seeds(s, [0, 1]))[0] for s in range(200)])
    for e in lay.entries:
        sl = slice(e.offset, e.offset + e.numel)
        xs, q = x[:, sl], reps[:, :, sl]
        norm = xs.abs().amax(1, keepdim=True)
        levels = q / (norm / 127)
        assert torch.allclose(levels, levels.round(), atol=1e-3)  # on the grid
        assert levels.abs().max() <= 127 + 1e-3
        assert ((q == 0) | (torch.sign(q) == torch.sign(xs))).all()  # sign kept (or rounded to 0)
        err = (q.mean(0) - xs).abs().max() / norm.max()
        assert err < 0.003, err  # unbiased: the mean of 200 draws sits well inside one level (norm / 127)


def test_nnadq_payload_roundtrip_bits_and_mask():
    lay = _layout()
    meta = compress.LayoutMeta.of(lay, "cpu")
    x = _rows(lay, seed=1)
    p = compress.pack_nnadq(x, meta, 0.01)
    dq_ref, _, _ = quant.nnadq_quantize(x, lay.segment_ids(), lay.segment_sizes(), 0.01)
    torch.testing.assert_close(p.decode(), dq_ref, rtol=0, atol=0)
    bits = p.bits.long()
    numel = meta.seg_numel[None, :]
    assert bits.min() >= 1 and bits.max() <= 8 and bits.float().mean() < 8  # adaptive widths
    code_bytes = ((bits * numel + 7) // 8).sum(1)
    assert p.codes.numel() == int(code_bytes.sum())
    assert p.row_bytes() == (code_bytes + 9 * len(lay.entries)).tolist()
    # tensors a client does not send (FedOBD block subsets): no bytes, decode to zero
    mask = torch.ones(4, meta.nseg, dtype=torch.bool)
    mask[0, 1] = mask[2, 3] = False
    pm = compress.pack_nnadq(x, meta, 0.01, mask)
    dm = pm.decode()
    e = lay.entries
    assert torch.all(dm[0, e[1].offset : e[1].offset + e[1].numel] == 0)
    assert torch.all(dm[2, e[3].offset : e[3].offset + e[3].numel] == 0)
    assert pm.row_bytes()[0] < p.row_bytes()[0] and pm.row_bytes()[1] == p.row_bytes()[1]


def test_fused_accumulate_equals_dense_weighted_sum():
    lay = _layout()
    meta = compress.LayoutMeta.of(lay, "cpu")
    x = _rows(lay, seed=2)
    w = torch.tensor([3.0, 1.0, 7.0, 2.0], dtype=torch.float64)
    for p in (compress.pack_nnadq(x, meta, 0.001), compress.pack_stochastic(x, meta, [1, 2, 3, 4])):
        acc = torch.zeros(lay.padded_size, dtype=torch.float64)
        p.accumulate(acc, w)
        exp = (w[:, None] * p.decode().double()).sum(0)
        torch.testing.assert_close(acc, exp, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sq8", "nnadq", "nnadq_masked"])
def test_hip_payload_matches_cpu_bit_for_bit(hip, kind):
    from distributed_learning_simulator_amd.engine.params import ParamLayout as PL

    lay = PL()
    for i, shape in enumerate([(64, 3, 3, 3), (64,), (10, 513), (10,), (1000,), (7,)]):
        lay.add(f"t{i}", shape)
    K = 5
    x = _rows(lay, K, seed=3)
    meta_c, meta_g = compress.LayoutMeta.of(lay, "cpu"), compress.LayoutMeta.of(lay, "cuda")
    mask = torch.rand(K, meta_c.nseg, generator=torch.Generator().manual_seed(0)) > 0.3
    seeds = fl.row_seeds(11, list(range(K)))
    if kind == "sq8":
        pc, pg = compress.pack_stochastic(x, meta_c, seeds), compress.pack_stochastic(x.cuda(), meta_g, seeds)
    else:
        m = mask if kind == "nnadq_masked" else None
        pc = compress.pack_nnadq(x, meta_c, 0.003, m)
        pg = compress.pack_nnadq(x.cuda(), meta_g, 0.003, None if m is None else m.cuda())
    assert torch.equal(pg.bits.cpu(), pc.bits) and pg.row_bytes() == pc.row_bytes()
    assert torch.equal(pg.codes.cpu(), pc.codes)  # identical wire bytes
    assert torch.equal(pg.decode().cpu(), pc.decode())
    w = torch.rand(K, dtype=torch.float64) * 100
    ag = torch.zeros(lay.padded_size, dtype=torch.float64, device="cuda")
    pg.accumulate(ag, w.cuda())
    ac = torch.zeros(lay.padded_size, dtype=torch.float64)
    pc.accumulate(ac, w)
    torch.testing.assert_close(ag.cpu(), ac, rtol=1e-12, atol=1e-12)
