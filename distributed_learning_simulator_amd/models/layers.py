"""Cohort layer library: modules whose parameters live in a flat `ParamLayout` and whose
forward runs the client-batched primitives of `ops.functional` for all K clients at once.

Module/param naming mirrors the equivalent `torch.nn` model's `state_dict` so messages,
checkpoints and FedOBD block discovery see the same names the reference would
(`method/fed_obd/obd_algorithm.py:8-22` discovers blocks over module types; `kind` plays
the role of the module type here).
"""

from __future__ import annotations

import torch

from ..engine.params import ParamLayout
from ..ops import functional as Fn


class RunCtx:
    """Per-pass context: bound params + per-client valid sample counts."""

    def __init__(self, params, valid: torch.Tensor | None = None, training: bool = True,
                 client_ids: torch.Tensor | None = None, seed: int = 0):
        self.P = params
        self.valid = valid  # [K] int32 number of real samples of each client this step
        self.training = training
        self.client_ids = client_ids  # [K] int64: dropout masks keyed by client, not cohort row
        self.seed = seed  # per training step
        self._site = 0
        self._rows_cache: dict[int, torch.Tensor] = {}

    def dropout_seeds(self) -> torch.Tensor:
        """[K] int32 mask seeds of the next dropout site of this step: hash(step seed, site,
        client id), so a client's masks do not depend on the rank / cohort row hosting it."""
        from ..ops.fl import _mix

        self._site += 1
        ids = self.client_ids
        if ids is None:
            ids = torch.arange(self.P.K, device=self.P.compute.device)
        h = _mix(ids.long(), (self.seed * 1_000_003 + self._site * 7919) & 0xFFFFFFFF)
        return (h - (h >= 2**31).long() * 2**32).to(torch.int32).contiguous()

    @property
    def token(self):
        return self.P.token

    def valid_rows(self, rows_per_sample: int):
        if self.valid is None:
            return None
        r = self._rows_cache.get(rows_per_sample)
        if r is None:
            r = (self.valid * rows_per_sample).to(torch.int32)
            self._rows_cache[rows_per_sample] = r
        return r


class Module:
    kind = "module"

    def __init__(self):
        self.name = ""
        self._named: list[tuple[str, "Module"]] = []

    @property
    def children(self) -> list["Module"]:
        return [m for _, m in self._named]

    def child(self, name: str, m: "Module") -> "Module":
        self._named.append((name, m))
        setattr(self, name, m)
        return m

    def assign_names(self, prefix: str = "") -> None:
        self.name = prefix
        for local, c in self._named:
            c.assign_names(f"{prefix}.{local}" if prefix else local)

    def register(self, layout: ParamLayout) -> None:
        for c in self.children:
            c.register(layout)

    def own_params(self) -> list[str]:
        return []

    def all_params(self) -> list[str]:
        out = list(self.own_params())
        for c in self.children:
            out.extend(c.all_params())
        return out

    def modules(self):
        yield self
        for c in self.children:
            yield from c.modules()


class Seq(Module):
    kind = "Sequential"

    def __init__(self, *mods):
        super().__init__()
        for i, m in enumerate(mods):
            self.child(str(i), m)

    def forward(self, x, ctx):
        for m in self.children:
            x = m.forward(x, ctx)
        return x


class ReLU(Module):
    kind = "ReLU"

    def forward(self, x, ctx):
        return torch.relu(x)


class Conv2d(Module):
    kind = "Conv2d"

    def __init__(self, cin, cout, k, stride=1, pad=0, bias=False):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.pad, self.bias = cin, cout, k, stride, pad, bias

    def register(self, layout):
        fan_in = self.cin * self.k * self.k
        self.w = layout.add(f"{self.name}.weight", (self.cout, self.k, self.k, self.cin),
                            "kaiming_conv", fan_in, self.name).name
        self.b = layout.add(f"{self.name}.bias", (self.cout,), "uniform_bias", fan_in, self.name).name if self.bias else None

    def own_params(self):
        return [self.w] + ([self.b] if self.b else [])

    def forward(self, x, ctx, link=None, stats=None, donor=None):
        P = ctx.P
        b = P.w(self.b) if self.b else None
        gb = P.g(self.b) if self.b else None
        return Fn.conv2d(x, ctx.token, P.w(self.w), P.g(self.w), self.stride, self.pad, b, gb, link=link, stats=stats,
                         w_split=P.ws(self.w), donor=donor, sgd=P.sgd_ref(self.w) if hasattr(P, "sgd_ref") else None)


class BatchNorm(Module):
    """BatchNorm with batch statistics only (reference disables running stats:
    `util/model.py:23`, `server/server.py:48`). Optional fused residual-add + ReLU."""

    kind = "BatchNorm2d"

    def __init__(self, c, relu=False):
        super().__init__()
        self.c, self.relu = c, relu

    def register(self, layout):
        self.gamma = layout.add(f"{self.name}.weight", (self.c,), "ones", 1, self.name).name
        self.beta = layout.add(f"{self.name}.bias", (self.c,), "zeros", 1, self.name).name

    def own_params(self):
        return [self.gamma, self.beta]

    def forward(self, x, ctx, residual=None, relu=None, link=None, stats=None, planes: int = 0):
        """`planes`: the output's consumers are split-plane convs (Fn.batch_norm): 1 = they and
        fp32 readers, 2 = split-plane convs only. Effective while the weights' planes are live
        (training steps with BoundParams.split); otherwise the output is plain fp32. 4: the output
        is read only as the next BatchNorm's residual, which folds this apply into its own."""
        P = ctx.P
        rps = 1
        for d in x.shape[2:-1]:
            rps *= d
        if (getattr(P, "split", None) is None or self.c % 32) and planes != 4:
            planes = 0
        return Fn.batch_norm(x, ctx.token, P.w(self.gamma), P.w(self.beta), P.g(self.gamma), P.g(self.beta),
                             ctx.valid_rows(rps), self.relu if relu is None else relu, residual, link=link,
                             stats=stats, planes=planes)


def conv_bn(conv: Conv2d, bn: BatchNorm, x, ctx, conv_link=None, conv_donor=None, **bn_kw):
    """conv → BatchNorm with the BN statistics taken from the conv's epilogue (Fn.BNStats) and,
    for fp32 split-plane GEMMs, the BN backward handing the conv only dX's planes."""
    st = Fn.BNStats(ctx.valid)
    return bn.forward(conv.forward(x, ctx, link=conv_link, stats=st, donor=conv_donor), ctx, stats=st, **bn_kw)


class Linear(Module):
    kind = "Linear"

    def __init__(self, fin, fout, bias=True):
        super().__init__()
        self.fin, self.fout, self.bias = fin, fout, bias

    def register(self, layout):
        self.w = layout.add(f"{self.name}.weight", (self.fout, self.fin), "kaiming_linear", self.fin, self.name).name
        self.b = layout.add(f"{self.name}.bias", (self.fout,), "uniform_bias", self.fin, self.name).name if self.bias else None

    def own_params(self):
        return [self.w] + ([self.b] if self.b else [])

    def forward(self, x, ctx, **fuse):
        """`fuse`: epilogue fusions of Fn.linear (relu, premasked, gate_input, residual)."""
        P = ctx.P
        return Fn.linear(x, ctx.token, P.w(self.w), P.w(self.b) if self.b else None,
                         P.g(self.w), P.g(self.b) if self.b else None, w_split=P.ws(self.w),
                         sgd=P.sgd_ref(self.w) if hasattr(P, "sgd_ref") else None, **fuse)


class LayerNorm(Module):
    kind = "LayerNorm"

    def __init__(self, c):
        super().__init__()
        self.c = c

    def register(self, layout):
        self.gamma = layout.add(f"{self.name}.weight", (self.c,), "ones", 1, self.name).name
        self.beta = layout.add(f"{self.name}.bias", (self.c,), "zeros", 1, self.name).name

    def own_params(self):
        return [self.gamma, self.beta]

    def forward(self, x, ctx, planes: bool = False):
        """`planes`: the output's readers include split-plane linears (Fn.layer_norm); effective
        while the weights' planes are live (as BatchNorm.forward)."""
        P = ctx.P
        planes = planes and getattr(P, "split", None) is not None and self.c % 32 == 0
        return Fn.layer_norm(x, ctx.token, P.w(self.gamma), P.w(self.beta), P.g(self.gamma), P.g(self.beta),
                             planes=planes)


class Embedding(Module):
    kind = "Embedding"

    def __init__(self, vocab, dim):
        super().__init__()
        self.vocab, self.dim = vocab, dim

    def register(self, layout):
        self.w = layout.add(f"{self.name}.weight", (self.vocab, self.dim), "normal", 1, self.name).name

    def own_params(self):
        return [self.w]

    def forward(self, tokens, ctx, scale: float = 1.0, pe=None):
        P = ctx.P
        return Fn.embedding(tokens, ctx.token, P.w(self.w), P.g(self.w), scale, pe)


class MaxPool(Module):
    kind = "MaxPool2d"

    def __init__(self, k, s=None, pad=0):
        super().__init__()
        self.k, self.s, self.pad = k, s or k, pad

    def forward(self, x, ctx):
        return Fn.max_pool2d(x, self.k, self.s, self.pad)


class AvgPool(Module):
    kind = "AvgPool2d"

    def __init__(self, k, s=None):
        super().__init__()
        self.k, self.s = k, s or k

    def forward(self, x, ctx):
        return Fn.avg_pool2d(x, self.k, self.s)


class Flatten(Module):
    kind = "Flatten"

    def forward(self, x, ctx):
        return x.reshape(x.shape[0], x.shape[1], -1)
