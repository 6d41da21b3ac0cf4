"""Model zoo (cohort form). Names used by the reference configs:
`LeNet5`, `densenet40`, `Resnet50`, `TransformerClassificationModel`, `TwoGCN`/`OneGCN`/
`SimpleGCN`, plus `ResNet18` (north-star) and `MLP`. Architectures are the standard ones the
reference's external zoos provide [KNOW]; parameter counts are pinned by tests:
LeNet5 61,706; ResNet-18 (CIFAR stem) 11,173,962; ResNet-50 25,557,032;
DenseNet-40 (k=12) 1,059,298 (CIFAR-10); Transformer layer (d=100, ff=2048) 452,548.
"""

from __future__ import annotations

import math

import torch

from ..engine.params import ParamLayout
from ..ops import functional as Fn
from .layers import (AvgPool, BatchNorm, Conv2d, Embedding, conv_bn, Flatten, LayerNorm, Linear,
                     MaxPool, Module, ReLU, RunCtx, Seq)


class CohortModel:
    """A model definition + its flat parameter layout."""

    def __init__(self, root: Module, name: str, input_kind: str, num_classes: int):
        self.root = root
        self.name = name
        self.input_kind = input_kind  # image | tokens | graph | vector
        self.num_classes = num_classes
        root.assign_names("")
        self.layout = ParamLayout()
        root.register(self.layout)

    def forward(self, x, ctx: RunCtx):
        return self.root.forward(x, ctx)

    @property
    def num_params(self) -> int:
        return self.layout.num_params


# ---------------------------------------------------------------------------- MLP
class MLPNet(Module):
    kind = "MLP"

    def __init__(self, fin, hidden, classes):
        super().__init__()
        dims = [fin] + list(hidden)
        self.layers = []
        for i in range(len(hidden)):
            self.layers.append(self.child(f"fc{i + 1}", Linear(dims[i], dims[i + 1])))
            self.child(f"relu{i + 1}", ReLU())
        self.out = self.child(f"fc{len(hidden) + 1}", Linear(dims[-1], classes))

    def forward(self, x, ctx):
        x = x.reshape(x.shape[0], x.shape[1], -1)
        for l in self.layers:
            x = torch.relu(l.forward(x, ctx))
        return self.out.forward(x, ctx)


# ------------------------------------------------------------------------- LeNet5
class LeNet5Net(Module):
    kind = "LeNet5"

    def __init__(self, cin=1, classes=10, hw=28):
        super().__init__()
        self.child("conv1", Conv2d(cin, 6, 5, 1, 2 if hw == 28 else 0, bias=True))
        self.child("relu1", ReLU())
        self.child("pool1", MaxPool(2))
        self.child("conv2", Conv2d(6, 16, 5, 1, 0, bias=True))
        self.child("relu2", ReLU())
        self.child("pool2", MaxPool(2))
        self.child("fc1", Linear(16 * 5 * 5, 120))
        self.child("relu3", ReLU())
        self.child("fc2", Linear(120, 84))
        self.child("relu4", ReLU())
        self.child("fc3", Linear(84, classes))

    def forward(self, x, ctx):
        x = self.pool1.forward(torch.relu(self.conv1.forward(x, ctx)), ctx)
        x = self.pool2.forward(torch.relu(self.conv2.forward(x, ctx)), ctx)
        x = x.reshape(x.shape[0], x.shape[1], -1)
        x = torch.relu(self.fc1.forward(x, ctx))
        x = torch.relu(self.fc2.forward(x, ctx))
        return self.fc3.forward(x, ctx)


# ------------------------------------------------------------------------- ResNets

def _residual_link(block, x, ctx):
    """Blocks in training route the shortcut's gradient of the block input through conv1's dgrad
    epilogue (Fn.ResidualLink) instead of a separate autograd add over the block input: the
    identity shortcut's from the last BN, a downsample shortcut's from its conv (the donor)."""
    if ctx.training and x.requires_grad:
        return Fn.ResidualLink()
    return None


def _down(seq: Seq, x, ctx, donor=None):
    """Downsample shortcut Seq(Conv2d 1x1, BatchNorm) with epilogue statistics; `donor`: the
    shortcut conv's input gradient goes to the block's first conv (Fn.ResidualLink). Its BN output
    is read only as the block's last BN's residual, which applies it (batch_norm planes=4)."""
    conv, bn = seq.children
    return conv_bn(conv, bn, x, ctx, conv_donor=donor, planes=4)


class BasicBlock(Module):
    kind = "BasicBlock"
    expansion = 1

    def __init__(self, cin, cout, stride):
        super().__init__()
        self.child("conv1", Conv2d(cin, cout, 3, stride, 1))
        self.child("bn1", BatchNorm(cout, relu=True))
        self.child("conv2", Conv2d(cout, cout, 3, 1, 1))
        self.child("bn2", BatchNorm(cout))
        self.down = None
        if stride != 1 or cin != cout:
            self.down = self.child("downsample", Seq(Conv2d(cin, cout, 1, stride, 0), BatchNorm(cout)))

    def forward(self, x, ctx, out_planes: int = 1):
        """`out_planes`: what reads the block output (ResNetNet.forward) — 1: the next block's convs
        (planes) and its identity shortcut (fp32); 2: convs only (a downsample block follows);
        0: the pooling head only (fp32)."""
        link = _residual_link(self, x, ctx)
        # bn1's output feeds conv2 only: its apply pass is deferred into conv2's halo loader where
        # the shape allows (Fn.DeferredBN), planes only otherwise (fp32 GEMMs, Fn.batch_norm)
        out = conv_bn(self.conv1, self.bn1, x, ctx, conv_link=link, planes=3)
        sc = x if self.down is None else _down(self.down, x, ctx, donor=link)
        return conv_bn(self.conv2, self.bn2, out, ctx, residual=sc, relu=True,
                       link=link if self.down is None else None, planes=out_planes)


class Bottleneck(Module):
    kind = "Bottleneck"
    expansion = 4

    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.child("conv1", Conv2d(cin, width, 1, 1, 0))
        self.child("bn1", BatchNorm(width, relu=True))
        self.child("conv2", Conv2d(width, width, 3, stride, 1))
        self.child("bn2", BatchNorm(width, relu=True))
        self.child("conv3", Conv2d(width, cout, 1, 1, 0))
        self.child("bn3", BatchNorm(cout))
        self.down = None
        if stride != 1 or cin != cout:
            self.down = self.child("downsample", Seq(Conv2d(cin, cout, 1, stride, 0), BatchNorm(cout)))

    def forward(self, x, ctx, out_planes: int = 1):
        """`out_planes`: as BasicBlock.forward."""
        link = _residual_link(self, x, ctx)
        out = conv_bn(self.conv1, self.bn1, x, ctx, conv_link=link, planes=2)
        out = conv_bn(self.conv2, self.bn2, out, ctx, planes=2)
        sc = x if self.down is None else _down(self.down, x, ctx, donor=link)
        return conv_bn(self.conv3, self.bn3, out, ctx, residual=sc, relu=True,
                       link=link if self.down is None else None, planes=out_planes)


class ResNetNet(Module):
    kind = "ResNet"

    def __init__(self, block, layers, classes=10, cin=3, cifar_stem=True):
        super().__init__()
        self.cifar_stem = cifar_stem
        if cifar_stem:
            self.child("conv1", Conv2d(cin, 64, 3, 1, 1))
        else:
            self.child("conv1", Conv2d(cin, 64, 7, 2, 3))
        self.child("bn1", BatchNorm(64, relu=True))
        if not cifar_stem:
            self.child("maxpool", MaxPool(3, 2, 1))
        c = 64
        self.stages = []
        for i, (n, w) in enumerate(zip(layers, (64, 128, 256, 512))):
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                b = block(c, w, stride)
                blocks.append(b)
                c = w * block.expansion
            self.stages.append(self.child(f"layer{i + 1}", Seq(*blocks)))
        self.child("fc", Linear(c, classes))

    def forward(self, x, ctx):
        x = conv_bn(self.conv1, self.bn1, x, ctx, planes=0 if not self.cifar_stem else 1)
        if not self.cifar_stem:
            x = self.maxpool.forward(x, ctx)
        # each block output is written in the form(s) its readers take: split planes only when a
        # downsample block follows (its convs read planes; its shortcut is a conv too), fp32 only
        # before the pooling head, both otherwise (planes for the convs, fp32 for the identity
        # shortcut's residual add)
        blocks = [b for s in self.stages for b in s.children]
        for i, b in enumerate(blocks):
            nxt = blocks[i + 1] if i + 1 < len(blocks) else None
            op = 0 if nxt is None else 2 if nxt.down is not None else 1
            x = b.forward(x, ctx, out_planes=op)
        x = Fn.global_avg_pool(x)
        return self.fc.forward(x, ctx)


# ------------------------------------------------------------------------ DenseNet
class DenseLayer(Module):
    """BN-ReLU-Conv3x3 (the reference's OBD pattern `(BN, ReLU, Conv)` matches it)."""

    kind = "DenseLayer"

    def __init__(self, cin, growth):
        super().__init__()
        self.child("norm", BatchNorm(cin, relu=True))
        self.child("relu", ReLU())
        self.child("conv", Conv2d(cin, growth, 3, 1, 1))

    def forward(self, x, ctx):
        y = self.conv.forward(self.norm.forward(x, ctx), ctx)
        return torch.cat([x, y], dim=-1)


class Transition(Module):
    kind = "Transition"

    def __init__(self, cin, cout):
        super().__init__()
        self.child("norm", BatchNorm(cin, relu=True))
        self.child("relu", ReLU())
        self.child("conv", Conv2d(cin, cout, 1, 1, 0))
        self.child("pool", AvgPool(2))

    def forward(self, x, ctx):
        return self.pool.forward(self.conv.forward(self.norm.forward(x, ctx), ctx), ctx)


class DenseBlock(Seq):
    """The layers of one dense block run as ONE fused autograd op over a preallocated feature
    buffer (Fn.dense_block: no per-layer concat). Module/param names are the Sequential's
    (`dense1.0.norm.weight`, ...), so OBD block discovery and messages see the same structure."""

    kind = "Sequential"

    def __init__(self, layers, growth):
        super().__init__(*layers)
        self.growth = growth

    def forward(self, x, ctx):
        P = ctx.P
        lps = [Fn.DenseLayerParams(P.w(l.norm.gamma), P.w(l.norm.beta), P.g(l.norm.gamma), P.g(l.norm.beta),
                                   P.w(l.conv.w), P.g(l.conv.w)) for l in self.children]
        rps = x.shape[2] * x.shape[3]
        return Fn.dense_block(x, ctx.token, lps, self.growth, ctx.valid_rows(rps), training=ctx.training)


class DenseNetNet(Module):
    kind = "DenseNet"

    def __init__(self, depth=40, growth=12, classes=10, cin=3):
        super().__init__()
        n = (depth - 4) // 3
        c = 2 * growth  # stem width 2k: pins 1,059,298 (CIFAR-10) / 1,100,428 (CIFAR-100)
        self.child("conv1", Conv2d(cin, c, 3, 1, 1))
        self.blocks = []
        for b in range(3):
            layers = []
            for _ in range(n):
                layers.append(DenseLayer(c, growth))
                c += growth
            self.blocks.append(self.child(f"dense{b + 1}", DenseBlock(layers, growth)))
            if b < 2:
                self.blocks.append(self.child(f"trans{b + 1}", Transition(c, c)))
        self.child("norm", BatchNorm(c, relu=True))
        self.child("relu", ReLU())
        self.child("fc", Linear(c, classes))

    def forward(self, x, ctx):
        x = self.conv1.forward(x, ctx)
        for b in self.blocks:
            x = b.forward(x, ctx)
        x = self.norm.forward(x, ctx)
        x = Fn.global_avg_pool(x)
        return self.fc.forward(x, ctx)


# --------------------------------------------------------------------- Transformer
class MultiheadAttention(Module):
    kind = "MultiheadAttention"

    def __init__(self, d, h):
        super().__init__()
        self.d, self.h = d, h
        self.child("in_proj", Linear(d, 3 * d))
        self.child("out_proj", Linear(d, d))

    def forward(self, x, ctx, key_valid, residual=None, attn_drop: float = 0.0, attn_seeds=None, link=None, **drop):
        """Returns out_proj(attention) (+ residual, added in the projection's epilogue; `drop`:
        dropout of the projection output before that add). `attn_drop`: dropout on the
        attention probabilities (nn.MultiheadAttention(dropout=...)), masks from this step's
        next dropout site. `link` (residual is x): out_proj deposits the residual's gradient,
        in_proj's dgrad adds it (Fn.linear res_link / acc_link)."""
        K, B, L, D = x.shape
        qkv = self.in_proj.forward(x, ctx, acc_link=link)
        if link is not None:
            drop = dict(drop, res_link=link)
        ad = {}
        if attn_drop:
            ad = {"drop_p": attn_drop, "drop_seeds": attn_seeds if attn_seeds is not None else ctx.dropout_seeds()}
        if Fn.packed_attention_ok(qkv, L, D // self.h):
            # heads read / written in place in the projections' row layouts (no permute copies)
            o = Fn.attention_packed(qkv, key_valid, self.h, **ad)
            return self.out_proj.forward(o, ctx, residual=residual, **drop)
        qkv = qkv.reshape(K, B, L, 3, self.h, D // self.h)
        qkv = qkv.permute(3, 0, 1, 4, 2, 5)  # 3,K,B,H,L,dh
        o = Fn.attention(qkv[0].contiguous(), qkv[1].contiguous(), qkv[2].contiguous(), key_valid, **ad)
        o = o.permute(0, 1, 3, 2, 4).reshape(K, B, L, D)
        return self.out_proj.forward(o, ctx, residual=residual, **drop)


class TransformerEncoderLayer(Module):
    """Post-norm encoder layer, PyTorch `nn.TransformerEncoderLayer` defaults (ReLU FFN,
    dropout 0.1 in training), the reference's TransformerClassificationModel blocks.

    Dropout sites: x + dropout(self_attn(x)), the FFN's dropout(relu(linear1)), x + dropout(ff).
    All three are masks inside the GEMM epilogues:
    - residual branches are masked before the residual add;
    - the FFN ReLU output is masked in linear1's epilogue, and linear2's ReLU'-gated dgrad
      epilogue (h > 0 iff kept and positive) carries the 1/(1-p).
    Masks come from (step seed, site, client id) hashes (RunCtx.dropout_seeds), so they do not
    depend on which rank or cohort row trains a client. The attention probabilities get the same
    dropout (nn.MultiheadAttention(dropout=p) inside nn.TransformerEncoderLayer), applied inside
    the flash-attention kernels from a (client, head, query, key) hash."""

    kind = "TransformerEncoderLayer"

    def __init__(self, d, h, ff, dropout: float = 0.1):
        super().__init__()
        self.dropout = float(dropout)
        self.child("self_attn", MultiheadAttention(d, h))
        self.child("linear1", Linear(d, ff))
        self.child("linear2", Linear(ff, d))
        self.child("norm1", LayerNorm(d))
        self.child("norm2", LayerNorm(d))

    def forward(self, x, ctx, key_valid):
        p = self.dropout if ctx.training else 0.0

        def drop():
            return {"drop_p": p, "drop_seeds": ctx.dropout_seeds()} if p else {}

        # residual adds, the FFN ReLU and the dropout masks (forward and backward) ride in the
        # GEMM epilogues
        sa = ctx.dropout_seeds() if p else None  # (the attention's site first: same order as unfused)
        # each residual input has two readers — a projection and the residual add of a later one — and
        # the later one hands its gradient to the first one's dgrad epilogue (no autograd add pass)
        fuse = ctx.training
        l1 = Fn.ResidualLink() if fuse else None
        l2 = Fn.ResidualLink() if fuse else None
        # the LayerNorm outputs feed linear1 / the next layer's in_proj (split planes: the LDS-DMA
        # plane GEMM) and the residual adds (fp32)
        x = self.norm1.forward(self.self_attn.forward(x, ctx, key_valid, residual=x, attn_drop=p, attn_seeds=sa,
                                                      link=l1, **drop()), ctx, planes=True)
        # the hidden activation goes to linear2 as split planes (linear1's epilogue writes them), and
        # its gradient back to linear1 likewise (linear2's dgrad epilogue)
        h = self.linear1.forward(x, ctx, relu=True, premasked=True, out_planes=True, acc_link=l2, **drop())
        y = self.linear2.forward(h, ctx, gate_input=True, residual=x, gate_scale=1.0 / (1.0 - p), dx_planes=True,
                                 res_link=l2, **drop())
        return self.norm2.forward(y, ctx, planes=True)


class TransformerClassifier(Module):
    kind = "TransformerClassificationModel"

    def __init__(self, vocab, d, h, layers, ff, classes, max_len, dropout: float = 0.1):
        super().__init__()
        self.d, self.max_len = d, max_len
        self.child("embedding", Embedding(vocab, d))
        self.layers = [self.child(f"encoder.layers.{i}", TransformerEncoderLayer(d, h, ff, dropout))
                       for i in range(layers)]
        self.child("classifier", Linear(d, classes))
        pe = torch.zeros(max_len, d)
        pos = torch.arange(max_len).float()[:, None]
        div = torch.exp(torch.arange(0, d, 2).float() * (-math.log(10000.0) / d))
        pe[:, 0::2] = torch.sin(pos * div)
        pe[:, 1::2] = torch.cos(pos * div[: d // 2])
        self._pe = pe
        self._pe_dev = {}

    def forward(self, batch, ctx):
        tokens, lengths = batch  # [K,B,L] int, [K,B] int
        L = tokens.shape[-1]
        key = tokens.device
        if key not in self._pe_dev:
            self._pe_dev[key] = self._pe.to(tokens.device, torch.float32)
        # embedding · √d + positional encoding: one fused kernel
        x = self.embedding.forward(tokens, ctx, scale=math.sqrt(self.d), pe=self._pe_dev[key][:L].contiguous())
        for l in self.layers:
            x = l.forward(x, ctx, lengths)
        pooled = Fn.seq_mean(x, lengths)  # masked mean over the valid tokens
        return self.classifier.forward(pooled, ctx)


# ---------------------------------------------------------------------------- GCN
class GCNConv(Module):
    """PyG `GCNConv`: out = Â (X Wᵀ) + b (bias after propagation); params `lin.weight`, `bias`."""

    kind = "GCNConv"

    def __init__(self, fin, fout):
        super().__init__()
        self.fout = fout
        self.child("lin", Linear(fin, fout, bias=False))

    def register(self, layout):
        super().register(layout)
        self.b = layout.add(f"{self.name}.bias", (self.fout,), "zeros", 1, self.name).name

    def own_params(self):
        return [self.b]

    def forward(self, x, ctx, edges, K):
        from ..data.graph import propagate

        P = ctx.P
        if x.dim() == 2:  # shared node features
            h = Fn.linear_shared_input(x, ctx.token, P.w(self.lin.w), P.g(self.lin.w))
        else:
            h = self.lin.forward(x, ctx)
        h = propagate(h, edges)
        return _AddBias.apply(h, ctx.token, P.w(self.b), P.g(self.b))


class _AddBias(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, token, b, gb):
        ctx.gb = gb
        K = h.shape[0]
        bb = b if b.shape[0] == K else b.repeat_interleave(K // b.shape[0], 0)
        return h + bb[:, None, :].to(h.dtype)

    @staticmethod
    def backward(ctx, dh):
        if ctx.gb is not None:
            ctx.gb.copy_(dh.float().sum(1))
        return dh, None, None, None


class GCNNet(Module):
    kind = "GCN"

    def __init__(self, fin, hidden, classes, layers):
        super().__init__()
        dims = [fin] + [hidden] * (layers - 1) + [classes]
        self.convs = [self.child(f"conv{i + 1}", GCNConv(dims[i], dims[i + 1])) for i in range(layers)]

    def forward(self, batch, ctx):
        K = ctx.P.K
        last = len(self.convs) - 1
        if batch.sub is None:  # evaluation: the whole graph, shared by the K models
            h = batch.x
            for i, c in enumerate(self.convs):
                h = c.forward(h, ctx, batch.full, K)
                if i < last:
                    h = torch.relu(h)
            idx = batch.seeds.long().unsqueeze(-1).expand(-1, -1, h.shape[-1])
            return torch.gather(h, 1, idx)
        # training: the cohort's sampled subgraphs ([K, Nmax] node table, seeds in rows [:, :B])
        sub, halo = batch.sub, batch.halo
        share = halo is not None and halo.cg.share_feature
        if share:
            halo.begin_batch()  # (fed_aas: exchange or skip this batch, same on every rank)
        real = (sub.nid >= 0).unsqueeze(-1)
        h = batch.x.index_select(0, sub.nid.clamp(min=0).reshape(-1)).view(K, sub.nmax, -1)
        h = torch.where(real, h, torch.zeros_like(h))
        for i, c in enumerate(self.convs):
            edges = sub.l0 if i == 0 else sub.l1
            if i > 0 and share:
                h = halo(h, sub)  # boundary embeddings of the other clients (detached)
                if halo.last_skip:
                    edges = sub.l0  # skipped exchange: no cross-client edges this batch
            h = c.forward(h, ctx, edges, K)
            if i < last:
                h = torch.relu(h)
        return h[:, : sub.B].contiguous()


# --------------------------------------------------------------------------- build
def count_params(model: CohortModel) -> int:
    return model.layout.num_params


def stored_image_channels(name: str, dataset_spec) -> int | None:
    """Channel count image data should be stored with for this model: conv-stem ResNet/DenseNet
    consume RGB zero-padded to 8 channels (16-byte im2col gathers, exact); others the raw C."""
    if dataset_spec.kind != "image":
        return None
    C = dataset_spec.shape[2]
    n = name.lower().replace("_", "")
    if (n.startswith("resnet") or n.startswith("densenet")) and C % 8:
        return (C + 7) // 8 * 8
    return C


def build_model(name: str, dataset_spec, model_kwargs: dict | None = None) -> CohortModel:
    kw = dict(model_kwargs or {})
    n = name.lower().replace("_", "")
    classes = dataset_spec.num_classes
    if dataset_spec.kind == "image":
        H, W, C = dataset_spec.shape
        if n == "lenet5":
            return CohortModel(LeNet5Net(C, classes, H), name, "image", classes)
        if n in ("mlp", "twonn", "2nn"):
            hidden = kw.get("hidden", [200, 200])
            return CohortModel(MLPNet(H * W * C, hidden, classes), name, "image", classes)
        if n in ("resnet18", "resnet34", "resnet50", "resnet101"):
            depth = int(n[6:])
            cfg = {18: (BasicBlock, [2, 2, 2, 2]), 34: (BasicBlock, [3, 4, 6, 3]),
                   50: (Bottleneck, [3, 4, 6, 3]), 101: (Bottleneck, [3, 4, 23, 3])}[depth]
            cifar = kw.get("cifar_stem", H <= 64)
            return CohortModel(ResNetNet(cfg[0], cfg[1], classes, C, cifar), name, "image", classes)
        if n.startswith("densenet"):
            depth = int(n[8:] or 40)
            return CohortModel(DenseNetNet(depth, kw.get("growth_rate", 12), classes, C), name, "image", classes)
    if dataset_spec.kind == "text":
        if n in ("transformerclassificationmodel", "transformer"):
            d = int(kw.get("d_model", 100))
            return CohortModel(
                TransformerClassifier(dataset_spec.vocab_size, d, int(kw.get("nhead", 5)),
                                      int(kw.get("num_encoder_layer", 2)), int(kw.get("dim_feedforward", 2048)),
                                      classes, int(kw.get("max_len", dataset_spec.max_len)),
                                      float(kw.get("dropout", 0.1))),
                name, "tokens", classes)
    if dataset_spec.kind == "graph":
        layers = {"onegcn": 1, "twogcn": 2, "simplegcn": 2, "gcn": 2}.get(n)
        if layers is not None:
            return CohortModel(GCNNet(dataset_spec.num_features, int(kw.get("hidden", 64)), classes, layers),
                               name, "graph", classes)
    raise ValueError(f"unknown model {name!r} for dataset kind {dataset_spec.kind}")
