"""Dataset zoo with the shapes of the datasets the reference configs name.

There is no network: by default every dataset is generated deterministically from (seed, name)
— class-conditional and learnable, so FL curves move, but accuracy is NOT comparable with the
reference (runs are tagged `synthetic: true` in metrics.jsonl / round_record.json). Real data
already on local disk is used instead when `dataset_kwargs.root` names a directory holding
`<root>/<name>/{train,test}.npz` (images: `x` [N,H,W,C] uint8 or float, `y` [N]; text:
`tokens` [N,L] int, `lengths` [N], `y` [N]); `numpy.load` with `allow_pickle=False`.

Images are stored device-resident in the compute layout (NHWC, bf16 on GPU) when they fit
(`materialize_limit` elements); larger ones (ImageNet-shaped) are generated procedurally per
batch from a per-index hash, so a 1.28 M-image dataset costs only its label vector.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch


@dataclass
class DatasetSpec:
    name: str
    kind: str  # image | text | graph
    num_classes: int
    n_train: int
    n_test: int
    shape: tuple = ()  # image (H, W, C)
    vocab_size: int = 0
    max_len: int = 0
    num_nodes: int = 0
    num_features: int = 0
    avg_degree: int = 0
    extra: dict = field(default_factory=dict)


_SPECS = {
    "mnist": DatasetSpec("MNIST", "image", 10, 60000, 10000, (28, 28, 1)),
    "fashionmnist": DatasetSpec("FashionMNIST", "image", 10, 60000, 10000, (28, 28, 1)),
    "cifar10": DatasetSpec("CIFAR10", "image", 10, 50000, 10000, (32, 32, 3)),
    "cifar100": DatasetSpec("CIFAR100", "image", 100, 50000, 10000, (32, 32, 3)),
    "imagenet": DatasetSpec("ImageNet", "image", 1000, 1281167, 50000, (224, 224, 3)),
    "imdb": DatasetSpec("imdb", "text", 2, 25000, 25000, vocab_size=20000, max_len=300),
    "agnews": DatasetSpec("AG_NEWS", "text", 4, 120000, 7600, vocab_size=30000, max_len=128),
    "coauthorcs": DatasetSpec("Coauthor_CS", "graph", 15, 0, 0, num_nodes=18333, num_features=6805, avg_degree=9),
    "cora": DatasetSpec("Cora", "graph", 7, 0, 0, num_nodes=2708, num_features=1433, avg_degree=4),
    "pubmed": DatasetSpec("PubMed", "graph", 3, 0, 0, num_nodes=19717, num_features=500, avg_degree=5),
    "citationfull": DatasetSpec("CitationFull", "graph", 4, 0, 0, num_nodes=17716, num_features=1639, avg_degree=6),
    "dblp": DatasetSpec("DBLP", "graph", 4, 0, 0, num_nodes=17716, num_features=1639, avg_degree=6),
    "yelp": DatasetSpec("Yelp", "graph", 100, 0, 0, num_nodes=716847, num_features=300, avg_degree=19),
    "amazonproducts": DatasetSpec("AmazonProducts", "graph", 107, 0, 0, num_nodes=1569960, num_features=200, avg_degree=168),
    "reddit": DatasetSpec("Reddit", "graph", 41, 0, 0, num_nodes=232965, num_features=602, avg_degree=492),
}


def get_spec(name: str, dataset_kwargs: dict | None = None) -> DatasetSpec:
    kw = dict(dataset_kwargs or {})
    key = kw.get("name", name).lower().replace("_", "").replace("-", "")
    if key not in _SPECS:
        raise ValueError(f"unknown dataset {name!r}; known: {sorted(s.name for s in _SPECS.values())}")
    spec = DatasetSpec(**{k: getattr(_SPECS[key], k) for k in _SPECS[key].__dataclass_fields__})
    if spec.kind == "text" and "max_len" in kw:
        spec.max_len = int(kw["max_len"])
    for k in ("n_train", "n_test", "num_nodes", "vocab_size", "num_features"):
        if k in kw:
            setattr(spec, k, int(kw[k]))
    if "scale" in kw:  # shrink a dataset for tests / smoke runs
        s = float(kw["scale"])
        spec.n_train = max(spec.num_classes * 4, int(spec.n_train * s))
        spec.n_test = max(spec.num_classes * 2, int(spec.n_test * s))
        spec.num_nodes = max(spec.num_classes * 20, int(spec.num_nodes * s)) if spec.num_nodes else 0
    return spec


def _hash_u32(x: torch.Tensor) -> torch.Tensor:
    """Integer mixing (lowbias32) on int64 tensors, result in [0, 2^32)."""
    m = 0xFFFFFFFF
    x = x & m
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & m
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & m
    x = x ^ (x >> 16)
    return x


def _load_npz(root: str, name: str, split: str):
    import os

    import numpy as np

    path = os.path.join(root, name, f"{split}.npz")
    if not os.path.exists(path):
        raise FileNotFoundError(f"dataset_kwargs.root given but {path} is missing")
    with np.load(path, allow_pickle=False) as f:
        return {k: torch.from_numpy(np.ascontiguousarray(f[k])) for k in f.files}


class ImageDataset:
    """Class-conditional images: x = prototype[y] (low-frequency pattern) + noise(index).

    Labels are a seeded balanced permutation. `gather(idx)` returns [.., H, W, Cs] where
    Cs = `channels` ≥ C: conv-first models store RGB with zero channels up to 8 so the stem's
    im2col gathers are 16-byte vectors (exact: the padded weight channels see only zeros)."""

    def __init__(self, spec: DatasetSpec, split: str, seed: int, device, dtype,
                 materialize_limit: int | None = None, noise: float = 1.0, signal: float = 0.35,
                 channels: int | None = None, arrays: dict | None = None, label_noise: float = 0.1):
        self.spec = spec
        self.split = split
        self.device = device
        self.dtype = dtype
        self.noise = noise
        H0, W0, C0 = spec.shape
        self.channels = max(int(channels or C0), C0)
        self.shape = (H0, W0, self.channels)
        n = spec.n_train if split == "train" else spec.n_test
        if arrays is not None:
            n = int(arrays["y"].shape[0])
        self.n = n
        g = torch.Generator().manual_seed(seed * 1000003 + (0 if split == "train" else 1))
        self.labels = (torch.randperm(n, generator=g) % spec.num_classes).to(torch.int32)
        # the image is drawn from `source` class; a `label_noise` fraction carries a random label,
        # so even a perfect model stays below 100 % (accuracy keeps discriminating numerics drift)
        self.source = self.labels.clone()
        if label_noise > 0:
            flip = torch.rand(n, generator=g) < label_noise
            self.labels = torch.where(flip, torch.randint(0, spec.num_classes, (n,), generator=g).to(torch.int32),
                                      self.labels)
        if arrays is not None:
            self.labels = arrays["y"].to(torch.int32).reshape(-1)
            self.source = self.labels
        H, W, C = spec.shape
        gp = torch.Generator().manual_seed(seed * 7919 + 17)  # prototypes shared by splits
        low = torch.randn(spec.num_classes, C, max(H // 4, 2), max(W // 4, 2), generator=gp)
        proto = torch.nn.functional.interpolate(low, size=(H, W), mode="bilinear", align_corners=False)
        # weak class signal under unit noise: learnable, but not in a single step
        self.prototypes = (proto * signal).permute(0, 2, 3, 1).contiguous()  # [classes, H, W, C]
        self.salt = seed * 2654435761 + (0 if split == "train" else 97)
        if materialize_limit is None:  # elements: 32 GB of bf16 on a 288 GB MI355X, 4 GB on the host
            materialize_limit = 16_000_000_000 if torch.device(device).type == "cuda" else 2_000_000_000
        self.materialized = n * H * W * self.channels <= materialize_limit or arrays is not None
        self.labels_dev = self.labels.to(device)
        self.source_dev = self.source.to(device)
        self.proto_dev = self.prototypes.to(device, dtype)
        if arrays is not None:
            x = arrays["x"].float()
            if arrays["x"].dtype == torch.uint8:
                x = x / 255.0
            x = x.reshape(n, H, W, C)
            mean = x.mean(dim=(0, 1, 2), keepdim=True)
            std = x.std(dim=(0, 1, 2), keepdim=True).clamp(min=1e-6)
            x = (x - mean) / std  # per-channel standardisation
            if self.channels > C:
                x = torch.nn.functional.pad(x, (0, self.channels - C))
            self.data = x.to(device, dtype)
        elif self.materialized:
            chunks = []
            dev = torch.device(device)
            for s in range(0, n, 8192):
                idx = torch.arange(s, min(n, s + 8192))
                chunks.append(self._generate(idx, dev, torch.float32).to(dtype))
            self.data = torch.cat(chunks)
        else:
            self.data = None

    def _generate(self, idx: torch.Tensor, device, dtype) -> torch.Tensor:
        H, W, C = self.spec.shape
        npix = H * W * C
        idx = idx.to(device).long()
        from ..ops import backend

        if backend.using_hip(self.proto_dev):  # one fused pass (csrc/elementwise.hip synth_images)
            from ..ops import hip

            if getattr(self, "_proto32", None) is None:
                self._proto32 = self.prototypes.to(device, torch.float32).contiguous()
                self._source32 = self.source.to(device, torch.int32).contiguous()
            img = hip.synth_images(idx.contiguous(), npix, C, self.channels, self._source32, self._proto32,
                                   self.salt, math.sqrt(6.0), self.noise)
            return img.view(-1, H, W, self.channels).to(dtype)
        pix = torch.arange(npix, device=device, dtype=torch.int64)
        h = _hash_u32(idx[:, None] * 0x9E3779B1 + pix[None, :] * 0x85EBCA77 + self.salt)
        h2 = _hash_u32(h + 0x68E31DA4)
        # Box-Muller-free approx normal: sum of two uniforms, centred, var 1/6 -> scale
        u = (h.float() + h2.float()) * (1.0 / 4294967296.0) - 1.0
        noise = u * math.sqrt(6.0) * self.noise
        lab = self.source[idx.cpu()].long() if device.type == "cpu" else self.source_dev[idx].long()
        proto = (self.prototypes if device.type == "cpu" else self.proto_dev.float())[lab]
        img = (proto + noise.view(-1, H, W, C)).to(dtype)
        if self.channels > C:
            img = torch.nn.functional.pad(img, (0, self.channels - C))
        return img

    def gather(self, idx: torch.Tensor) -> torch.Tensor:
        """idx: any-shape int tensor on device -> [*idx.shape, H, W, C]."""
        flat = idx.reshape(-1).long()
        if self.data is not None:
            from ..ops import backend

            if backend.using_hip(self.data) and (self.data[0].numel() * self.data.element_size()) % 16 == 0:
                from ..ops import hip

                return hip.gather_rows(self.data, idx).reshape(*idx.shape, *self.shape)
            out = self.data.index_select(0, flat)
        else:
            out = self._generate(flat, self.device, self.dtype)
        return out.reshape(*idx.shape, *self.shape)

    def gather_labels(self, idx: torch.Tensor) -> torch.Tensor:
        return self.labels_dev.index_select(0, idx.reshape(-1).long()).reshape(idx.shape)


class TextDataset:
    """Class-conditional token sequences: each class has its own Zipf-like preference over a
    slice of the vocabulary; lengths vary in [max_len/4, max_len]. Token 0 = padding."""

    def __init__(self, spec: DatasetSpec, split: str, seed: int, device, arrays: dict | None = None):
        self.spec = spec
        if arrays is not None:
            tok = arrays["tokens"].to(torch.int32)[:, : spec.max_len]
            if tok.shape[1] < spec.max_len:
                tok = torch.nn.functional.pad(tok, (0, spec.max_len - tok.shape[1]))
            self.n = int(tok.shape[0])
            self.labels = arrays["y"].to(torch.int32).reshape(-1)
            self.tokens = tok.to(device)
            self.lengths = arrays["lengths"].to(torch.int32).clamp(max=spec.max_len).to(device)
            self.labels_dev = self.labels.to(device)
            return
        n = spec.n_train if split == "train" else spec.n_test
        self.n = n
        g = torch.Generator().manual_seed(seed * 1000033 + (0 if split == "train" else 1))
        self.labels = (torch.randperm(n, generator=g) % spec.num_classes).to(torch.int32)
        L, V = spec.max_len, spec.vocab_size
        lengths = torch.randint(max(L // 4, 1), L + 1, (n,), generator=g)
        base = torch.randint(1, V, (n, L), generator=g)
        # class-informative tokens: with p=0.3 a token is drawn from the class slice
        slice_w = max((V - 1) // (spec.num_classes * 4), 1)
        cls_tok = 1 + self.labels.long()[:, None] * slice_w + torch.randint(0, slice_w, (n, L), generator=g)
        use = torch.rand(n, L, generator=g) < 0.3
        tokens = torch.where(use, cls_tok, base)
        pos = torch.arange(L)[None, :]
        tokens = torch.where(pos < lengths[:, None], tokens, torch.zeros_like(tokens))
        self.tokens = tokens.to(torch.int32).to(device)
        self.lengths = lengths.to(torch.int32).to(device)
        self.labels_dev = self.labels.to(device)

    def gather(self, idx):
        flat = idx.reshape(-1).long()
        t = self.tokens.index_select(0, flat).reshape(*idx.shape, self.spec.max_len)
        l = self.lengths.index_select(0, flat).reshape(idx.shape)
        return t, l

    def gather_labels(self, idx):
        return self.labels_dev.index_select(0, idx.reshape(-1).long()).reshape(idx.shape)


@dataclass
class DatasetCollection:
    spec: DatasetSpec
    train: object
    test: object
    graph: object = None
    # Validation phase carved out of the test split (`split_validation`); None = whole test set
    test_indices: torch.Tensor | None = None
    validation_indices: torch.Tensor | None = None
    synthetic: bool = True

    @property
    def name(self):
        return self.spec.name

    def split_validation(self, seed: int) -> None:
        """Give the collection a Validation phase: a seeded half of the test split becomes
        validation (dealt to clients for keep-best-model selection), the other half stays the
        server's test set. Parity unpinned: the reference's external toolbox owns this split."""
        if self.graph is not None or self.validation_indices is not None:
            return
        n = self.test.n
        perm = torch.randperm(n, generator=torch.Generator().manual_seed(seed * 31 + 7))
        self.validation_indices = perm[: n // 2].sort().values
        self.test_indices = perm[n // 2 :].sort().values

    def validation_labels(self) -> torch.Tensor:
        return self.test.labels[self.validation_indices]

    def merge_validation_into_train(self, seed: int) -> None:
        """`merge_validation_to_training_set` (reference config.py:27, consumed by its external
        toolbox): the Validation phase (a seeded half of the test split, `split_validation`) is
        appended to the training split — its samples become training indices n_train.. — and the
        collection keeps no Validation phase (so no keep-best-model selection); the server tests
        on the other half. Device-resident splits only (materialised images, token sets)."""
        if self.graph is not None:
            raise ValueError("merge_validation_to_training_set: graph datasets have no separate validation split")
        self.split_validation(seed)
        tr, te, vi = self.train, self.test, self.validation_indices
        if isinstance(tr, ImageDataset):
            if tr.data is None or te.data is None:
                raise ValueError("merge_validation_to_training_set: needs materialised image splits "
                                 "(this dataset is generated on the fly; lower dataset_kwargs.scale)")
            tr.data = torch.cat([tr.data, te.data.index_select(0, vi.to(te.data.device))])
            tr.source = torch.cat([tr.source, te.source[vi]])
            tr.source_dev = tr.source.to(tr.device)
            tr._proto32 = None
        elif isinstance(tr, TextDataset):
            tr.tokens = torch.cat([tr.tokens, te.tokens.index_select(0, vi.to(te.tokens.device))])
            tr.lengths = torch.cat([tr.lengths, te.lengths.index_select(0, vi.to(te.lengths.device))])
        else:
            raise ValueError(f"merge_validation_to_training_set: unsupported split type {type(tr).__name__}")
        tr.labels = torch.cat([tr.labels, te.labels[vi]])
        tr.labels_dev = tr.labels.to(tr.labels_dev.device)
        tr.n = int(tr.labels.shape[0])
        self.validation_indices = None  # (merged: no Validation phase left)


def create_dataset_collection(name: str, dataset_kwargs: dict | None, seed: int, device,
                              dtype=torch.float32, image_channels: int | None = None) -> DatasetCollection:
    """`image_channels`: stored channel count for image sets (≥ the dataset's; zero-padded)."""
    spec = get_spec(name, dataset_kwargs)
    kw = dict(dataset_kwargs or {})
    root = kw.get("root")
    arrays = {sp: _load_npz(root, spec.name, sp) for sp in ("train", "test")} if root else {"train": None, "test": None}
    if root and spec.kind == "image":
        spec.n_train, spec.n_test = (int(arrays[sp]["y"].shape[0]) for sp in ("train", "test"))
    if spec.kind == "image":
        noise = float(kw.get("noise", 1.0))
        signal = float(kw.get("signal", 0.35))
        ln = float(kw.get("label_noise", 0.1))
        return DatasetCollection(spec, ImageDataset(spec, "train", seed, device, dtype, noise=noise, signal=signal,
                                                    channels=image_channels, arrays=arrays["train"], label_noise=ln),
                                 ImageDataset(spec, "test", seed, device, dtype, noise=noise, signal=signal,
                                              channels=image_channels, arrays=arrays["test"], label_noise=ln),
                                 synthetic=not root)
    if spec.kind == "text":
        return DatasetCollection(spec, TextDataset(spec, "train", seed, device, arrays["train"]),
                                 TextDataset(spec, "test", seed, device, arrays["test"]), synthetic=not root)
    if spec.kind == "graph":
        from .graph import GraphDataset

        g = GraphDataset(spec, seed, device, dtype)
        return DatasetCollection(spec, g, g, graph=g)
    raise ValueError(spec.kind)
