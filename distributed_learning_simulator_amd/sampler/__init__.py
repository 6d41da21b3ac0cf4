"""Data partitioners (client shards), registry-based like the reference
(`sampler/__init__.py:2-7` registers `random_label_iid` into the external
`global_sampler_factory`; `iid` is the external default, `config.py:24`).

All partitioners are deterministic functions of (labels, part_number, seed), so every rank
computes identical shards without communication.
"""

from __future__ import annotations

from typing import Callable

import numpy as np
import torch

from ..utils.logging import get_logger

_REGISTRY: dict[str, Callable] = {}


def register(name: str):
    def deco(fn):
        _REGISTRY[name] = fn
        return fn

    return deco


class _Factory:
    def register(self, name, fn):
        _REGISTRY[name] = fn

    def get(self, name):
        return _REGISTRY[name]

    def has(self, name):
        return name in _REGISTRY


global_sampler_factory = _Factory()


def get_partition(name: str, labels: torch.Tensor, part_number: int, seed: int = 0, **kwargs) -> list[torch.Tensor]:
    if name not in _REGISTRY:
        raise ValueError(f"unknown dataset_sampling {name!r}; registered: {sorted(_REGISTRY)}")
    return _REGISTRY[name](labels.cpu(), part_number, seed=seed, **kwargs)


@register("iid")
def iid_split(labels: torch.Tensor, part_number: int, seed: int = 0, **_) -> list[torch.Tensor]:
    """Label-stratified equal split: every part receives ~n/parts samples of every label."""
    g = torch.Generator().manual_seed(seed + 11)
    parts: list[list[torch.Tensor]] = [[] for _ in range(part_number)]
    num_classes = int(labels.max().item()) + 1 if labels.numel() else 0
    offset = 0
    for c in range(num_classes):
        idx = (labels == c).nonzero().flatten()
        idx = idx[torch.randperm(idx.numel(), generator=g)]
        chunks = torch.tensor_split(idx, part_number)
        for p in range(part_number):
            parts[(p + offset) % part_number].append(chunks[p])
        offset += idx.numel() % part_number  # rotate remainders so sizes stay balanced
    return [torch.cat(p).sort().values if p else torch.zeros(0, dtype=torch.long) for p in parts]


@register("random_label_iid")
def random_label_iid_split(labels: torch.Tensor, part_number: int, seed: int = 0,
                           sampled_class_number: int = 2, **_) -> list[torch.Tensor]:
    """Reference `sampler/base.py:9-46` (RandomLabelIIDSplit): each part gets
    `sampled_class_number` random labels, every label must be held by some part, and the
    samples of a label are split equally among the parts that hold it."""
    num_classes = int(labels.max().item()) + 1
    g = torch.Generator().manual_seed(seed + 23)
    assigned: list[list[int]] = []
    for attempt in range(1000):
        assigned = [torch.randperm(num_classes, generator=g)[:sampled_class_number].tolist()
                    for _ in range(part_number)]
        covered = set(c for a in assigned for c in a)
        if len(covered) == num_classes:
            break
    else:
        raise AssertionError("random_label_iid could not cover all labels; raise sampled_class_number")
    holders: dict[int, list[int]] = {c: [] for c in range(num_classes)}
    for p, a in enumerate(assigned):
        for c in a:
            holders[c].append(p)
    parts: list[list[torch.Tensor]] = [[] for _ in range(part_number)]
    for c in range(num_classes):
        idx = (labels == c).nonzero().flatten()
        idx = idx[torch.randperm(idx.numel(), generator=g)]
        for chunk, p in zip(torch.tensor_split(idx, len(holders[c])), holders[c]):
            parts[p].append(chunk)
    out = [torch.cat(p).sort().values for p in parts]
    for p, a in enumerate(assigned):
        get_logger().debug("worker %d labels %s size %d", p, sorted(a), out[p].numel())
    return out


@register("dirichlet_non_iid")
def dirichlet_split(labels: torch.Tensor, part_number: int, seed: int = 0, alpha: float = 0.5,
                    **_) -> list[torch.Tensor]:
    """Per-label Dirichlet(alpha) proportions over parts (common non-IID benchmark)."""
    num_classes = int(labels.max().item()) + 1
    g = torch.Generator().manual_seed(seed + 37)
    parts: list[list[torch.Tensor]] = [[] for _ in range(part_number)]
    # a private generator: partitioning must not reseed the process-wide torch RNG
    rng = np.random.default_rng(seed + 41)
    for c in range(num_classes):
        idx = (labels == c).nonzero().flatten()
        idx = idx[torch.randperm(idx.numel(), generator=g)]
        prop = torch.from_numpy(rng.dirichlet(np.full(part_number, float(alpha))))
        cuts = (prop.cumsum(0) * idx.numel()).round().long().tolist()[:-1]
        for p, chunk in enumerate(torch.tensor_split(idx, cuts)):
            parts[p].append(chunk)
    return [torch.cat(p).sort().values for p in parts]


# alias used by some configs / papers
_REGISTRY["non_iid"] = random_label_iid_split
