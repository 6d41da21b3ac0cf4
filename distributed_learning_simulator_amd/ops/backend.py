"""Backend selection for the client-batched primitives.

* CUDA (ROCm/HIP) tensors run the hand-written gfx950 kernels in `ops.hip` — the in-tree
  `_dls_hip*.so` extension. If it is missing on a GPU box this FAILS LOUDLY (no silent
  fallback): run `python -m distributed_learning_simulator_amd.ops.build` first.
* CPU tensors run the PyTorch oracle in `ops.ref` (used by the CPU test-suite).

`DLS_BACKEND=torch` forces the oracle on GPU too; it exists only so `bench.py --backend
torch` can measure the vendor-library (MIOpen/hipBLASLt) execution of the same cohort
schedule as a comparison point. It is never selected implicitly.
"""

from __future__ import annotations

import os

import torch

from . import ref

_forced = os.environ.get("DLS_BACKEND", "").lower()


def set_backend(name: str) -> None:
    global _forced
    _forced = name.lower()


def get(t: torch.Tensor):
    if t.is_cuda and _forced not in ("torch", "ref"):
        from . import hip

        return hip
    return ref


def using_hip(t: torch.Tensor) -> bool:
    return t.is_cuda and _forced not in ("torch", "ref")
