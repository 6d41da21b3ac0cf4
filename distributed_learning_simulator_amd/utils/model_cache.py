"""Last-global-model cache and parameter loading.

Reference `util/model_cache.py:10-51` (`ModelCache`: a DataStorage-backed name→tensor dict
kept on the CPU; `cache_parameter_dict`, `get_parameter_diff(new) = new − cached`,
`add_parameter_diff`, `save`, `get_parameter_path`, `load_file`) and `util/model.py:6-23`
(`load_parameters(trainer, dict, reuse_learning_rate)`: rebuild the optimizer keeping its
hyper-parameters but clearing state when reusing the learning rate, otherwise a plain load;
always disable BN running stats).

Here a model is one flat fp32 row of a `ParamLayout` and it stays on the device: the cache
holds that row (dict views are produced on demand by `layout.unflatten`), and persistence is
`torch.save` of the name→tensor dict (read back with `torch.load(weights_only=True)`; no
pickle of arbitrary objects). BN never keeps running stats in this framework, so there is
nothing to disable.
"""

from __future__ import annotations

import os

import torch

from ..engine.params import ParamLayout


class ModelCache:
    def __init__(self, layout: ParamLayout):
        self.layout = layout
        self._row: torch.Tensor | None = None
        self._path: str | None = None
        self._dirty = False

    # ------------------------------------------------------------- access
    @property
    def parameter(self) -> torch.Tensor:
        """The cached model as a flat row [P_pad]."""
        if self._row is None and self._path is not None:
            self._load(self._path)
        assert self._row is not None, "empty model cache"
        return self._row

    @property
    def parameter_dict(self) -> dict[str, torch.Tensor]:
        return self.layout.unflatten(self.parameter)

    def _as_row(self, parameter) -> torch.Tensor:
        if isinstance(parameter, dict):
            return self.layout.flatten(parameter)
        return parameter.reshape(-1)

    # ------------------------------------------------------------ updates
    def cache_parameter(self, parameter, path: str | None = None) -> None:
        """Cache a model (flat row or name→tensor dict); `path` = where `save` writes it."""
        self._row = self._as_row(parameter).detach().clone().float()
        self._path = path
        self._dirty = True

    cache_parameter_dict = cache_parameter

    def get_parameter_diff(self, new_parameter) -> torch.Tensor:
        """Δ = new − cached (flat row)."""
        new = self._as_row(new_parameter).to(self.parameter.device, torch.float32)
        return new - self.parameter

    def add_parameter_diff(self, diff, path: str | None = None) -> None:
        """θ ← θ + Δ; the previous model is saved first when it has a path (reference order)."""
        if self._path is not None and self._dirty:
            self.save()
        self._row = self.parameter + self._as_row(diff).to(self.parameter.device, torch.float32)
        self._path = path if path is not None else self._path
        self._dirty = True

    # -------------------------------------------------------- persistence
    def save(self) -> None:
        if self._path is None or self._row is None:
            return
        os.makedirs(os.path.dirname(os.path.abspath(self._path)), exist_ok=True)
        torch.save({k: v.cpu() for k, v in self.layout.unflatten(self._row).items()}, self._path)
        self._dirty = False

    def get_parameter_path(self) -> str:
        self.save()
        assert self._path, "no path set"
        return self._path

    def load_file(self, path: str, device=None) -> None:
        self._path = path
        self._row = None
        self._load(path, device)

    def _load(self, path: str, device=None) -> None:
        tensors = torch.load(path, map_location="cpu", weights_only=True)
        row = self.layout.flatten(tensors)
        self._row = row.to(device) if device is not None else row
        self._dirty = False


def load_parameters(trainer, parameter, reuse_learning_rate: bool, K: int | None = None) -> None:
    """Load a global model into the first K client rows of a cohort trainer.

    `reuse_learning_rate=False` (the default in every aggregation worker) starts each client
    with a fresh optimizer (momentum re-initialised by the first gradient); True keeps the
    optimizer state rows as they are (hyper-parameters are per-trainer, always kept)."""
    K = K or trainer.capacity
    row = parameter if not isinstance(parameter, dict) else trainer.layout.flatten(parameter)
    trainer.load_global(row, K)
    if not reuse_learning_rate:
        trainer.reset_optimizer(K)
