"""Practitioner = a logical client identity bound to a data shard.

Reference `practitioner.py:5-35`: `Practitioner(id)`, `worker_id` (defaults to id,
`set_worker_id`), `set_sampler`, `has_dataset`, `create_trainer(config)`. Here a
practitioner only holds its shard's *indices*; the data stays device-resident in the
rank's `DatasetCollection` and the cohort trainer gathers batches from it.
"""

from __future__ import annotations

import torch

from .sampler import get_partition


class Practitioner:
    def __init__(self, practitioner_id: int):
        self.id = practitioner_id
        self._worker_id: int | None = None
        self._datasets: dict[str, torch.Tensor] = {}

    @property
    def worker_id(self) -> int:
        return self.id if self._worker_id is None else self._worker_id

    def set_worker_id(self, worker_id: int) -> None:
        self._worker_id = worker_id

    def set_sampler(self, name: str, indices: torch.Tensor) -> None:
        self._datasets[name] = indices

    def has_dataset(self, name: str) -> bool:
        return name in self._datasets

    def indices(self, name: str) -> torch.Tensor:
        return self._datasets[name]

    def dataset_size(self, name: str) -> int:
        return int(self._datasets[name].numel())

    def __repr__(self) -> str:
        return f"Practitioner({self.id})"


def create_practitioners(config, labels: torch.Tensor | None = None) -> list[Practitioner]:
    """Reference `config.py:55-72`: one practitioner per worker with the configured
    sampler's shard."""
    from .data.datasets import get_spec

    if labels is None:
        from .data.datasets import create_dataset_collection

        dc = create_dataset_collection(config.dataset_name, config.dataset_kwargs, config.seed, "cpu")
        labels = dc.train.labels
    spec = get_spec(config.dataset_name, config.dataset_kwargs)
    parts = get_partition(config.dataset_sampling, labels, config.worker_number, seed=config.seed,
                          **(config.dataset_sampling_kwargs or {}))
    out = []
    for pid in range(config.worker_number):
        p = Practitioner(pid)
        p.set_sampler(spec.name, parts[pid])
        out.append(p)
    return out
