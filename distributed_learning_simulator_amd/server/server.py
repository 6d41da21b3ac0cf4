"""Server role (replicated on every rank).

Reference `server/server.py:20-134`: lazy tester on the Test split, `get_metric(params)`,
poll loop over worker pipes, `_send_result` (per-worker unicast or broadcast to
`_select_workers()` and `None` to the rest), `_select_workers` (uniform
`random_client_number` or all). Here there is no polling: the `Session` drives the round
and every rank runs an identical server replica (deterministic selection seeded by round),
so the "broadcast" is free between ranks and only its simulated wire bytes are charged.
"""

from __future__ import annotations

import os
import random

import torch

from ..executor import Executor
from ..utils.logging import get_logger


class Server(Executor):
    def __init__(self, config, endpoint, algorithm=None, session=None, **kwargs):
        super().__init__(config, "server", session)
        self.endpoint = endpoint
        self._algorithm = algorithm
        self.worker_number = config.worker_number

    @property
    def algorithm(self):
        return self._algorithm

    # reference server.py:123-131
    def _select_workers(self) -> list[int]:
        n = self.config.algorithm_kwargs.get("random_client_number")
        if n is None or int(n) >= self.worker_number:
            return list(range(self.worker_number))
        rng = random.Random((self.config.seed + 1) * 1_000_003 + self._selection_key() * 7919)
        return sorted(rng.sample(range(self.worker_number), int(n)))

    def _selection_key(self) -> int:
        """Seed of the round's client selection: the round number (not the stat key, which
        stays constant between evaluations when `eval_every` > 1 or in FedOBD's stage 1)."""
        return int(getattr(self, "_round_number", 0))

    def _get_stat_key(self):
        return 0

    def get_metric(self, parameter: torch.Tensor) -> dict:
        """Test-split metric of a flat parameter vector (sharded across ranks)."""
        loss, acc = self.session.evaluate(parameter)
        return {"loss": float(loss[0]), "accuracy": float(acc[0])}

    def get_metrics_many(self, rows: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        return self.session.evaluate(rows)

    def _server_exit(self) -> None:
        if self._algorithm is not None:
            self._algorithm.exit()
        get_logger().debug("server exits")
