"""single_model_afd — config-only in the reference (`conf/smafd/*`, `conf/large_scale/smafd/*`,
`dropout_rate: 0.3`); its building block is the unused `RandomDropoutAlgorithm`
(`algorithm/random_dropout_algorithm.py:7-31`): shuffle the parameter tensors and keep whole
tensors while the kept size stays ≤ (1 − dropout_rate)·P. That file never increments its
counter (B5); here the budget is enforced. Server: each tensor is averaged over the clients
that sent it, tensors nobody sent keep θ_g. Wire bytes: kept elements × 4 B (the
reference's analysis sums the logged `send_num`, `analyze_log.py:191-209`).
"""

from __future__ import annotations

import random

import torch

from ...algorithm.fed_avg_algorithm import FedAVGAlgorithm
from ...message import CohortMessage
from ...server.aggregation_server import AggregationServer
from ...topology.endpoints import ClientEndpoint
from ...worker.aggregation_worker import AggregationWorker
from ..algorithm_factory import CentralizedAlgorithmFactory


def random_tensor_subset(numels: list[int], dropout_rate: float, rng: random.Random) -> list[int]:
    order = list(range(len(numels)))
    rng.shuffle(order)
    budget = (1 - dropout_rate) * sum(numels)
    kept, partial = [], 0
    for i in order:
        if partial + numels[i] <= budget:
            kept.append(i)
            partial += numels[i]  # (B5 fix: the reference never incremented this)
    return sorted(kept)


class SingleModelAFDWorker(AggregationWorker):
    def __init__(self, config, endpoint, session=None, **kwargs):
        super().__init__(config, endpoint, session, **kwargs)
        self._dropout_rate = float(config.algorithm_kwargs.get("dropout_rate", 0.3))

    def _get_sent_data(self, wave, theta_g, stats) -> CohortMessage:
        msg = super()._get_sent_data(wave, theta_g, stats)
        layout = self.session.layout
        numels = [e.numel for e in layout.entries]
        ids = _tensor_ids(layout, msg.data.device)
        K = len(wave)
        mask = torch.zeros((K, len(numels)), dtype=torch.bool)
        for i, c in enumerate(wave):
            rng = random.Random((self.config.seed * 1_000_003 + self._round_num * 7919 + c) & 0x7FFFFFFF)
            mask[i, random_tensor_subset(numels, self._dropout_rate, rng)] = True
        mask = mask.to(msg.data.device)
        msg.data.mul_(mask[:, ids.clamp(min=0).long()] & (ids >= 0)[None, :])
        msg.block_mask = mask
        msg.extra["block_ids"] = ids
        msg.extra["block_param_sizes"] = torch.tensor(numels, device=msg.data.device)
        return msg


_ids_cache: dict = {}


def _tensor_ids(layout, device):
    key = (id(layout), str(device))
    if key not in _ids_cache:
        ids = layout.segment_ids(device)
        ids[ids == len(layout.entries)] = -1
        _ids_cache[key] = ids
    return _ids_cache[key]


class SingleModelAFDServer(AggregationServer):
    def _before_start(self):
        msg = super()._before_start()
        self._algorithm.num_blocks = len(self.session.layout.entries)
        self._algorithm.block_ids = _tensor_ids(self.session.layout, self.session.device)
        return msg


CentralizedAlgorithmFactory.register_algorithm(
    algorithm_name="single_model_afd",
    client_cls=SingleModelAFDWorker,
    server_cls=SingleModelAFDServer,
    client_endpoint_cls=ClientEndpoint,
    algorithm_cls=FedAVGAlgorithm,
)
