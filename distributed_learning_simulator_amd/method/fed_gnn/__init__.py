"""Federated GNN (node-split): `fed_gnn`, `fed_gcn` (share_feature forced) and the
config-only `fed_aas` (treated as fed_gnn with its configs' defaults).

Reference `worker/graph_worker.py` + `algorithm/graph_algorithm.py` + `server/graph_server.py`
(SURVEY C16/C19/C22, §3.6): training nodes are split among clients; each client trains a GCN
on its kept edges; with `share_feature`, message-passing layers ≥ 1 see the boundary-node
embeddings computed by the other clients (exchanged every batch, every layer); GCN weights are
FedAvg-aggregated per round; `graph_worker_stat.json` records edge counts and per-round
communicated / skipped embedding bytes.

MI355X-native: all clients of a rank run the GCN together over one concatenated edge list
(client-offset node ids → one gather/scatter per layer), the node features are shared and the
first layer is ONE GEMM against the concatenated client weights; the per-batch halo exchange
is an on-device gather, merged across ranks with one all-reduce of the boundary table.
Full-graph propagation per batch (loss on the batch's seed nodes); neighbour sampling
(`num_neighbor`) is accepted and recorded but not applied (parity unpinned).
"""

from __future__ import annotations

import json
import math
import os

import torch

from ...algorithm.fed_avg_algorithm import FedAVGAlgorithm
from ...data.graph import ClientGraphViews
from ...server.aggregation_server import AggregationServer
from ...utils.logging import get_logger
from ...worker.aggregation_worker import AggregationWorker
from ..algorithm_factory import CentralizedAlgorithmFactory


class GraphWorker(AggregationWorker):
    force_share_feature: bool | None = None

    def __init__(self, config, endpoint, session=None, **kwargs):
        super().__init__(config, endpoint, session, **kwargs)
        ak = config.algorithm_kwargs
        self._share_feature = bool(ak.get("share_feature", True)) if self.force_share_feature is None \
            else self.force_share_feature
        self._batch_number = int(ak.get("batch_number", 1) or 1)
        self._edge_drop_rate = ak.get("edge_drop_rate")
        self._views: dict = {}
        self._owner = None
        self._communicated_embedding_bytes = 0
        self._aggregated_bytes = 0
        self._round_communicated_bytes: dict = {}
        self._round_skipped_bytes: dict = {}
        self._stats: dict = {}
        ds = session.dc.graph
        ds.comm = session.comm

    def shards(self, client_ids):
        ds = self.session.dc.graph
        return [ds.node_ids(self.session.practitioners[c].indices(self.session.dc.spec.name)) for c in client_ids]

    def _ensure_owner(self):
        if self._owner is None:
            ds = self.session.dc.graph
            owner = torch.full((ds.num_nodes,), -1, dtype=torch.int64)
            for c in range(self.config.worker_number):
                owner[self.shards([c])[0]] = c
            self._owner = owner
            if self.session.is_main:
                get_logger().info("%s feature", "share" if self._share_feature else "not share")

    def _views_for(self, wave):
        key = tuple(wave)
        if key not in self._views:
            self._ensure_owner()
            self._views[key] = ClientGraphViews(self.session.dc.graph, self._owner, list(wave), self._share_feature,
                                                self._edge_drop_rate, self.config.seed)
        return self._views[key]

    def build_schedule(self, round_num, wave):
        shards = self.shards(wave)
        ds = self.session.dc.graph
        # every rank runs the same number of steps (the halo all-reduce is collective)
        max_shard = max(self.session.practitioners[c].dataset_size(self.session.dc.spec.name)
                        for c in range(self.config.worker_number))
        B = max(1, math.ceil(max_shard / self._batch_number))
        saved = self.trainer.hyper.batch_size
        self.trainer.hyper.batch_size = B
        try:
            return self.trainer.build_schedule(shards, self.local_epochs(),
                                               seed=self.config.seed * 100_003 + round_num * 1009, client_ids=list(wave),
                                               min_steps_per_epoch=self._batch_number)
        finally:
            self.trainer.hyper.batch_size = saved

    def train_wave(self, round_num, theta_g, wave):
        views = self._views_for(wave)
        self.session.dc.graph.views = views
        msg = super().train_wave(round_num, theta_g, wave)
        # embedding exchange accounting: per step, every layer >= 1, each client sends its
        # boundary rows (reference `_pass_node_feature`, fp32 element size)
        layers = len(self.session.model.root.convs)
        hidden = [c.lin.fout for c in self.session.model.root.convs[:-1]]
        steps = self._batch_number * self.local_epochs()
        if self._share_feature and layers > 1:
            per_step = sum(cnt * sum(hidden[: layers - 1]) * 4 for cnt in views.boundary_cnt)
            self._communicated_embedding_bytes += per_step * steps
            msg.wire_bytes = [w for w in msg.wire_bytes]
            msg.extra["embedding_bytes"] = per_step * steps
        self._aggregated_bytes += int(sum(msg.wire_bytes))
        self._round_communicated_bytes[round_num] = self._aggregated_bytes + self._communicated_embedding_bytes
        self._round_skipped_bytes[round_num] = 0
        for c, st in zip(wave, views.stats):
            self._stats[c] = st
        return msg

    def _after_training(self) -> None:
        if not self.session.is_main:
            return
        os.makedirs(self.save_dir, exist_ok=True)
        model_bytes = self.session.layout.num_params * 4
        stat = {"per_client": {str(k): v for k, v in self._stats.items()},
                "skipped_embedding_bytes": self._round_skipped_bytes,
                "communicated_bytes": self._round_communicated_bytes,
                "model_bytes": model_bytes}
        with open(os.path.join(self.save_dir, "graph_worker_stat.json"), "wt", encoding="utf8") as f:
            json.dump(stat, f)


class FedGCNWorker(GraphWorker):
    """FedGCN (arXiv 2201.12433): share_feature forced (`method/fed_gcn/worker.py:4-7`)."""

    force_share_feature = True


class GraphNodeServer(AggregationServer):
    """Reference `server/graph_server.py:5-7`: FedAvg of the GCN weights; the embedding
    relay is the on-device halo table (no server round trip)."""


for _name, _client in (("fed_gnn", GraphWorker), ("fed_gcn", FedGCNWorker), ("fed_aas", GraphWorker)):
    CentralizedAlgorithmFactory.register_algorithm(
        algorithm_name=_name, client_cls=_client, server_cls=GraphNodeServer, algorithm_cls=FedAVGAlgorithm)
