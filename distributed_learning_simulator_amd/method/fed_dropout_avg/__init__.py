"""FedDropoutAvg (arXiv 2111.13230) — reference `method/fed_dropout_avg/*`.

Client: uploads full parameters θ_k ⊙ m_k, m_k ~ Bernoulli(1 − dropout_rate) per element
(`fed_dropout_avg/worker.py:16-30`); the mask is a counter-based hash of (seed, round,
client, element) generated on device in one launch for the whole cohort.
Server: per-element weights n_k·[θ_k⊙m_k ≠ 0], zero total weight → 1 so fully-dropped
elements become 0 (`fed_dropout_avg/algorithm.py:8-19`).
Wire bytes: only the kept elements are charged (the reference's analysis sums the logged
`send_num`, `analyze_log.py:172-190`).
"""

from __future__ import annotations

from ...algorithm.fed_avg_algorithm import FedAVGAlgorithm
from ...message import CohortMessage
from ...ops import fl
from ...server.aggregation_server import AggregationServer
from ...topology.endpoints import ClientEndpoint
from ...utils.logging import get_logger
from ...worker.aggregation_worker import AggregationWorker
from ..algorithm_factory import CentralizedAlgorithmFactory


class FedDropoutAvgWorker(AggregationWorker):
    def __init__(self, config, endpoint, session=None, **kwargs):
        super().__init__(config, endpoint, session, **kwargs)
        self._dropout_rate = float(config.algorithm_kwargs["dropout_rate"])
        self._send_parameter_diff = False
        get_logger().info("use dropout_rate %s", self._dropout_rate)

    def _get_sent_data(self, wave, theta_g, stats) -> CohortMessage:
        msg = super()._get_sent_data(wave, theta_g, stats)
        K, P = msg.data.shape
        seed = (self.config.seed * 1_000_003 + self._round_num * 7919) & 0x7FFFFFFF
        mask = fl.dropout_mask((K, P), self._dropout_rate, fl.row_seeds(seed, list(wave)), msg.data.device)
        mask &= self.session.layout.valid_mask(msg.data.device).unsqueeze(0)
        msg.data.mul_(mask)
        msg.mask = mask
        send_num = mask.sum(1).tolist()
        msg.extra["send_num"] = send_num
        for c, n in zip(wave, send_num):
            get_logger().debug("worker %d send_num %s", c, n)
        return msg


class FedDropoutAvgAlgorithm(FedAVGAlgorithm):
    expected_kind = "parameter"
    expects_element_mask = True


class SparseClientEndpoint(ClientEndpoint):
    """Charges only the transmitted (non-dropped) elements, 4 B each."""

    def encode(self, msg, seed):
        if "send_num" in msg.extra:
            msg.wire_bytes = [int(n) * 4 for n in msg.extra["send_num"]]
        else:
            msg.wire_bytes = self._dense_wire(msg)
        return msg


CentralizedAlgorithmFactory.register_algorithm(
    algorithm_name="fed_dropout_avg",
    client_cls=FedDropoutAvgWorker,
    server_cls=AggregationServer,
    client_endpoint_cls=SparseClientEndpoint,
    algorithm_cls=FedDropoutAvgAlgorithm,
)
