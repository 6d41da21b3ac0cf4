"""FedPAQ (arXiv 1909.13014) — reference `method/fed_paq/__init__.py:7-14`: FedAvg with
255-level stochastic quantisation of the client uploads (of Δ — fixed B3: the reference's
client endpoint skipped Δ messages although its analysis charges 1 B/param for uploads),
unquantised downlink, typically partial participation."""

from ...algorithm.fed_avg_algorithm import FedAVGAlgorithm
from ...server.aggregation_server import AggregationServer
from ...topology.endpoints import StochasticQuantClientEndpoint, StochasticQuantServerEndpoint
from ...worker.aggregation_worker import AggregationWorker
from ..algorithm_factory import CentralizedAlgorithmFactory

CentralizedAlgorithmFactory.register_algorithm(
    algorithm_name="fed_paq",
    client_cls=AggregationWorker,
    server_cls=AggregationServer,
    client_endpoint_cls=StochasticQuantClientEndpoint,
    server_endpoint_cls=StochasticQuantServerEndpoint,
    algorithm_cls=FedAVGAlgorithm,
)
