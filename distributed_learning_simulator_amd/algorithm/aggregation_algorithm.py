"""Server-side aggregation algorithm base.

Reference `algorithm/aggregation_algorithm.py:9-96`: `get_ratios`, `weighted_avg` (static,
dict-of-messages form — kept for API parity and used by tests/analysis),
`process_worker_data(worker_id, worker_data, old_parameter_dict, save_dir)` (`None` ⇒
skipped worker), `aggregate_worker_data()`, `clear_worker_data()`, `exit()`.

Cohort form: `process_worker_data` receives a `CohortMessage` holding the uploads of every
client of one resident cohort (device rows), and the aggregation is a fused weighted
row-reduction followed by one all-reduce across ranks (see `FedAVGAlgorithm`).
"""

from __future__ import annotations

from typing import Any

import torch

from ..message import CohortMessage, Message, ParameterMessage
from ..parallel.comm import get_comm
from ..utils.logging import get_logger


class AggregationAlgorithm:
    def __init__(self) -> None:
        self._skipped_workers: set[int] = set()
        self._worker_ids: list[int] = []
        self._other_data: dict = {}
        self._end_training: bool | None = None
        self.config = None
        self.layout = None
        self.device = torch.device("cpu")
        self.comm = get_comm()
        self.server = None

    def bind(self, config, layout, device, comm=None, server=None) -> None:
        self.config = config
        self.layout = layout
        self.device = torch.device(device)
        self.comm = comm or get_comm()
        self.server = server

    # --------------------------------------------------------- reference helpers
    @classmethod
    def get_ratios(cls, data_dict: dict[int, ParameterMessage], key_name: str | None = None) -> dict[int, float]:
        if key_name is None:
            total = sum(v.dataset_size for v in data_dict.values())
            return {k: float(v.dataset_size) / float(total) for k, v in data_dict.items()}
        total = sum(v.other_data[key_name] for v in data_dict.values())
        return {k: float(v.other_data[key_name]) / float(total) for k, v in data_dict.items()}

    @classmethod
    def weighted_avg(cls, data_dict: dict[int, ParameterMessage], weight_dict: dict[int, float]) -> dict:
        assert data_dict
        avg: dict[str, torch.Tensor] = {}
        for wid, v in data_dict.items():
            ratio = weight_dict[wid]
            assert 0 <= ratio <= 1
            for k, t in v.parameter.items():
                avg[k] = avg[k] + t * ratio if k in avg else t * ratio
        for t in avg.values():
            assert not t.isnan().any()
        return avg

    # ------------------------------------------------------------- cohort API
    def _check_other_data(self, msg: Message) -> None:
        """`fed_avg_algorithm.py:99-110`: other_data must agree across workers."""
        for k, v in msg.other_data.items():
            if k in self._other_data and self._other_data[k] != v:
                get_logger().error("different values on key %s", k)
                raise RuntimeError(f"different values on key {k}")
            self._other_data[k] = v
        if self._end_training is None:
            self._end_training = msg.end_training

    def process_worker_data(self, worker_data: CohortMessage | None, old_parameter: torch.Tensor | None,
                            worker_ids: list[int] | None = None, save_dir: str | None = None) -> None:
        if worker_data is None:
            self._skipped_workers.update(worker_ids or [])
            return
        self._check_other_data(worker_data)
        self._worker_ids.extend(worker_data.client_ids)
        self._process(worker_data, old_parameter)

    def _process(self, msg: CohortMessage, old_parameter) -> None:
        raise NotImplementedError

    def aggregate_worker_data(self, old_parameter: torch.Tensor) -> Any:
        raise NotImplementedError

    def clear_worker_data(self) -> None:
        self._skipped_workers.clear()
        self._worker_ids.clear()
        self._other_data = {}
        self._end_training = None

    def exit(self) -> None:
        pass
