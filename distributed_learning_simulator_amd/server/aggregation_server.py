"""Synchronous-round FL server.

Reference `server/aggregation_server.py:15-184`: init model (pickle from
`algorithm_kwargs.global_model_path` or tester random init), send θ0 with `in_round=True`,
aggregate when all workers reported, evaluate + record `round_record.json` and
`best_global_model.pk`, early stop on a 5-round plateau, cache
`aggregated_model/round_N.pk`, `round += 1` unless `in_round`.

Fixed defects: B6 (early stop now also stops the server: `_stopped` checks the end flag),
B7 (plateau compared against the best accuracy *before* this round).
Checkpoints are written with `torch.save` of a name→tensor dict (loadable with
`torch.load(weights_only=True)`), not pickle.
"""

from __future__ import annotations

import json
import os

import torch

from ..message import FlatParameterMessage, Message
from ..utils.logging import get_logger
from .server import Server


class AggregationServer(Server):
    def __init__(self, config, endpoint, algorithm=None, session=None, **kwargs):
        super().__init__(config, endpoint, algorithm, session, **kwargs)
        self._round_number = 1
        self._compute_stat = True
        self._stat: dict = {}
        self._max_acc = 0.0
        self._plateau = 0
        self._ended = False
        self.need_init_performance = False
        self.early_stop = bool(config.algorithm_kwargs.get("early_stop", False))
        self.global_parameter: torch.Tensor | None = None
        self.selected: list[int] = []
        self.last_result = None

    @property
    def round_number(self) -> int:
        return self._round_number

    def state_dict(self) -> dict:
        st = {"max_acc": self._max_acc, "plateau": self._plateau, "ended": self._ended,
              "selected": list(self.selected)}
        if self._algorithm is not None and hasattr(self._algorithm, "state_dict"):
            st["algorithm"] = self._algorithm.state_dict()
        return st

    def load_state_dict(self, state: dict) -> None:
        self._max_acc = float(state.get("max_acc", 0.0))
        self._plateau = int(state.get("plateau", 0))
        self._ended = bool(state.get("ended", False))
        self.selected = list(state.get("selected", []))
        if "algorithm" in state and self._algorithm is not None and hasattr(self._algorithm, "load_state_dict"):
            self._algorithm.load_state_dict(state["algorithm"])

    @property
    def performance_stat(self) -> dict:
        return self._stat

    def _get_stat_key(self):
        return self._round_number

    # ------------------------------------------------------------------ init
    def get_init_model(self) -> torch.Tensor:
        layout = self.session.layout
        path = self.config.algorithm_kwargs.get("global_model_path")
        if path:
            tensors = torch.load(path, map_location="cpu", weights_only=True)
            flat = layout.init_flat(torch.Generator().manual_seed(self.config.seed))
            return layout.flatten(tensors, flat)
        return layout.init_flat(torch.Generator().manual_seed(self.config.seed))

    def _before_start(self) -> FlatParameterMessage:
        theta0 = self.get_init_model().to(self.session.device)
        self.global_parameter = theta0
        return FlatParameterMessage(parameter=theta0, layout=self.session.layout, in_round=True,
                                    other_data={"init": True})

    # --------------------------------------------------------------- process
    def _process_worker_data(self, msg, worker_ids=None) -> None:
        msg = self.endpoint.get(msg, defer_payload=bool(getattr(self._algorithm, "fuses_payload", False)))
        self._algorithm.process_worker_data(msg, self.global_parameter, worker_ids=worker_ids,
                                            save_dir=self.save_dir)

    def _aggregate_worker_data(self) -> Message:
        return self._algorithm.aggregate_worker_data(self.global_parameter)

    # ------------------------------------------------------------ send result
    def _before_send_result(self, result: Message) -> None:
        if not isinstance(result, FlatParameterMessage):
            return
        if self.need_init_performance and "init" in result.other_data:
            self._record_compute_stat(result.parameter, key=0)
        elif self._compute_stat and "init" not in result.other_data:
            if self._should_eval(result):
                self._record_compute_stat(result.parameter)
                if not result.end_training and self.early_stop and self._convergent():
                    result.end_training = True
        elif result.end_training:
            self._record_compute_stat(result.parameter)
        self.global_parameter = result.parameter
        # (`limited_resource` does not spill here: its memory saving is the smaller HBM budget
        # fraction the session gives client cohorts, session.py; a per-round file nobody reads
        # back would only cost disk writes)
        if self.config.save_models and self.session.is_main and "init" not in result.other_data:
            self._save_model(result.parameter, os.path.join(self.config.save_dir, "aggregated_model",
                                                            f"round_{self._round_number}.pk"))

    def _should_eval(self, result) -> bool:
        every = max(1, int(self.config.eval_every))
        return self._round_number % every == 0 or self._round_number >= self.config.round or result.end_training

    def send_result(self, result: FlatParameterMessage) -> tuple[torch.Tensor, int]:
        """Broadcast to the next round's selected workers (M5/M1); `None` to the rest (M2,
        0 bytes). Returns (parameters as the clients receive them, downlink bytes)."""
        self._before_send_result(result)
        self.last_result = result
        if result.end_training:
            self._ended = True
        self.selected = self._select_workers_next(result)
        received, nbytes = self.endpoint.broadcast(result.parameter, len(self.selected),
                                                   seed=self.config.seed * 31 + self._round_number)
        self._after_send_result(result)
        return received, nbytes

    def _select_workers_next(self, result) -> list[int]:
        # selection for the round that this broadcast starts
        saved = self._round_number
        if not result.in_round:
            self._round_number += 1
        sel = self._select_workers()
        self._round_number = saved
        return sel

    def _after_send_result(self, result: Message) -> None:
        if isinstance(result, FlatParameterMessage) and not result.in_round:
            self._round_number += 1
        if self._algorithm is not None:
            self._algorithm.clear_worker_data()

    def _stopped(self) -> bool:
        return self._ended or self._round_number > self.config.round

    # ------------------------------------------------------------- records
    def _record_compute_stat(self, parameter: torch.Tensor, key=None) -> None:
        metric = self.get_metric(parameter)
        round_stat = {f"test_{k}": v for k, v in metric.items()}
        # synthetic data (the default, no network): accuracy is not comparable with the reference
        round_stat["synthetic"] = bool(getattr(self.session.dc, "synthetic", True))
        key = self._get_stat_key() if key is None else key
        self._stat[key] = round_stat
        self.last_recorded = (key, round_stat)
        get_logger().info("round: %s, test accuracy %.4f loss %.4f", key, metric["accuracy"], metric["loss"])
        if self.session.is_main:
            os.makedirs(self.save_dir, exist_ok=True)
            with open(os.path.join(self.save_dir, "round_record.json"), "wt", encoding="utf8") as f:
                json.dump(self._stat, f)
        if key == 0:
            return
        # plateau bookkeeping against the best accuracy *before* this round (fixes B7)
        if metric["accuracy"] > self._max_acc + 0.001:
            self._plateau = 0
        else:
            self._plateau += 1
            get_logger().info("plateau is %s (best %.4f, current %.4f)", self._plateau, self._max_acc,
                              metric["accuracy"])
        if metric["accuracy"] > self._max_acc:
            self._max_acc = metric["accuracy"]
            if self.config.save_models and self.session.is_main:
                self._save_model(parameter, os.path.join(self.save_dir, "best_global_model.pk"))

    def _convergent(self) -> bool:
        """≥5 consecutive evaluations without beating the best by 0.001
        (reference `aggregation_server.py:166-184`)."""
        return self._plateau >= 5

    def _save_model(self, parameter: torch.Tensor, path: str) -> None:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tensors = {k: v.detach().cpu().clone() for k, v in self.session.layout.unflatten(parameter).items()}
        torch.save(tensors, path)
