"""Update sparsification with error feedback.

Reference `worker/error_feedback_worker.py:9-19`: an abstract AggregationWorker that
requires diff uploads (`send_parameter_diff`), keeps an `_error` residual and leaves
`sparsify()` unimplemented (no concrete subclass in the reference tree).

Here the residual is a per-client row of a device buffer: each round a client uploads
S(Δ + e) and keeps e ← (Δ + e) − S(Δ + e). The residual lives on the rank that trains the
client, so the client→rank assignment must be stable across rounds (full participation, or
one rank). `TopKErrorFeedbackWorker` is a concrete sparsifier (largest-|x| fraction per
client row; wire bytes = k values + k int32 indices).
"""

from __future__ import annotations

import torch

from ..message import CohortMessage
from .aggregation_worker import AggregationWorker


class ErrorFeedbackWorker(AggregationWorker):
    def __init__(self, config, endpoint, session=None, **kwargs):
        super().__init__(config, endpoint, session, **kwargs)
        assert self._send_parameter_diff, "error feedback needs delta uploads"
        self._error: torch.Tensor | None = None  # [worker_number, P_pad] residuals

    def state_dict(self) -> dict:
        return {"error": self._error.cpu()} if self._error is not None else {}

    def load_state_dict(self, state: dict) -> None:
        if "error" in state:
            self._error = state["error"].to(self.trainer.buffers.theta.device)

    def sparsify(self, rows: torch.Tensor) -> tuple[torch.Tensor, list[int]]:
        """rows [K,P] (Δ + e) → (sparse rows [K,P] with zeros where not sent, wire bytes per row)."""
        raise NotImplementedError

    def _error_rows(self, wave: list[int], P: int, device) -> torch.Tensor:
        if self._error is None:
            W = self.config.worker_number
            sel = self.config.algorithm_kwargs.get("random_client_number", W) or W
            world = self.session.comm.world if self.session is not None else 1
            assert sel >= W or world == 1, "error feedback residuals need a stable client→rank assignment"
            self._error = torch.zeros((W, P), dtype=torch.float32, device=device)
        return self._error[torch.tensor(wave, device=device)]

    def _get_sent_data(self, wave, theta_g, stats) -> CohortMessage:
        msg = super()._get_sent_data(wave, theta_g, stats)
        rows = msg.data
        idx = torch.tensor(wave, device=rows.device)
        rows += self._error_rows(wave, rows.shape[1], rows.device)
        sparse, nbytes = self.sparsify(rows)
        self._error[idx] = rows - sparse
        rows.copy_(sparse)
        msg.extra["wire_bytes"] = list(nbytes)
        return msg


class TopKErrorFeedbackWorker(ErrorFeedbackWorker):
    def __init__(self, config, endpoint, session=None, **kwargs):
        super().__init__(config, endpoint, session, **kwargs)
        self.ratio = float(config.algorithm_kwargs.get("topk_ratio", 0.01))

    def sparsify(self, rows):
        n = self.trainer.layout.num_params
        k = max(1, int(n * self.ratio))
        valid = self.trainer.layout.valid_mask(rows.device)
        mag = rows.abs().masked_fill(~valid, -1.0)
        top = mag.topk(k, dim=1).indices
        out = torch.zeros_like(rows)
        out.scatter_(1, top, rows.gather(1, top))
        return out, [k * 8] * rows.shape[0]
