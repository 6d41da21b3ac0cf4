"""Offline analysis of finished runs (reference `simulation_lib/analysis/`):
session readers, log-based accuracy / communication-volume accounting, per-round curves,
the federated-GNN experiment table and the per-module parameter-change hook."""

from .analyze_log import compute_acc, compute_data_amount
from .module_diff import ModuleDiff
from .session import GraphSession, Session

__all__ = ["Session", "GraphSession", "compute_acc", "compute_data_amount", "ModuleDiff"]
