"""Readers for a finished experiment's output directory.

Reference `analysis/session.py:9-63`: `Session(session_dir)` loads the server's
`round_record.json` (round → metrics) and the pickled config, and walks sibling `worker*`
directories for per-worker data; `GraphSession` adds each worker's `graph_worker_stat.json`.

Here every file is JSON (no pickle/dill): the session directory is `config.save_dir`
(`session/<algo>/<dataset>_<sampling>/<model>/<date>/<uuid>`), holding
  server/round_record.json         (AggregationServer._record_compute_stat)
  config.json                      (Session.run)
  metrics.jsonl                    (per-round wall time / comm bytes, the BASELINE metric)
  worker_rank<r>/*.json            (per-rank worker stats: epoch_stat.json, graph_worker_stat.json)
`session_dir` may be the save_dir itself or its `server/` sub-directory.
"""

from __future__ import annotations

import functools
import json
import os


def _find_root(session_dir: str) -> str:
    session_dir = os.path.abspath(session_dir)
    if os.path.isfile(os.path.join(session_dir, "server", "round_record.json")):
        return session_dir
    if os.path.isfile(os.path.join(session_dir, "round_record.json")):
        return os.path.dirname(session_dir) if os.path.basename(session_dir) == "server" else session_dir
    raise FileNotFoundError(f"no round_record.json under {session_dir}")


class Session:
    def __init__(self, session_dir: str):
        self.root = _find_root(session_dir)
        rr = os.path.join(self.root, "server", "round_record.json")
        if not os.path.isfile(rr):
            rr = os.path.join(self.root, "round_record.json")
        with open(rr, "rt", encoding="utf8") as f:
            self.round_record = {int(k): v for k, v in json.load(f).items()}
        self.config: dict = {}
        cfg = os.path.join(self.root, "config.json")
        if os.path.isfile(cfg):
            with open(cfg, "rt", encoding="utf8") as f:
                self.config = json.load(f)
        self.metrics: list[dict] = []
        mpath = os.path.join(self.root, "metrics.jsonl")
        if os.path.isfile(mpath):
            with open(mpath, "rt", encoding="utf8") as f:
                self.metrics = [json.loads(line) for line in f if line.strip()]
        self.worker_data: dict[str, dict] = {}
        for name in sorted(os.listdir(self.root)):
            path = os.path.join(self.root, name)
            if name.startswith("worker") and os.path.isdir(path):
                self.worker_data[name] = self._load_worker(path)

    @staticmethod
    def _load_worker(path: str) -> dict:
        data = {}
        for f in sorted(os.listdir(path)):
            if f.endswith(".json"):
                with open(os.path.join(path, f), "rt", encoding="utf8") as fh:
                    data[f[:-5]] = json.load(fh)
        return data

    @functools.cached_property
    def rounds(self) -> list[int]:
        return sorted(k for k in self.round_record if k > 0) or sorted(self.round_record)

    @functools.cached_property
    def last_round(self) -> int:
        return self.rounds[-1]

    @functools.cached_property
    def last_test_acc(self) -> float:
        return self.round_record[self.last_round]["test_accuracy"]

    @functools.cached_property
    def mean_test_acc(self) -> float:
        rows = [self.round_record[r]["test_accuracy"] for r in self.rounds]
        return sum(rows) / len(rows)

    @functools.cached_property
    def rounds_per_s(self) -> float | None:
        walls = [m["wall_s"] for m in self.metrics if "wall_s" in m]
        return len(walls) / sum(walls) if walls else None

    @functools.cached_property
    def comm_bytes_per_round(self) -> float | None:
        b = [m["comm_bytes_total"] for m in self.metrics if "comm_bytes_total" in m]
        return sum(b) / len(b) if b else None


class GraphSession(Session):
    """Session whose workers wrote `graph_worker_stat.json` (fed_gnn / fed_gcn / fed_aas)."""

    def __init__(self, session_dir: str):
        super().__init__(session_dir)
        self.worker_data = {k: v.get("graph_worker_stat", v) for k, v in self.worker_data.items()}
