"""One-row experiment summary of a federated-GNN session, appended to `exp.txt` / `exp.json`.

Reference `analysis/graph_exp_analyzer.py:14-91`: from a `GraphSession`, collect the config
(algorithm, dataset, model, rounds, workers, algorithm_kwargs, extra hyper-parameters), last /
mean test accuracy, per-worker byte counters summed over workers and edge/node counts as
mean±std, the full per-round performance record; sort columns, append to `exp.txt` (CSV) and
write `exp.xlsx` / `exp.json`. The xlsx is written only when an Excel writer is importable.

    session_path=session/fed_gnn/... python -m distributed_learning_simulator_amd.analysis.graph_exp_analyzer
"""

from __future__ import annotations

import json
import os
import statistics
import sys

import pandas as pd

from .session import GraphSession


def summarize(session_path: str) -> dict:
    s = GraphSession(session_path)
    cfg = s.config
    res: dict = {
        "exp_name": cfg.get("exp_name", ""),
        "distributed_algorithm": cfg.get("distributed_algorithm"),
        "dataset_name": cfg.get("dataset_name"),
        "model_name": cfg.get("model_name"),
        "round": cfg.get("round"),
        "worker_number": cfg.get("worker_number"),
    }
    res |= cfg.get("algorithm_kwargs") or {}
    res |= cfg.get("extra_hyper_parameters") or {}
    res["last_test_acc"] = s.last_test_acc
    res["mean_test_acc"] = s.mean_test_acc
    counters: dict = {}
    per_client_counts: dict[str, list[float]] = {}
    for data in s.worker_data.values():
        for k, v in data.items():
            if k == "model_bytes":
                counters[k] = v
            elif k == "per_client":
                for stats in v.values():
                    for name, cnt in stats.items():
                        if "edge_cnt" in name or "node_cnt" in name:
                            per_client_counts.setdefault(name, []).append(float(cnt))
            elif isinstance(v, dict) and ("byte" in k or "cnt" in k):
                acc = counters.setdefault(k, {})
                for rk, rv in v.items():
                    acc[rk] = acc.get(rk, 0) + rv
    for name, vals in per_client_counts.items():
        counters[name] = {"mean": statistics.fmean(vals), "std": statistics.stdev(vals) if len(vals) > 1 else 0.0}
    res |= counters
    res["performance"] = {str(k): v for k, v in s.round_record.items()}
    return res


def write(res: dict, out_prefix: str = "exp") -> pd.DataFrame:
    flat = {k: json.dumps(v) if isinstance(v, dict) else v for k, v in res.items()}
    lead = ["exp_name", "distributed_algorithm", "dataset_name", "model_name", "last_test_acc", "mean_test_acc",
            "round", "worker_number"]
    cols = [c for c in lead if c in flat] + sorted(set(flat) - set(lead))
    df = pd.DataFrame([flat])[cols]
    txt = f"{out_prefix}.txt"
    if os.path.isfile(txt):
        df = pd.concat([pd.read_csv(txt), df], ignore_index=True)
    df = df.drop_duplicates(ignore_index=True)
    df.to_csv(txt, index=False)
    df.to_json(f"{out_prefix}.json")
    try:
        df.to_excel(f"{out_prefix}.xlsx", index=False, sheet_name="result")
    except (ImportError, ValueError):
        pass
    return df


def main(argv: list[str] | None = None) -> None:
    argv = sys.argv[1:] if argv is None else argv
    path = (argv[0] if argv else os.getenv("session_path", "")).strip()
    if not path:
        raise SystemExit("usage: graph_exp_analyzer <session_dir>  (or session_path=...)")
    print(write(summarize(path)).tail(1).to_string())


if __name__ == "__main__":
    main()
