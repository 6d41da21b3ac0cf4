"""Per-round test-metric curves across experiments.

Reference `analysis/analyze_round.py:16-70`: for each config file, find the server sessions of
`session/<algo>/<dataset>/`, collect every round's test metrics into one DataFrame per metric
(columns round, value, algorithm), then line-plot mean±sd per algorithm to `<metric>.png`.
Here the per-round metrics come from `server/round_record.json` (one JSON per session) instead
of per-round `performance_metric.json` files; plotting uses matplotlib when it is importable and
the frames are always written as `<metric>.csv`.

    python -m distributed_learning_simulator_amd.analysis.analyze_round conf/fed_avg/mnist.yaml ...
"""

from __future__ import annotations

import os
import sys

import pandas as pd

from .session import Session


def find_sessions(root: str) -> list[str]:
    out = []
    for dirpath, _dirs, files in os.walk(root):
        if "round_record.json" in files and os.path.basename(dirpath) == "server":
            out.append(os.path.dirname(dirpath))
    return sorted(out)


def extract_data(session_root: str, algorithm: str, aggregated: dict[str, pd.DataFrame]) -> dict[str, pd.DataFrame]:
    for path in find_sessions(session_root):
        s = Session(path)
        rows: dict[str, list] = {}
        for r in s.rounds:
            for k, v in s.round_record[r].items():
                rows.setdefault(k, []).append([r, v, algorithm])
        for k, v in rows.items():
            df = pd.DataFrame(v, columns=["round", k, "algorithm"])
            aggregated[k] = df if k not in aggregated else pd.concat([aggregated[k], df], ignore_index=True)
    return aggregated


def plot(aggregated: dict[str, pd.DataFrame], out_dir: str = ".") -> list[str]:
    written = []
    for metric, df in aggregated.items():
        csv = os.path.join(out_dir, f"{metric}.csv")
        df.to_csv(csv, index=False)
        written.append(csv)
        try:
            import matplotlib

            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except ImportError:
            continue
        fig, ax = plt.subplots()
        for algo, g in df.groupby("algorithm"):
            stat = g.groupby("round")[metric].agg(["mean", "std"]).fillna(0.0)
            ax.plot(stat.index, stat["mean"], label=algo)
            ax.fill_between(stat.index, stat["mean"] - stat["std"], stat["mean"] + stat["std"], alpha=0.2)
        ax.set_xlabel("round")
        ax.set_ylabel(metric)
        ax.legend()
        fig.tight_layout()
        png = os.path.join(out_dir, f"{metric}.png")
        fig.savefig(png)
        plt.close(fig)
        written.append(png)
    return written


def main(argv: list[str] | None = None) -> None:
    from ..config import load_config_from_file

    argv = sys.argv[1:] if argv is None else argv
    files = argv or os.getenv("config_files", "").split()
    aggregated: dict[str, pd.DataFrame] = {}
    for cf in files:
        cfg = load_config_from_file(cf)
        root = os.path.join("session", cfg.distributed_algorithm, f"{cfg.dataset_name}_{cfg.dataset_sampling}")
        extract_data(root, cfg.distributed_algorithm, aggregated)
    for p in plot(aggregated):
        print("wrote", p)


if __name__ == "__main__":
    main()
