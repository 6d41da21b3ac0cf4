"""Offline accuracy / communication-volume report from run logs.

Reference `analysis/analyze_log.py:14-66` (`compute_acc`: last test accuracy per log, mean±std
over runs; last per-worker train accuracy) and `:69-279` (`compute_data_amount`: message count
and MiB moved, per algorithm, from the model size plus what the logs say about compression /
dropout). Same accounting rules, re-expressed over this framework's log lines:

  server   "round: <r>, test accuracy <acc> loss <l>"                (INFO)
  worker   "worker <id> round <r> train loss <l> accuracy <acc>"    (DEBUG)
  dropout  "worker <id> send_num <n>"                                (DEBUG; fed_dropout_avg, smafd)
  NNADQ    "worker <id> NNABQ compression ratio is <x>"              (DEBUG; fed_obd)
           "broadcast NNABQ compression ratio is <x>"                (INFO)

Run with `DLS_LOG_LEVEL=DEBUG` to keep the per-worker lines. For the exact bytes a run put on
the wire, prefer `metrics.jsonl` (see `analysis.session.Session.comm_bytes_per_round`); this
module reproduces the reference's *analytic* numbers.

    python -m distributed_learning_simulator_amd.analysis.analyze_log --config-name fed_avg/mnist.yaml \
        --logs log/a.log log/b.log
"""

from __future__ import annotations

import argparse
import re
import statistics

_NUM = r"([0-9.eE+-]+)"
_TEST = re.compile(r"round: (\d+), test accuracy " + _NUM)
_WORKER_ACC = re.compile(r"worker (\d+) round \d+ train loss \S+ accuracy " + _NUM)
_SEND_NUM = re.compile(r"send_num " + _NUM + r"\s*$")
_W_RATIO = re.compile(r"worker \d+ NNABQ compression ratio is " + _NUM)
_B_RATIO = re.compile(r"broadcast NNABQ compression ratio is " + _NUM)


def _read(path: str) -> list[str]:
    with open(path, "rt", encoding="utf8") as f:
        return f.readlines()


def _mean_std(values: list[float]) -> dict:
    mean = statistics.fmean(values)
    std = statistics.stdev(values) if len(values) > 1 else 0.0
    return {"mean": round(mean, 2), "std": round(std, 2)}


def compute_acc(paths: list[str], worker_number: int | None = None) -> dict:
    """Final test accuracy (percent) of each run → mean/std; last train accuracy per worker."""
    final = []
    worker_acc: dict[int, list[float]] = {}
    for path in paths:
        lines = _read(path)
        last = None
        for line in reversed(lines):
            m = _TEST.search(line)
            if m:
                last = float(m.group(2)) * 100
                break
        if last is None:
            raise ValueError(f"{path}: no test accuracy line")
        final.append(last)
        seen: set[int] = set()
        for line in reversed(lines):
            m = _WORKER_ACC.search(line)
            if m:
                wid = int(m.group(1))
                if wid in seen or (worker_number is not None and wid >= worker_number):
                    continue
                seen.add(wid)
                worker_acc.setdefault(wid, []).append(float(m.group(2)) * 100)
    return {"test_acc": _mean_std(final), "worker_acc": {k: _mean_std(v) for k, v in sorted(worker_acc.items())}}


def compute_data_amount(config, paths: list[str], num_params: int | None = None, element_size: int = 4) -> dict:
    """Message count and MiB moved over the whole run (reference accounting rules)."""
    if num_params is None:
        from ..data.datasets import get_spec
        from ..models.zoo import build_model

        num_params = build_model(config.model_name, get_spec(config.dataset_name, config.dataset_kwargs),
                                 config.model_kwargs).num_params
    P, W, R = num_params, config.worker_number, config.round
    ak = config.algorithm_kwargs
    sel = min(int(ak.get("random_client_number", W) or W), W)  # as the server samples (Session)
    up_msgs = R * sel
    up_params = up_msgs * P
    down_params = up_params
    init_msgs = W  # initial model distribution
    init_params = W * P
    msg_num = up_msgs + up_msgs + init_msgs
    mib = 1024 * 1024
    algo = config.distributed_algorithm.lower()

    if algo in ("fed_avg", "gtg_shapley_value", "multiround_shapley_value"):
        amount: float | dict = P * element_size * msg_num / mib
    elif algo == "fed_paq":
        # uploads stochastic-quantised to 1 byte/param; downloads and init in fp32
        msg_num = R * sel * 2 + W
        amount = (up_params * 1 + (down_params + init_params) * element_size) / mib
    elif algo == "fed_obd_sq":
        p = float(ak["dropout_rate"])
        stage2 = int(ak["second_phase_epoch"]) * W * 2
        msg_num += stage2
        amount = (up_params * (1 - p) + down_params + stage2 * P + init_params * element_size) / mib
    elif algo in ("fed_obd", "fed_obd_first_stage"):
        p = float(ak["dropout_rate"])
        stage2 = int(ak["second_phase_epoch"]) * W * 2
        msg_num += stage2
        runs = []
        for path in paths:
            remaining = msg_num
            units = 0.0  # message-equivalents of a full fp32 model
            n_broadcast = 0
            stage_one = True
            for line in _read(path):
                m = _B_RATIO.search(line)
                if m:
                    ratio = float(m.group(1))
                    n_broadcast += 1
                    if n_broadcast <= R:
                        units += ratio * sel
                        remaining -= sel
                    elif algo == "fed_obd_first_stage":
                        break
                    else:
                        stage_one = False
                        if remaining > W:
                            units += ratio * W
                            remaining -= W
                    continue
                m = _W_RATIO.search(line)
                if m:
                    ratio = float(m.group(1))
                    units += ratio * (1 - p) if stage_one else ratio
                    remaining -= 1
            units += W  # the uncompressed initial distribution
            runs.append(P * element_size * units / mib)
        amount = _mean_std(runs)
    elif algo in ("fed_dropout_avg", "single_model_afd"):
        runs = []
        for path in paths:
            sent = sum(float(m.group(1)) for line in _read(path) if (m := _SEND_NUM.search(line)))
            if sent <= 0:
                raise ValueError(f"{path}: no send_num lines (run with DLS_LOG_LEVEL=DEBUG)")
            other = (down_params + init_params) if algo == "fed_dropout_avg" else init_params
            runs.append((sent + other) * element_size / mib)
        amount = _mean_std(runs)
    else:
        raise ValueError(f"no data-amount rule for {config.distributed_algorithm}")
    if isinstance(amount, float):
        amount = round(amount, 2)
    return {"msg_num": msg_num, "data_amount": amount}


def main(argv: list[str] | None = None) -> None:
    from ..config import load_config

    ap = argparse.ArgumentParser()
    ap.add_argument("--logs", nargs="+", required=True)
    args, rest = ap.parse_known_args(argv)
    config = load_config(rest)
    print("test acc", compute_acc(args.logs, config.worker_number)["test_acc"])
    res = compute_data_amount(config, args.logs)
    print("msg_num is", res["msg_num"])
    print("data_amount is", res["data_amount"])


if __name__ == "__main__":
    main()
