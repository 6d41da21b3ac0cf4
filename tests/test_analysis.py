"""Offline analysis (reference `analysis/`): session readers, log-based accuracy and the
reference's analytic communication-volume rules, per-round curves, GNN experiment table,
per-module diff hook."""

import logging
import os

import pandas as pd
import torch

from distributed_learning_simulator_amd.analysis import ModuleDiff, Session, compute_acc, compute_data_amount
from distributed_learning_simulator_amd.analysis import analyze_round, graph_exp_analyzer
from distributed_learning_simulator_amd.config import load_config
from distributed_learning_simulator_amd.data.datasets import get_spec
from distributed_learning_simulator_amd.models.zoo import build_model
from distributed_learning_simulator_amd.parallel.comm import Comm
from distributed_learning_simulator_amd.session import Session as RunSession
from distributed_learning_simulator_amd.utils.logging import add_file_handler, get_logger, remove_handler


def _run(cfg_name, overrides, tmp_path, log_path=None):
    group = os.path.dirname(cfg_name).replace("/", ".")
    args = ["--config-name", cfg_name] + [f"++{group}.{k}={v}" for k, v in overrides.items()]
    args.append(f"++{group}.save_dir={tmp_path}")
    cfg = load_config(args)
    handler = add_file_handler(str(log_path)) if log_path else None
    old = get_logger().level
    get_logger().setLevel(logging.DEBUG)
    try:
        sess = RunSession(cfg, comm=Comm())
        res = sess.run()
    finally:
        get_logger().setLevel(old)
        if handler:
            remove_handler(handler)
    return cfg, res


def test_session_reader_and_log_accounting(tmp_path):
    log = tmp_path / "run.log"
    cfg, res = _run("fed_avg/mnist.yaml", {"round": 2, "epoch": 1, "worker_number": 3,
                                           "dataset_kwargs.scale": 0.04}, tmp_path / "s", log)
    s = Session(str(tmp_path / "s"))
    assert s.rounds == [1, 2] and s.last_round == 2
    assert abs(s.last_test_acc - res["performance"][2]["test_accuracy"]) < 1e-9
    assert s.config["distributed_algorithm"] == "fed_avg"
    assert len(s.metrics) == 2 and s.rounds_per_s > 0
    # the server's last recorded accuracy, in percent
    acc = compute_acc([str(log)], worker_number=3)
    assert abs(acc["test_acc"]["mean"] - round(100 * s.last_test_acc, 2)) < 0.01
    assert set(acc["worker_acc"]) == {0, 1, 2}
    # analytic FedAvg volume: (R·W up + R·W down + W init) fp32 models
    P = build_model(cfg.model_name, get_spec(cfg.dataset_name, cfg.dataset_kwargs)).num_params
    out = compute_data_amount(cfg, [str(log)])
    assert out["msg_num"] == 2 * 3 * 2 + 3
    assert abs(out["data_amount"] - round(P * 4 * 15 / 2**20, 2)) < 0.01
    # that analytic figure matches the bytes the run measured on the wire (plus the init send)
    measured = res["bytes_up"] + res["bytes_down"]
    assert measured == P * 4 * 15


def test_fed_paq_and_dropout_rules(tmp_path):
    log = tmp_path / "d.log"
    cfg, _ = _run("fed_dropout_avg/cifar10.yaml", {"round": 1, "epoch": 1, "worker_number": 3,
                                                   "model_name": "LeNet5", "dataset_kwargs.scale": 0.04},
                  tmp_path / "s", log)
    P = build_model("LeNet5", get_spec("CIFAR10")).num_params
    out = compute_data_amount(cfg, [str(log)], num_params=P)
    sent = sum(float(line.rsplit(" ", 1)[1]) for line in open(log) if "send_num" in line)
    assert 0 < sent < 3 * P
    assert abs(out["data_amount"]["mean"] - round((sent + 3 * P + 3 * P) * 4 / 2**20, 2)) < 0.01
    cfg.distributed_algorithm = "fed_paq"
    cfg.round, cfg.worker_number = 100, 10
    cfg.algorithm_kwargs = {"random_client_number": 5}
    out = compute_data_amount(cfg, [], num_params=1_059_298)
    # fed_paq/cifar10 → 1,010 messages, 2,566 MiB
    assert out["msg_num"] == 1010
    assert abs(out["data_amount"] - 2566) < 1.0


def test_round_curves_and_graph_table(tmp_path, monkeypatch):
    root = tmp_path / "session" / "fed_gnn"
    _run("fed_gnn/cs.yaml", {"round": 2, "epoch": 1, "worker_number": 2, "dataset_kwargs.scale": 0.05},
         root / "run1")
    agg = analyze_round.extract_data(str(root), "fed_gnn", {})
    assert "test_accuracy" in agg and set(agg["test_accuracy"]["round"]) == {1, 2}
    monkeypatch.chdir(tmp_path)
    written = analyze_round.plot(agg, str(tmp_path))
    assert any(p.endswith("test_accuracy.csv") for p in written)
    res = graph_exp_analyzer.summarize(str(root / "run1"))
    assert res["distributed_algorithm"] == "fed_gnn" and "in_client_training_edge_cnt" in res
    df = graph_exp_analyzer.write(res, str(tmp_path / "exp"))
    assert len(pd.read_csv(tmp_path / "exp.txt")) == len(df) == 1


def test_module_diff():
    model = build_model("LeNet5", get_spec("MNIST"))
    md = ModuleDiff(model.layout, delta=0.0)
    theta = model.layout.init_flat(torch.Generator().manual_seed(0))
    assert md.update(theta) == {}
    e = model.layout.entries[0]
    theta2 = theta.clone()
    theta2[e.offset : e.offset + e.numel] += 1.0
    changed = md.update(theta2)
    assert list(changed) == [md.modules[0]]
    assert abs(changed[md.modules[0]] - e.numel ** 0.5) < 1e-4
