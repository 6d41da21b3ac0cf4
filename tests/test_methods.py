"""End-to-end protocol tests for every registered method on the CPU oracle path (small
synthetic data), mirroring the reference's smoke scripts (`test.sh`, `other_method_test.sh`)
plus golden checks of the aggregation math and regression tests for fixed reference bugs."""

import json
import os

import pytest
import torch

from distributed_learning_simulator_amd.config import config_from_dict, load_config
from distributed_learning_simulator_amd.message import (DeltaParameterMessage, ParameterMessage,
                                                        get_message_size)
from distributed_learning_simulator_amd.parallel.comm import Comm
from distributed_learning_simulator_amd.session import Session


def _run(cfg_name, overrides, tmp_path):
    group = os.path.dirname(cfg_name).replace("/", ".")
    args = ["--config-name", cfg_name] + [f"++{group}.{k}={v}" for k, v in overrides.items()]
    args.append(f"++{group}.save_dir={tmp_path}")
    cfg = load_config(args)
    sess = Session(cfg, comm=Comm())
    return sess, sess.run()


SMALL = {"round": 2, "epoch": 1, "dataset_kwargs.scale": 0.04, "log_level": "WARNING"}


@pytest.mark.parametrize("cfg_name,extra", [
    ("fed_avg/mnist.yaml", {"worker_number": 3}),
    ("fed_dropout_avg/cifar10.yaml", {"worker_number": 3, "model_name": "LeNet5",
                                      "algorithm_kwargs.random_client_number": 2}),
    ("fed_paq/cifar10.yaml", {"worker_number": 4, "model_name": "LeNet5"}),
    ("fed_obd/cifar10.yaml", {"worker_number": 4, "model_name": "LeNet5", "algorithm_kwargs.random_client_number": 2,
                              "algorithm_kwargs.second_phase_epoch": 2}),
    ("fed_obd_sq/cifar100.yaml", {"worker_number": 4, "model_name": "LeNet5",
                                  "algorithm_kwargs.random_client_number": 4,
                                  "algorithm_kwargs.second_phase_epoch": 1}),
    ("gtg_sv/mnist.yaml", {"worker_number": 3}),
    ("multiround_sv/cifar10.yaml", {"worker_number": 3, "model_name": "LeNet5"}),
    ("hierarchical_sv/mnist.yaml", {"worker_number": 4}),
    ("smafd/cifar10.yaml", {"worker_number": 3, "model_name": "LeNet5", "algorithm_kwargs.random_client_number": 2}),
    ("sign_sgd/cifar10.yaml", {"worker_number": 3, "model_name": "LeNet5", "learning_rate": 0.001}),
    ("fed_gnn/cs.yaml", {"worker_number": 3, "dataset_kwargs.scale": 0.05}),
    ("fed_gnn/amazonproduct.yaml", {"worker_number": 2, "dataset_kwargs.scale": 0.002}),
    ("fed_aas/cora.yaml", {"worker_number": 2, "dataset_kwargs.scale": 0.2}),
    ("fed_avg/imdb.yaml", {"worker_number": 2, "dataset_kwargs.scale": 0.004, "dataset_kwargs.max_len": 32,
                           "model_kwargs.max_len": 32}),
])
def test_method_runs(cfg_name, extra, tmp_path):
    ov = dict(SMALL)
    ov.update(extra)
    sess, result = _run(cfg_name, ov, tmp_path)
    assert result["performance"], "no evaluation recorded"
    for stat in result["performance"].values():
        assert 0.0 <= stat["test_accuracy"] <= 1.0
    assert result["bytes_up"] > 0 and result["bytes_down"] > 0
    assert os.path.exists(os.path.join(tmp_path, "metrics.jsonl"))
    assert os.path.exists(os.path.join(tmp_path, "server", "round_record.json"))


def test_fedavg_golden_weighted_mean(tmp_path):
    """θ_{t+1} = Σ n_k θ_k / Σ n_k (reference FedAVGAlgorithm), unequal shards."""
    cfg = config_from_dict({"distributed_algorithm": "fed_avg", "dataset_name": "MNIST", "model_name": "LeNet5",
                            "worker_number": 3, "round": 1, "epoch": 1, "batch_size": 32,
                            "dataset_sampling": "dirichlet_non_iid", "dataset_sampling_kwargs": {"alpha": 1.0},
                            "dataset_kwargs": {"scale": 0.03}, "save_dir": str(tmp_path), "save_models": False,
                            "log_level": "WARNING"})
    sess = Session(cfg, comm=Comm())
    server, worker = sess.server, sess.worker
    theta0 = server._before_start().parameter
    server.send_result(server._before_start())
    msgs = list(worker.run_round(1, theta0, [0, 1, 2]))
    assert len(msgs) == 1
    msg = msgs[0]
    rows = msg.data + theta0  # restore θ_k from Δ_k
    n = msg.dataset_sizes.double()
    expected = ((rows.double() * n[:, None]).sum(0) / n.sum()).float()
    server._process_worker_data(msg)
    result = server._aggregate_worker_data()
    torch.testing.assert_close(result.parameter, expected, rtol=1e-5, atol=1e-6)


def test_message_size_rule():
    p = {"w": torch.zeros(10, 3), "b": torch.zeros(3, dtype=torch.float64)}
    assert get_message_size(ParameterMessage(parameter=p)) == 10 * 3 * 4 + 3 * 8
    d = DeltaParameterMessage(delta_parameter={"w": torch.ones(10, 3)}, dataset_size=5)
    restored = d.restore({"w": torch.ones(10, 3), "b": torch.zeros(3)})
    assert torch.equal(restored.parameter["w"], torch.full((10, 3), 2.0)) and restored.dataset_size == 5


def test_resnet18_comm_bytes_per_round_matches_reference_rule(tmp_path):
    """8.94 GB/round for 100-client full-participation FedAvg ResNet-18."""
    from distributed_learning_simulator_amd.data.datasets import get_spec
    from distributed_learning_simulator_amd.models.zoo import build_model

    P = build_model("ResNet18", get_spec("CIFAR10")).num_params
    assert 2 * 100 * P * 4 == 8_939_169_600


def test_partial_participation_skip_protocol(tmp_path):
    """B1 regression: unselected clients skip the round; the run completes."""
    sess, result = _run("fed_avg/mnist.yaml", {"round": 3, "epoch": 1, "worker_number": 5,
                                                 "algorithm_kwargs.random_client_number": 2,
                                                 "dataset_kwargs.scale": 0.03, "log_level": "WARNING"}, tmp_path)
    assert [m["selected_clients"] for m in result["metrics"]] == [2, 2, 2]
    assert len(result["performance"]) == 3


def test_early_stop_ends_server(tmp_path):
    """B6 regression: early stop must also stop the server (no hang)."""
    sess, result = _run("fed_avg/mnist.yaml", {"round": 40, "epoch": 1, "worker_number": 2, "learning_rate": 0.0,
                                                 "algorithm_kwargs.early_stop": True, "dataset_kwargs.scale": 0.02,
                                                 "log_level": "WARNING"}, tmp_path)
    assert len(result["metrics"]) < 40  # plateau (lr=0 => no improvement) stops after 5 more rounds


def test_fed_obd_phase_switch_and_end(tmp_path):
    sess, result = _run("fed_obd/cifar10.yaml", {"round": 2, "epoch": 1, "worker_number": 4, "model_name": "LeNet5",
                                                   "algorithm_kwargs.random_client_number": 2,
                                                   "algorithm_kwargs.second_phase_epoch": 3,
                                                   "dataset_kwargs.scale": 0.04, "log_level": "WARNING"}, tmp_path)
    sel = [m["selected_clients"] for m in result["metrics"]]
    assert sel == [2, 2, 4, 4, 4]  # 2 stage-1 rounds, 3 stage-2 per-epoch aggregations
    keys = sorted(result["performance"])
    assert keys == list(range(1, 6))  # stat keys monotone in stage 2
    # stage-1 uploads are block subsets + NNADQ (much smaller than dense fp32)
    P = sess.layout.num_params
    assert result["metrics"][0]["comm_bytes_up"] < 0.5 * 2 * P * 4


def test_shapley_values_written(tmp_path):
    sess, result = _run("gtg_sv/mnist.yaml", {"round": 2, "epoch": 1, "worker_number": 3,
                                                "dataset_kwargs.scale": 0.04, "log_level": "WARNING"}, tmp_path)
    sv = json.load(open(os.path.join(tmp_path, "shapley_values.json")))
    assert set(sv) == {"1", "2"} and all(len(v) == 3 for v in sv.values())
    assert 0 in result["performance"]  # round-0 (init) performance recorded


def test_sign_sgd_bytes(tmp_path):
    sess, result = _run("sign_sgd/cifar10.yaml", {"epoch": 1, "worker_number": 3, "model_name": "LeNet5",
                                                    "dataset_kwargs.scale": 0.04, "log_level": "WARNING"}, tmp_path)
    P = sess.layout.num_params
    steps = (sess.practitioners[0].dataset_size(sess.dc.spec.name) + 63) // 64
    assert result["metrics"][0]["comm_bytes_up"] == 3 * steps * ((P + 7) // 8)


def test_gradient_worker_frees_each_wave_graph(tmp_path, monkeypatch):
    """A synchronous-gradient step trained in several waves must drop a wave's autograd graph
    before the next wave's forward: the convolutions keep activations in the graph's contexts, so
    a live `loss` from the previous wave doubled the footprint (sign-SGD ResNet-50's second
    15-client wave ran out of memory)."""
    import weakref

    from distributed_learning_simulator_amd.engine import trainer as trainer_mod

    orig = trainer_mod.CohortTrainer.forward_loss
    prev: list = []
    waves = [0]

    def forward_loss(self, K, *a, **kw):
        if kw.get("shared"):
            waves[0] += 1
            if prev:
                gc_alive = [r() is not None for r in prev]
                assert not any(gc_alive), "the previous wave's loss graph is still alive"
            prev.clear()
        loss, correct = orig(self, K, *a, **kw)
        if kw.get("shared"):
            prev.extend([weakref.ref(loss), weakref.ref(correct)])
        return loss, correct

    monkeypatch.setattr(trainer_mod.CohortTrainer, "forward_loss", forward_loss)
    _run("sign_sgd/cifar10.yaml", {"epoch": 1, "worker_number": 4, "model_name": "LeNet5", "cohort_size": 2,
                                   "dataset_kwargs.scale": 0.02, "log_level": "WARNING"}, tmp_path)
    assert waves[0] >= 4  # two waves per step


def test_iid_keeps_best_validation_model(tmp_path, monkeypatch):
    """IID sampling ⇒ each client uploads its best-validation-accuracy model of the round
    (reference aggregation_worker.py:28-29,82-86), not the last epoch's."""
    group = "fed_avg"
    args = ["--config-name", "fed_avg/mnist.yaml", f"++{group}.round=1", f"++{group}.epoch=2",
            f"++{group}.worker_number=2", f"++{group}.dataset_kwargs.scale=0.04", f"++{group}.save_dir={tmp_path}",
            f"++{group}.log_level=WARNING"]
    cfg = load_config(args)
    assert cfg.dataset_sampling == "iid"
    sess = Session(cfg, comm=Comm())
    assert sess.dc.validation_indices is not None
    assert sess.worker._choose_model_by_validation
    key = sess.dc.spec.name + "/validation"
    val = [sess.practitioners[c].indices(key) for c in range(2)]
    assert all(v.numel() > 0 for v in val) and not set(val[0].tolist()) & set(val[1].tolist())
    assert not set(sess.dc.validation_indices.tolist()) & set(sess.dc.test_indices.tolist())
    snaps = []
    accs = iter([torch.tensor([0.5, 0.2]), torch.tensor([0.3, 0.4])])  # client 0 best @1, client 1 @2

    def fake_eval(K, shards, dataset=None, batch_size=None):
        snaps.append(sess.trainer.buffers.theta[:K].clone())
        return next(accs)

    monkeypatch.setattr(sess.trainer, "evaluate_clients", fake_eval)
    sent = []
    orig = sess.worker._get_sent_data

    def spy(wave, theta_g, stats):
        msg = orig(wave, theta_g, stats)
        sent.append(msg.data.clone() + theta_g)
        return msg

    monkeypatch.setattr(sess.worker, "_get_sent_data", spy)
    sess.run()
    assert len(snaps) == 2
    torch.testing.assert_close(sent[0][0], snaps[0][0])
    torch.testing.assert_close(sent[0][1], snaps[1][1])


def test_sync_sgd_gradient_worker(tmp_path):
    """GradientWorker substrate (reference gradient_worker.py): dense weighted-mean gradient
    all-reduce every step; wire = P·4 B per client per step each way."""
    sess, result = _run("sign_sgd/cifar10.yaml", {"round": 1, "epoch": 1, "worker_number": 3, "model_name": "LeNet5",
                                                  "distributed_algorithm": "sync_SGD", "learning_rate": 0.01,
                                                  "dataset_kwargs.scale": 0.04, "log_level": "WARNING"}, tmp_path)
    P = sess.layout.num_params
    B = sess.trainer.hyper.batch_size
    steps = max((sess.practitioners[c].dataset_size(sess.dc.spec.name) + B - 1) // B for c in range(3))
    assert result["bytes_up"] == steps * 3 * P * 4
    assert all(torch.isfinite(torch.tensor(v["test_loss"])) for v in result["performance"].values())


def test_topk_error_feedback_worker(tmp_path):
    from distributed_learning_simulator_amd.algorithm.fed_avg_algorithm import FedAVGAlgorithm
    from distributed_learning_simulator_amd.method.algorithm_factory import CentralizedAlgorithmFactory
    from distributed_learning_simulator_amd.server.aggregation_server import AggregationServer
    from distributed_learning_simulator_amd.worker.error_feedback_worker import TopKErrorFeedbackWorker

    if "test_topk_ef" not in CentralizedAlgorithmFactory.config:
        CentralizedAlgorithmFactory.register_algorithm("test_topk_ef", TopKErrorFeedbackWorker, AggregationServer,
                                                       algorithm_cls=FedAVGAlgorithm)
    captured = []
    orig = TopKErrorFeedbackWorker.sparsify

    def spy(self, rows):
        before = rows.clone()
        out, nb = orig(self, rows)
        captured.append((before, out))
        return out, nb

    TopKErrorFeedbackWorker.sparsify = spy
    try:
        sess, result = _run("fed_avg/mnist.yaml", {"round": 2, "epoch": 1, "worker_number": 2,
                                                   "distributed_algorithm": "test_topk_ef",
                                                   "algorithm_kwargs.topk_ratio": 0.05,
                                                   "dataset_kwargs.scale": 0.04, "log_level": "WARNING"}, tmp_path)
    finally:
        TopKErrorFeedbackWorker.sparsify = orig
    P = sess.layout.num_params
    k = int(P * 0.05)
    assert result["bytes_up"] == 2 * 2 * k * 8
    (b1, s1), (b2, s2) = captured
    assert int((s1 != 0).sum(1).max()) <= k
    # residual carried into round 2: what round 1 did not send
    err = sess.worker._error
    torch.testing.assert_close(err, b2 - s2)


def test_checkpoint_resume_reproduces_run(tmp_path):
    """Resumable checkpoints: a run resumed from its round-2 checkpoint ends with
    exactly the global model of the uninterrupted run."""
    base = {"round": 3, "epoch": 1, "worker_number": 3, "dataset_kwargs.scale": 0.04, "log_level": "WARNING",
            "checkpoint_every": 1}
    full, res_full = _run("fed_avg/mnist.yaml", base, tmp_path / "full")
    ck = tmp_path / "full" / "checkpoint.pt"
    assert ck.exists()
    # stop after round 2 (the checkpoint written then), resume for round 3
    part, _ = _run("fed_avg/mnist.yaml", {**base, "round": 2}, tmp_path / "part")
    resumed, res = _run("fed_avg/mnist.yaml", {**base, "resume_from": str(tmp_path / "part" / "checkpoint.pt")},
                        tmp_path / "resumed")
    torch.testing.assert_close(resumed.server.global_parameter, full.server.global_parameter, rtol=0, atol=0)
    assert sorted(res["performance"]) == sorted(res_full["performance"])
    assert [m["round"] for m in resumed.metrics] == [1, 2, 3]


def test_failure_injection_and_phase_timers(tmp_path):
    sess, res = _run("fed_avg/mnist.yaml", {"round": 2, "epoch": 1, "worker_number": 6, "dataset_kwargs.scale": 0.04,
                                            "log_level": "WARNING", "algorithm_kwargs.failure_rate": 0.5,
                                            "debug": True}, tmp_path)
    rows = sess.metrics
    assert any(r.get("failed_clients", 0) > 0 for r in rows)
    for r in rows:
        assert r["selected_clients"] + r.get("failed_clients", 0) == 6
        assert r["comm_bytes_up"] == r["selected_clients"] * sess.layout.num_params * 4
        assert {"train_s", "aggregate_s", "eval_broadcast_s"} <= set(r)


def test_checkpoint_resume_gtg_keeps_shapley_values(tmp_path):
    """ShapleyValueAlgorithm state (per-round SV dicts) survives checkpoint/resume."""
    base = {"round": 3, "epoch": 1, "worker_number": 3, "dataset_kwargs.scale": 0.04, "log_level": "WARNING",
            "checkpoint_every": 1}
    full, res_full = _run("gtg_sv/mnist.yaml", base, tmp_path / "full")
    part, _ = _run("gtg_sv/mnist.yaml", {**base, "round": 2}, tmp_path / "part")
    resumed, res = _run("gtg_sv/mnist.yaml", {**base, "resume_from": str(tmp_path / "part" / "checkpoint.pt")},
                        tmp_path / "resumed")
    assert sorted(res["sv"]) == sorted(res_full["sv"]) == [1, 2, 3]
    for r in res_full["sv"]:
        for w, v in res_full["sv"][r].items():
            assert abs(res["sv"][r][w] - v) < 1e-9
    import json

    sv_json = json.load(open(tmp_path / "resumed" / "shapley_values.json"))
    assert sorted(int(k) for k in sv_json) == [1, 2, 3]


def test_no_initial_distribution_own_init(tmp_path):
    """`distribute_init_parameters: false` (reference aggregation_server.py:58): no θ0 message,
    round-1 clients start from their own init and upload full parameters."""
    sess, res = _run("fed_avg/mnist.yaml", {"round": 2, "epoch": 1, "worker_number": 3, "dataset_kwargs.scale": 0.04,
                                            "log_level": "WARNING", "distribute_init_parameters": False}, tmp_path)
    P = sess.layout.num_params * 4
    # M1 costs nothing; rounds 1 and 2 broadcast to the 3 clients
    assert res["bytes_down"] == 2 * 3 * P
    assert torch.isfinite(sess.server.global_parameter).all()
    ref_sess, _ = _run("fed_avg/mnist.yaml", {"round": 2, "epoch": 1, "worker_number": 3,
                                              "dataset_kwargs.scale": 0.04, "log_level": "WARNING"}, tmp_path / "b")
    assert not torch.equal(ref_sess.server.global_parameter, sess.server.global_parameter)


def test_limited_resource_shrinks_cohorts_without_spilling(tmp_path):
    """`limited_resource` gives client cohorts a smaller memory budget (session.plan_capacity
    fraction) and writes no per-round model files (nothing read them back);
    `save_models` still writes them, weights-only."""
    sess, _ = _run("fed_avg/mnist.yaml", {"round": 2, "epoch": 1, "worker_number": 2, "dataset_kwargs.scale": 0.04,
                                          "log_level": "WARNING", "limited_resource": True, "save_models": False},
                   tmp_path / "a")
    assert not (tmp_path / "a" / "aggregated_model").exists()
    sess, _ = _run("fed_avg/mnist.yaml", {"round": 2, "epoch": 1, "worker_number": 2, "dataset_kwargs.scale": 0.04,
                                          "log_level": "WARNING", "save_models": True}, tmp_path / "b")
    saved = sorted(os.listdir(tmp_path / "b" / "aggregated_model"))
    assert saved == ["round_1.pk", "round_2.pk"]
    t = torch.load(tmp_path / "b" / "aggregated_model" / "round_2.pk", weights_only=True)
    assert set(t) == {e.name for e in sess.layout.entries}


def test_dirichlet_split_deterministic_and_leaves_global_rng():
    """Partitioning is a pure function of (labels, parts, seed) and does not reseed torch's
    process-wide generator (VERDICT r1 minor issue)."""
    from distributed_learning_simulator_amd.sampler import dirichlet_split

    labels = torch.randint(0, 10, (2000,), generator=torch.Generator().manual_seed(0))
    torch.manual_seed(1234)
    before = torch.get_rng_state()
    a = dirichlet_split(labels, 7, seed=3, alpha=0.5)
    assert torch.equal(torch.get_rng_state(), before)
    b = dirichlet_split(labels, 7, seed=3, alpha=0.5)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    assert torch.equal(torch.cat(a).sort().values, torch.arange(2000))


def test_per_client_hyper_parameter_artefacts(tmp_path):
    """Reference `worker/worker.py:50-55` + `executor.py:60-67`: each client writes its trainer's
    hyper-parameters into its own `worker_<id>` directory after training."""
    import json
    import os

    from distributed_learning_simulator_amd.config import config_from_dict
    from distributed_learning_simulator_amd.parallel.comm import Comm
    from distributed_learning_simulator_amd.session import Session

    cfg = config_from_dict({"distributed_algorithm": "fed_avg", "dataset_name": "MNIST", "model_name": "LeNet5",
                            "worker_number": 3, "round": 1, "epoch": 1, "dataset_kwargs": {"scale": 0.01},
                            "learning_rate": 0.02, "save_dir": str(tmp_path), "log_level": "WARNING"})
    Session(cfg, comm=Comm()).run()
    for c in range(3):
        with open(os.path.join(tmp_path, f"worker_{c}", "hyper_parameter.json")) as f:
            h = json.load(f)
        assert h["learning_rate"] == 0.02 and h["epoch"] == 1 and h["batch_size"] == cfg.batch_size


@pytest.mark.parametrize("cfg_name,extra", [
    ("fed_avg/mnist.yaml", {"worker_number": 3}),
    ("fed_avg/imdb.yaml", {"worker_number": 2, "dataset_kwargs.scale": 0.004, "dataset_kwargs.max_len": 32,
                           "model_kwargs.max_len": 32}),
])
def test_merge_validation_to_training_set(cfg_name, extra, tmp_path):
    """`merge_validation_to_training_set: true` (reference config.py:27): the Validation half of
    the test split joins the training split before the partition — the clients' shards cover
    n_train + n_test // 2 samples, some of them test-split samples — and no Validation phase is
    left (no keep-best-model selection); the server tests on the other half."""
    sess, res = _run(cfg_name, {**SMALL, **extra, "merge_validation_to_training_set": True}, tmp_path / "m")
    base, _ = _run(cfg_name, {**SMALL, **extra}, tmp_path / "b")
    dc, dcb = sess.dc, base.dc
    n_val = dcb.validation_indices.numel()
    assert dc.validation_indices is None and dcb.validation_indices is not None
    assert dc.train.n == dcb.train.n + n_val
    assert torch.equal(dc.test_indices, dcb.test_indices)
    assert torch.equal(dc.train.labels[dcb.train.n:], dcb.test.labels[dcb.validation_indices])
    shards = torch.cat([p.indices(dc.spec.name) for p in sess.practitioners.values()])
    assert int(shards.max()) >= dcb.train.n  # merged samples are dealt to clients
    assert not sess.worker._choose_model_by_validation
    assert res["performance"]
