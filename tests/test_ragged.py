"""Ragged steps (OPTIONS.ragged_steps): the cohort's rows are ordered by shard size so that in an
epoch's last steps the clients that still have a batch form a row prefix, and those steps run
only that prefix. Every client trains exactly the same batches either way, so the round's result
equals the full-cohort run (up to the fp64 aggregation order)."""

import pytest
import torch

from distributed_learning_simulator_amd import options
from distributed_learning_simulator_amd.config import config_from_dict
from distributed_learning_simulator_amd.engine.trainer import CohortTrainer
from distributed_learning_simulator_amd.parallel.comm import Comm
from distributed_learning_simulator_amd.session import Session

CFG = {"distributed_algorithm": "fed_avg", "dataset_name": "MNIST", "model_name": "LeNet5", "worker_number": 6,
       "round": 1, "epoch": 2, "batch_size": 16, "learning_rate": 0.05, "dataset_kwargs": {"scale": 0.02},
       "dataset_sampling": "random_label_iid", "dataset_sampling_kwargs": {"sampled_class_number": 3},
       "log_level": "WARNING", "save_models": False, "seed": 3}


def _run(tmp, ragged: bool):
    with options.override(ragged_steps=ragged):
        sess = Session(config_from_dict(dict(CFG, save_dir=str(tmp))), comm=Comm())
        calls = []
        orig = CohortTrainer._train_step

        def spy(self, schedule, ds, s, e, a, b, stats, executor):
            calls.append((s, a, b, schedule.K))
            return orig(self, schedule, ds, s, e, a, b, stats, executor)

        CohortTrainer._train_step = spy
        try:
            res = sess.run()
        finally:
            CohortTrainer._train_step = orig
    return sess.server.global_parameter.clone(), res, calls


def test_ragged_steps_equal_full_cohort(tmp_path):
    g_on, r_on, calls_on = _run(tmp_path / "on", True)
    g_off, r_off, calls_off = _run(tmp_path / "off", False)
    assert all(b - a == K for _, a, b, K in calls_off)
    assert any(b - a < K for _, a, b, K in calls_on), "uneven shards must produce ragged steps"
    assert sum(b - a for _, a, b, _ in calls_on) < sum(b - a for _, a, b, _ in calls_off)
    assert torch.allclose(g_on, g_off, rtol=0, atol=1e-6), (g_on - g_off).abs().max()
    assert r_on["bytes_up"] == r_off["bytes_up"]


def test_schedule_active_prefix():
    """active_rows is the active-prefix length of each step, K where the active rows are no prefix."""
    from distributed_learning_simulator_amd.engine.trainer import HyperParameter

    class _M:
        layout = None

    tr = CohortTrainer.__new__(CohortTrainer)
    tr.hyper = HyperParameter(batch_size=4)
    tr.device = torch.device("cpu")
    tr.use_graphs = False
    tr.model = type("M", (), {"input_kind": "image"})()
    tr.debug = False
    sch = tr.build_schedule([torch.arange(10), torch.arange(6), torch.arange(3)], epochs=1, seed=0)
    assert sch.steps == 3 and sch.active_rows == [3, 2, 1]
    sch = tr.build_schedule([torch.arange(3), torch.arange(10)], epochs=1, seed=0)
    assert sch.active_rows == [2, 2, 2]  # (rows 1 active alone: not a prefix)


@pytest.mark.gpu
def test_ragged_step_graphs_bounded_gpu(tmp_path):
    """Graph-replayed ragged steps (the image models' HIP-graph path) with strongly uneven
    Dirichlet shards: more distinct ragged row counts per epoch than the graph budget holds. The
    full cohort's graph is never evicted for a ragged one; once the budget is full, a new ragged
    count runs on this round's smallest graph with more rows (extra rows masked) — so the cache
    never exceeds max_graphs — and the round equals the full-cohort run (ragged_steps off)."""
    assert torch.cuda.is_available()
    from distributed_learning_simulator_amd.parallel.comm import init_distributed

    assert init_distributed().device.type == "cuda"
    cfg = dict(CFG, dataset_sampling="dirichlet_non_iid", dataset_sampling_kwargs={"alpha": 0.3}, worker_number=8,
               round=2, epoch=2, batch_size=8, dataset_kwargs={"scale": 0.03})
    fallbacks = []
    orig = CohortTrainer._step_graph

    def spy(self, n, parts, full=True, keep=()):
        sg = orig(self, n, parts, full=full, keep=keep)
        if sg is None:
            fallbacks.append(n)
        assert len(self._graphs) <= max(self.max_graphs, 1)
        return sg

    out = {}
    for ragged in (True, False):
        CohortTrainer._step_graph = spy
        try:
            with options.override(ragged_steps=ragged, graphs=True, max_graphs=3):
                sess = Session(config_from_dict(dict(cfg, save_dir=str(tmp_path / str(ragged)))),
                               comm=Comm(device=torch.device("cuda")))
                assert sess.trainer._graphs_enabled()
                res = sess.run()
        finally:
            CohortTrainer._step_graph = orig
        out[ragged] = (sess.server.global_parameter.clone(), res)
    assert fallbacks, "the uneven shards must overflow the ragged graph budget"
    (g_on, r_on), (g_off, r_off) = out[True], out[False]
    assert torch.allclose(g_on, g_off, rtol=1e-5, atol=1e-6), (g_on - g_off).abs().max()
    for k in r_off["performance"]:
        assert abs(r_on["performance"][k]["test_loss"] - r_off["performance"][k]["test_loss"]) < 1e-4
