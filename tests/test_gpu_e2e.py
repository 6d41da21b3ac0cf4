"""End-to-end sessions on the GPU through the native kernels (the HIP path must be the one
that runs: ops fail loudly if `_dls_hip` is missing)."""

import pytest
import torch

from distributed_learning_simulator_amd.config import load_config
from distributed_learning_simulator_amd.engine.memory import probe_activation_bytes
from distributed_learning_simulator_amd.ops import backend
from distributed_learning_simulator_amd.parallel.comm import Comm
from distributed_learning_simulator_amd.session import Session

pytestmark = pytest.mark.gpu


def _session(cfg_name, overrides, tmp_path):
    group = cfg_name.split("/")[0]
    args = ["--config-name", cfg_name] + [f"++{group}.{k}={v}" for k, v in overrides.items()]
    args.append(f"++{group}.save_dir={tmp_path}")
    return Session(load_config(args), comm=Comm(device=torch.device("cuda", 0)))


def test_fedavg_resnet18_on_gpu(hip, tmp_path):
    sess = _session("fed_avg/cifar10.yaml", {"round": 1, "epoch": 1, "worker_number": 4, "model_name": "ResNet18",
                                             "dataset_kwargs.scale": 0.02, "log_level": "WARNING"}, tmp_path)
    assert sess.device.type == "cuda" and backend.using_hip(sess.trainer.buffers.theta)
    assert sess.trainer.capacity == 4  # memory planner: all 4 clients fit in one wave
    res = sess.run()
    perf = res["performance"][1]
    assert 0.0 <= perf["test_accuracy"] <= 1.0 and torch.isfinite(torch.tensor(perf["test_loss"]))
    assert res["bytes_up"] == 4 * sess.layout.num_params * 4


def test_memory_probe_measures_activations(hip, tmp_path):
    sess = _session("fed_avg/cifar10.yaml", {"round": 1, "epoch": 1, "worker_number": 2, "model_name": "ResNet18",
                                             "dataset_kwargs.scale": 0.02, "log_level": "WARNING"}, tmp_path)
    act = probe_activation_bytes(sess.model, sess.dc, sess.hyper, sess.device, sess.compute_dtype)
    print("probe bytes", act, "batch", sess.hyper.batch_size, "x", sess.dc.train.shape, sess.model.name)
    # ResNet-18/CIFAR, batch 64, bf16: tens of MiB of saved activations per client
    assert 8 * 2**20 < act < 2 * 2**30


def test_transformer_imdb_on_gpu(hip, tmp_path):
    sess = _session("fed_avg/imdb.yaml", {"round": 1, "epoch": 1, "worker_number": 2, "dataset_kwargs.scale": 0.004,
                                          "log_level": "WARNING"}, tmp_path)
    res = sess.run()
    assert torch.isfinite(torch.tensor(res["performance"][1]["test_loss"]))


def test_fed_gnn_on_gpu(hip, tmp_path):
    sess = _session("fed_gnn/cs.yaml", {"round": 1, "epoch": 1, "worker_number": 3, "dataset_kwargs.scale": 0.05,
                                        "log_level": "WARNING"}, tmp_path)
    res = sess.run()
    assert torch.isfinite(torch.tensor(res["performance"][1]["test_loss"]))


def test_graph_replayed_steps_match_eager(hip):
    """HIP-graph replay of training steps (CohortTrainer._train_graphed) computes the same
    local training as the eager launches: same kernels, same order, inputs via the slot."""
    from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
    from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
    from distributed_learning_simulator_amd.models.zoo import build_model

    dev = torch.device("cuda", 0)
    dc = create_dataset_collection("CIFAR10", {"n_train": 512, "n_test": 128}, 0, dev, torch.bfloat16,
                                   image_channels=8)
    model = build_model("ResNet18", dc.spec)
    theta0 = model.layout.init_flat(torch.Generator().manual_seed(0)).to(dev)
    shards = [torch.arange(0, 100), torch.arange(100, 260), torch.arange(260, 300), torch.arange(300, 512)]
    out = {}
    for graphs in (False, True):
        tr = CohortTrainer(model, dc, HyperParameter(epoch=2, batch_size=32, learning_rate=0.002), dev,
                           torch.bfloat16, capacity=4)
        tr.use_graphs = graphs
        tr.num_streams = 2
        tr.load_global(theta0, 4)
        tr.reset_optimizer(4)
        sched = tr.build_schedule(shards, 2, seed=0)
        assert (sched.packed is not None) == graphs
        stats = tr.train(sched)
        torch.cuda.synchronize()
        if graphs:
            assert any(sg.graph is not None for sg in tr._graphs.values()), "no step was graph-replayed"
        out[graphs] = (tr.buffers.theta[:4].clone(), stats.loss_sum.clone(), stats.samples.clone())
    th_e, loss_e, n_e = out[False]
    th_g, loss_g, n_g = out[True]
    assert torch.equal(n_e, n_g)
    # (a small lr keeps the two runs on one trajectory: split-K wgrad atomics are not bitwise
    # reproducible, and a diverging run amplifies that noise)
    torch.testing.assert_close(loss_g, loss_e, rtol=1e-2, atol=1e-2)
    diff = (th_g - th_e).abs()
    assert diff.max().item() < 1e-2 and diff.mean().item() < 1e-4, (diff.max().item(), diff.mean().item())


@pytest.mark.parametrize("graphs", [False, True])
def test_multi_stream_cohort_equals_serial(hip, graphs):
    """Race check: sub-cohorts trained concurrently on 3 HIP streams give the
    same result as one stream. A missing stream dependency (an input consumed before its
    producer on another stream finished) would show up as a divergence here. fp32; split-K
    atomics make the two runs differ only by reduction-order noise."""
    from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
    from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
    from distributed_learning_simulator_amd.models.zoo import build_model

    dev = torch.device("cuda", 0)
    dc = create_dataset_collection("CIFAR10", {"n_train": 768, "n_test": 64}, 0, dev, torch.float32,
                                   image_channels=8)
    model = build_model("ResNet18", dc.spec)
    theta0 = model.layout.init_flat(torch.Generator().manual_seed(1)).to(dev)
    K = 12
    shards = [torch.arange(64 * i, 64 * i + 40 + 2 * i) for i in range(K)]
    out = {}
    for streams in (1, 3):
        tr = CohortTrainer(model, dc, HyperParameter(epoch=1, batch_size=16, learning_rate=0.001), dev,
                           torch.float32, capacity=K)
        tr.use_graphs = graphs
        tr.num_streams = streams
        tr.load_global(theta0, K)
        tr.reset_optimizer(K)
        sched = tr.build_schedule(shards, 1, seed=3)
        assert len(tr._sub_cohorts(K)) == streams
        stats = tr.train(sched)
        torch.cuda.synchronize()
        out[streams] = (tr.buffers.theta[:K].clone(), stats.loss_sum.clone())
    (t1, l1), (t3, l3) = out[1], out[3]
    torch.testing.assert_close(l3, l1, rtol=1e-4, atol=1e-4)
    rel = ((t3 - t1).abs().max() / t1.abs().max()).item()
    assert rel < 1e-4, rel
