"""Model cache / parameter loading (reference util/model_cache.py, util/model.py), executor
base, memory planner arithmetic."""

import torch

from distributed_learning_simulator_amd.data.datasets import create_dataset_collection, get_spec
from distributed_learning_simulator_amd.engine.memory import plan_capacity, state_bytes_per_client
from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
from distributed_learning_simulator_amd.models.zoo import build_model
from distributed_learning_simulator_amd.utils.model_cache import ModelCache, load_parameters


def test_model_cache_roundtrip(tmp_path):
    model = build_model("LeNet5", get_spec("MNIST"))
    layout = model.layout
    g = torch.Generator().manual_seed(0)
    a, b = layout.init_flat(g), layout.init_flat(g)
    cache = ModelCache(layout)
    cache.cache_parameter(layout.unflatten(a), str(tmp_path / "r1.pt"))
    d = cache.get_parameter_diff(b)
    torch.testing.assert_close(d, b - a)
    cache.add_parameter_diff(d, str(tmp_path / "r2.pt"))
    torch.testing.assert_close(cache.parameter, b)
    assert (tmp_path / "r1.pt").exists()  # previous model saved before the update
    path = cache.get_parameter_path()
    c2 = ModelCache(layout)
    c2.load_file(path)
    torch.testing.assert_close(c2.parameter, b)
    assert set(c2.parameter_dict) == {e.name for e in layout.entries}


def test_load_parameters_resets_optimizer():
    spec = get_spec("MNIST", {"scale": 0.01})
    dc = create_dataset_collection("MNIST", {"scale": 0.01}, 0, "cpu")
    model = build_model("LeNet5", spec)
    tr = CohortTrainer(model, dc, HyperParameter(epoch=1, batch_size=8, learning_rate=0.1), torch.device("cpu"),
                       torch.float32, capacity=2)
    theta = model.layout.init_flat(torch.Generator().manual_seed(1))
    tr.buffers.state1.fill_(3.0)
    load_parameters(tr, theta, reuse_learning_rate=True, K=2)
    assert torch.all(tr.buffers.state1 == 3.0)
    torch.testing.assert_close(tr.buffers.theta[1], theta)
    load_parameters(tr, model.layout.unflatten(theta), reuse_learning_rate=False, K=2)
    assert torch.all(tr.buffers.state1 == 0.0)


def test_memory_plan_cpu_and_state_bytes():
    model = build_model("ResNet18", get_spec("CIFAR10"))
    P = model.layout.padded_size
    assert state_bytes_per_client(model.layout, torch.bfloat16, "SGD") == P * (12 + 2)
    assert state_bytes_per_client(model.layout, torch.float32, "Adam") == P * 16
    # CPU: no device budget → every client resident; explicit cohort_size wins
    assert plan_capacity(37, model.layout, model, None, None, torch.device("cpu"), torch.float32) == 37
    assert plan_capacity(37, model.layout, model, None, None, torch.device("cpu"), torch.float32, explicit=8) == 8


def test_local_npz_dataset_and_synthetic_tag(tmp_path):
    """`dataset_kwargs.root`: real arrays from local disk replace the synthetic generator, and
    runs say which one they used."""
    import json

    import numpy as np

    from distributed_learning_simulator_amd.config import config_from_dict
    from distributed_learning_simulator_amd.parallel.comm import Comm
    from distributed_learning_simulator_amd.session import Session

    rng = np.random.default_rng(0)
    d = tmp_path / "data" / "MNIST"
    d.mkdir(parents=True)
    for split, n in (("train", 240), ("test", 80)):
        y = rng.integers(0, 10, n)
        x = (rng.random((n, 28, 28, 1)) * 60 + y[:, None, None, None] * 19).astype(np.uint8)
        np.savez(d / f"{split}.npz", x=x, y=y)
    base = {"distributed_algorithm": "fed_avg", "dataset_name": "MNIST", "model_name": "LeNet5", "worker_number": 2,
            "round": 1, "epoch": 1, "batch_size": 32, "log_level": "WARNING"}
    sess = Session(config_from_dict({**base, "dataset_kwargs": {"root": str(tmp_path / "data")},
                                     "save_dir": str(tmp_path / "real")}), comm=Comm())
    assert sess.dc.train.n == 240 and not sess.dc.synthetic
    assert torch.equal(sess.dc.train.labels.long(), torch.from_numpy(np.load(d / "train.npz")["y"]).long())
    sess.run()
    row = json.loads(open(tmp_path / "real" / "metrics.jsonl").readline())
    assert row["synthetic"] is False
    rec = json.load(open(tmp_path / "real" / "server" / "round_record.json"))
    assert rec["1"]["synthetic"] is False
    syn = Session(config_from_dict({**base, "dataset_kwargs": {"scale": 0.01}, "save_dir": str(tmp_path / "syn")}),
                  comm=Comm())
    syn.run()
    assert json.loads(open(tmp_path / "syn" / "metrics.jsonl").readline())["synthetic"] is True
