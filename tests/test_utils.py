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
