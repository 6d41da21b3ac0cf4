"""Concurrent training tasks through the public API — the reference's only pytest,
`simulation_lib/test/test_concurrent.py:11-46`: `fed_avg/mnist.yaml` with one epoch, one round
and three workers; three practitioners on one shared partition; five `train(config,
practitioners)` tasks launched together; every `get_training_result` must come back.

Beyond the reference (which only checks that results arrive), each task's global model must
equal the model of the same run done serially: the tasks share the process (threads), the
device and — on the GPU — the HIP-graph machinery, so any cross-task interference (shared
workspaces, captures overlapping, output files) shows up as a difference."""

import os

import pytest
import torch

from distributed_learning_simulator_amd.config import load_config_from_file
from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
from distributed_learning_simulator_amd.parallel.comm import Comm
from distributed_learning_simulator_amd.practitioner import Practitioner
from distributed_learning_simulator_amd.sampler import get_partition
from distributed_learning_simulator_amd.session import Session
from distributed_learning_simulator_amd.training import get_training_result, train

TASKS = 5


def _config(save_dir, name="fed_avg/mnist.yaml", scale=0.03, workers=3, **extra):
    config = load_config_from_file(name, overrides={"dataset_kwargs": {"scale": scale}, "log_level": "WARNING",
                                                    **extra})
    config.epoch = 1
    config.round = 1
    config.worker_number = workers
    config.save_dir = str(save_dir)
    return config


def _practitioners(config):
    """Reference: one sampler over the dataset collection, shared by every practitioner."""
    labels = create_dataset_collection(config.dataset_name, config.dataset_kwargs, config.seed, "cpu").train.labels
    parts = get_partition(config.dataset_sampling, labels, config.worker_number, seed=config.seed,
                          **config.dataset_sampling_kwargs)
    out = set()
    for pid in range(config.worker_number):
        p = Practitioner(pid)
        p.set_sampler(config.dataset_name, parts[pid])
        out.add(p)
    return out


def _global_model(save_dir):
    path = os.path.join(save_dir, "aggregated_model", "round_1.pk")
    return torch.load(path, map_location="cpu", weights_only=True)


def _check_concurrent(tmp_path, device, tasks=TASKS, serial_options=None, **cfg):
    config = _config(tmp_path / "concurrent", **cfg)
    practitioners = _practitioners(config)
    task_ids = set()
    for _ in range(tasks):
        task_id = train(config=config, practitioners=practitioners)
        assert task_id is not None
        task_ids.add(task_id)
    results = [get_training_result(task_id=t, timeout=600) for t in task_ids]
    assert all(r is not None for r in results)
    assert len({r["save_dir"] for r in results}) == tasks, "tasks must not share an output directory"

    from distributed_learning_simulator_amd import options

    serial_cfg = _config(tmp_path / "serial", **cfg)
    with options.override(**(serial_options or {})):
        serial = Session(serial_cfg, practitioners=_practitioners(serial_cfg), comm=Comm(device=torch.device(device)))
        expected = serial.run()
    ref = _global_model(expected["save_dir"])
    for r in results:
        assert r["performance"] == expected["performance"]
        got = _global_model(r["save_dir"])
        assert got.keys() == ref.keys()
        for k in ref:
            assert torch.equal(got[k], ref[k]), k


def test_concurrent_training(tmp_path, monkeypatch):
    """CPU: five concurrent tasks, each equal to the serial run."""
    from distributed_learning_simulator_amd.parallel import comm as comm_mod

    monkeypatch.setenv("DLS_FORCE_CPU", "1")
    monkeypatch.setattr(comm_mod, "_COMM", None)  # (restored after: a GPU box keeps its own)
    _check_concurrent(tmp_path, "cpu")


@pytest.mark.gpu
def test_concurrent_training_gpu(tmp_path):
    """GPU: the same five tasks sharing one MI355X (native kernels, HIP-graph step replay in
    every task), each bitwise equal to the serial GPU run."""
    assert torch.cuda.is_available()
    from distributed_learning_simulator_amd.ops import backend
    from distributed_learning_simulator_amd.parallel.comm import init_distributed

    assert init_distributed().device.type == "cuda"
    assert backend.using_hip(torch.empty(1, device="cuda"))
    _check_concurrent(tmp_path, "cuda")


@pytest.mark.gpu
def test_concurrent_fused_sgd_gpu(tmp_path):
    """ResNet-18 tasks in concurrent threads, each with the SGD step inside its weight-gradient
    kernels (engine.params.FusedSGD): every launch carries its own epilogue (bindings.cpp sgd_arg),
    so a task can never step another task's weights. Each task's global model must equal, bit for
    bit, a serial run that steps the flat parameters in a separate pass (fused_sgd off)."""
    assert torch.cuda.is_available()
    from distributed_learning_simulator_amd.parallel.comm import init_distributed

    assert init_distributed().device.type == "cuda"
    _check_concurrent(tmp_path, "cuda", tasks=3, serial_options={"fused_sgd": False}, name="fed_avg/cifar10.yaml",
                      scale=0.004, workers=2, model_name="ResNet18")
