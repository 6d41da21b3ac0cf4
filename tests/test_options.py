"""Runtime options (options.py): one object read when the ops run, settable per run from the
config, programmatically or for a block — not import-time module constants."""

import pytest

from distributed_learning_simulator_amd import options
from distributed_learning_simulator_amd.config import config_from_dict
from distributed_learning_simulator_amd.parallel.comm import Comm
from distributed_learning_simulator_amd.session import Session


def test_override_restores():
    before = options.OPTIONS.streams, options.OPTIONS.planes
    with options.override(streams=1, planes=False) as o:
        assert o.streams == 1 and o.planes is False
    assert (options.OPTIONS.streams, options.OPTIONS.planes) == before
    with pytest.raises(KeyError):
        options.update(no_such_switch=1)


def test_session_applies_runtime_options(tmp_path):
    """A run's `runtime_options:` mapping reaches the engine (trainer stream count) while the session
    builds and runs, and does not leak into the process afterwards (options scoped to the
    run)."""
    before = options.OPTIONS.streams, options.OPTIONS.ragged_steps
    cfg = config_from_dict({"distributed_algorithm": "fed_avg", "dataset_name": "MNIST", "model_name": "LeNet5",
                            "worker_number": 2, "round": 1, "epoch": 1, "dataset_kwargs": {"scale": 0.01},
                            "save_dir": str(tmp_path), "log_level": "WARNING",
                            "runtime_options": {"streams": 3, "ragged_steps": False}})
    sess = Session(cfg, comm=Comm())
    assert sess.trainer.num_streams == 3
    assert (options.OPTIONS.streams, options.OPTIONS.ragged_steps) == before
    sess.run()
    assert (options.OPTIONS.streams, options.OPTIONS.ragged_steps) == before


def test_scoped_options_refuse_conflicting_concurrent_runs():
    """Concurrent runs share the process-wide options the kernels read: a second run with different
    runtime_options is refused while the first is in flight; equal ones nest, and the last one out
    restores the previous values."""
    before = options.OPTIONS.streams
    with options.scoped({"streams": 1}):
        assert options.OPTIONS.streams == 1
        with options.scoped({"streams": 1}):
            assert options.OPTIONS.streams == 1
        assert options.OPTIONS.streams == 1
        with pytest.raises(RuntimeError):
            with options.scoped({"streams": 2}):
                pass
    assert options.OPTIONS.streams == before


def test_env_seeds_defaults(monkeypatch):
    monkeypatch.setenv("DLS_STREAMS", "4")
    monkeypatch.setenv("DLS_PLANES", "0")
    o = options.RuntimeOptions()
    assert o.streams == 4 and o.planes is False
