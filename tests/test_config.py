"""Config surface parity: every YAML under conf/ parses, resolves to a
registered algorithm (ghost methods included), and Hydra-style overrides apply."""

import glob
import os

import pytest

from distributed_learning_simulator_amd.config import CONF_DIR, load_config, load_config_from_file, parse_override
from distributed_learning_simulator_amd.method import CentralizedAlgorithmFactory

ALL = sorted(os.path.relpath(p, CONF_DIR) for p in glob.glob(os.path.join(CONF_DIR, "**", "*.yaml"), recursive=True)
             if not p.endswith("global.yaml"))


def test_conf_tree_complete():
    # 53 method configs + global.yaml, same relative paths as the reference tree
    assert len(ALL) >= 53


@pytest.mark.parametrize("rel", ALL)
def test_every_config_loads_and_is_registered(rel):
    cfg = load_config(["--config-name", rel])
    assert cfg.dataset_name and cfg.model_name and cfg.worker_number > 0
    assert CentralizedAlgorithmFactory.has_algorithm(cfg.distributed_algorithm), cfg.distributed_algorithm
    assert cfg.save_dir.startswith("session") and cfg.log_file.startswith("log")


def test_hydra_override_nesting():
    cfg = load_config(["--config-name", "fed_avg/mnist.yaml", "++fed_avg.round=1", "++fed_avg.epoch=1",
                       "++fed_avg.worker_number=2", "++fed_avg.debug=True"])
    assert (cfg.round, cfg.epoch, cfg.worker_number, cfg.debug) == (1, 1, 2, True)
    assert cfg.learning_rate == 0.01 and cfg.batch_size == 64
    cfg = load_config(["--config-name", "large_scale/fed_obd/imdb.yaml", "++large_scale.fed_obd.round=3",
                       "++large_scale.fed_obd.algorithm_kwargs.random_client_number=7"])
    assert cfg.round == 3 and cfg.algorithm_kwargs["random_client_number"] == 7
    assert cfg.algorithm_kwargs["dropout_rate"] == 0.3
    assert cfg.model_kwargs["d_model"] == 100
    assert cfg.endpoint_kwargs["worker"]["weight"] == 0.0001


def test_global_merge_and_file_loader():
    cfg = load_config_from_file(os.path.join(CONF_DIR, "fed_avg", "mnist.yaml"))
    assert cfg.log_level == "INFO" and cfg.use_amp is False and cfg.cache_transforms == "cpu"


def test_parse_override_types():
    assert parse_override("++a.b=1") == (["a", "b"], 1)
    assert parse_override("a=0.5") == (["a"], 0.5)
    assert parse_override("+x.y=True") == (["x", "y"], True)
    assert parse_override("x=hello") == (["x"], "hello")


def test_save_dir_layout():
    cfg = load_config(["--config-name", "gtg_sv/mnist.yaml", "++gtg_sv.exp_name=myexp"])
    parts = cfg.save_dir.split(os.sep)
    assert parts[:5] == ["session", "myexp", "GTG_shapley_value", "MNIST_iid", "LeNet5"]
