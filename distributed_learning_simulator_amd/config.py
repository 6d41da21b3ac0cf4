"""Configuration: YAML tree + Hydra-style CLI, without Hydra.

Reference behaviour reproduced (reference `simulation_lib/config.py`):
  * `DistributedTrainingConfig` fields and defaults (`config.py:16-31`);
  * `--config-name <group>/<file>.yaml` loads the file *nested under its directory path*
    and single-key levels are unwrapped until `dataset_name` appears (`config.py:91-95`),
    so overrides are written `++fed_avg.round=1` exactly as in the reference `test.sh:2`;
  * the primary config is merged over `conf/global.yaml` (`config.py:78-88`);
  * `load_config_from_file(path)` for programmatic use (`config.py:98-104`);
  * `save_dir = session/[exp/]<algo>/<dataset>_<sampling>/<model>/<date>/<uuid>` and
    `log/<same>.log` (`config.py:33-52`).

Hydra/OmegaConf are not installed here; PyYAML + a 100-line override parser cover the
surface the reference uses. The trainer-level keys that the reference forwards to the
external `cyy_torch_toolbox.Config` (dataset/model/hyper-parameter keys) are
first-class fields here.
"""

from __future__ import annotations

import copy
import datetime
import os
import sys
import uuid
from dataclasses import dataclass, field, fields
from typing import Any

import yaml

from .utils.logging import get_logger

CONF_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conf")


@dataclass
class DistributedTrainingConfig:
    # --- FL orchestration (reference config.py:16-31) ---
    exp_name: str = ""
    distributed_algorithm: str = ""
    worker_number: int = 0
    parallel_number: int = 0  # 0 => number of ranks (GPUs) at run time
    round: int = 0
    dataset_sampling: str = "iid"
    dataset_sampling_kwargs: dict = field(default_factory=dict)
    distribute_init_parameters: bool = True
    merge_validation_to_training_set: bool = False
    log_file: str = ""
    limited_resource: bool = False
    endpoint_kwargs: dict = field(default_factory=dict)
    algorithm_kwargs: dict = field(default_factory=dict)
    # --- trainer / model / data keys (external Config in the reference) ---
    dataset_name: str = ""
    model_name: str = ""
    optimizer_name: str = ""  # "" => SGD (Adam for graph datasets; parity unpinned)
    learning_rate: float = 0.01
    learning_rate_scheduler_name: str | None = None
    epoch: int = 1
    batch_size: int = 64
    weight_decay: float = 0.0
    momentum: float = 0.9
    dampening: float = 0.0
    nesterov: bool = False
    use_amp: bool = False
    dataset_kwargs: dict = field(default_factory=dict)
    model_kwargs: dict = field(default_factory=dict)
    extra_hyper_parameters: dict = field(default_factory=dict)
    cache_transforms: str | None = None
    log_level: str = "INFO"
    save_performance_metric: bool = False
    use_slow_performance_metrics: bool = False
    debug: bool = False
    # --- MI355X-native knobs ---
    seed: int = 0
    compute_dtype: str = "auto"  # auto => fp32 unless use_amp (then bf16 on GPU)
    backend: str = "auto"  # auto => hip kernels on GPU, torch oracle on CPU
    cohort_size: int = 0  # max clients resident per rank (0 => all of them)
    eval_batch_size: int = 0  # 0 => batch_size (BN uses batch stats, so it matters)
    eval_every: int = 1
    save_dir: str = ""
    save_models: bool = True
    deterministic: bool = False
    checkpoint_every: int = 0  # rounds between resumable checkpoints (0 => off)
    resume_from: str = ""  # checkpoint.pt to resume the run from
    extra: dict = field(default_factory=dict)

    # ------------------------------------------------------------------ processing
    def load_config_and_process(self, conf: dict) -> None:
        conf = dict(conf)
        names = {f.name for f in fields(self)}
        for k, v in conf.items():
            if k in names:
                setattr(self, k, copy.deepcopy(v))
            else:
                self.extra[k] = copy.deepcopy(v)
        self._normalise()
        # ranks spawned by parallel/launch.py share the parent's run id (one save_dir per run)
        run_id = os.environ.get("DLS_RUN_ID")
        date_time = os.environ.get("DLS_RUN_TIME") or f"{datetime.datetime.now():%Y-%m-%d_%H_%M_%S}"
        dataset_name = self.dataset_kwargs.get("name", self.dataset_name)
        sampling = (
            self.dataset_sampling
            if isinstance(self.dataset_sampling, str)
            else "_".join(self.dataset_sampling)
        )
        dir_suffix = os.path.join(
            self.distributed_algorithm,
            f"{dataset_name}_{sampling}",
            self.model_name,
            date_time,
            run_id or str(uuid.uuid4()),
        )
        if self.exp_name:
            dir_suffix = os.path.join(self.exp_name, dir_suffix)
        if not self.save_dir:
            self.save_dir = os.path.join("session", dir_suffix)
        if not self.log_file:
            self.log_file = os.path.join("log", dir_suffix) + ".log"

    def _normalise(self) -> None:
        for key in ("worker_number", "round", "epoch", "batch_size", "seed"):
            setattr(self, key, int(getattr(self, key)))
        for key in ("learning_rate", "weight_decay", "momentum", "dampening"):
            setattr(self, key, float(getattr(self, key)))
        for key in ("endpoint_kwargs", "algorithm_kwargs", "dataset_kwargs", "model_kwargs",
                    "dataset_sampling_kwargs", "extra_hyper_parameters"):
            if getattr(self, key) is None:
                setattr(self, key, {})

    def get_save_dir(self) -> str:
        return self.save_dir

    def apply_global_config(self) -> None:
        from .utils.logging import set_level

        set_level(self.log_level)

    def to_dict(self) -> dict:
        return {f.name: copy.deepcopy(getattr(self, f.name)) for f in fields(self)}

    # practitioners: reference config.py:55-72
    def create_practitioners(self) -> list:
        from .practitioner import create_practitioners

        return create_practitioners(self)


global_config: DistributedTrainingConfig = DistributedTrainingConfig()


# ---------------------------------------------------------------------- YAML helpers
def _read_yaml(path: str) -> dict:
    with open(path, encoding="utf8") as f:
        data = yaml.safe_load(f)
    return data or {}


def merge_dict(base: dict, other: dict) -> dict:
    """Recursive merge (OmegaConf.merge_with semantics for plain dicts)."""
    out = copy.deepcopy(base)
    for k, v in other.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge_dict(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def parse_override(text: str) -> tuple[list[str], Any]:
    """`++a.b.c=value` / `+a.b=value` / `a.b=value` -> (["a","b","c"], value)."""
    text = text.lstrip("+")
    key, sep, value = text.partition("=")
    if not sep:
        raise ValueError(f"override {text!r} has no '='")
    return key.split("."), yaml.safe_load(value) if value != "" else ""


def apply_override(tree: dict, path: list[str], value: Any) -> None:
    node = tree
    for p in path[:-1]:
        if not isinstance(node.get(p), dict):
            node[p] = {}
        node = node[p]
    node[path[-1]] = value


def _unwrap(conf: dict) -> dict:
    # reference config.py:93-94
    while "dataset_name" not in conf and len(conf) == 1:
        inner = next(iter(conf.values()))
        if not isinstance(inner, dict):
            break
        conf = inner
    return conf


def _nest(conf: dict, config_name: str) -> dict:
    group = os.path.dirname(config_name)
    for part in reversed([p for p in group.split("/") if p]):
        conf = {part: conf}
    return conf


def _finish(conf: dict) -> DistributedTrainingConfig:
    global_path = os.path.join(CONF_DIR, "global.yaml")
    merged = merge_dict(_read_yaml(global_path) if os.path.isfile(global_path) else {}, conf)
    global_config.__init__()  # reset to defaults (reference reuses one global object)
    global_config.load_config_and_process(merged)
    return global_config


def load_config(argv: list[str] | None = None, config_dir: str | None = None) -> DistributedTrainingConfig:
    """CLI entry: `--config-name fed_avg/mnist.yaml ++fed_avg.round=1 ...`."""
    argv = list(sys.argv[1:] if argv is None else argv)
    config_dir = config_dir or CONF_DIR
    config_name = None
    overrides: list[str] = []
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("--config-name", "-cn"):
            config_name = argv[i + 1]
            i += 2
            continue
        if a.startswith("--config-name="):
            config_name = a.split("=", 1)[1]
        elif a in ("--config-path", "-cp"):
            config_dir = argv[i + 1]
            i += 2
            continue
        elif a.startswith("--config-path="):
            config_dir = a.split("=", 1)[1]
        elif "=" in a:
            overrides.append(a)
        else:
            get_logger().warning("ignoring argument %s", a)
        i += 1
    if config_name is None:
        raise SystemExit("--config-name <group>/<file>.yaml is required")
    if not config_name.endswith(".yaml"):
        config_name += ".yaml"
    conf = _nest(_read_yaml(os.path.join(config_dir, config_name)), config_name)
    for o in overrides:
        path, value = parse_override(o)
        apply_override(conf, path, value)
    return _finish(_unwrap(conf))


def load_config_from_file(config_file: str | None = None, overrides: dict | None = None) -> DistributedTrainingConfig:
    assert config_file is not None
    if not os.path.isabs(config_file) and not os.path.exists(config_file):
        config_file = os.path.join(CONF_DIR, config_file)
    conf = _unwrap(_read_yaml(config_file))
    if overrides:
        conf = merge_dict(conf, overrides)
    return _finish(conf)


def config_from_dict(conf: dict) -> DistributedTrainingConfig:
    """Build a fresh (non-global) config object from a flat dict (tests / embedding API)."""
    cfg = DistributedTrainingConfig()
    global_path = os.path.join(CONF_DIR, "global.yaml")
    merged = merge_dict(_read_yaml(global_path) if os.path.isfile(global_path) else {}, conf)
    cfg.load_config_and_process(merged)
    return cfg
