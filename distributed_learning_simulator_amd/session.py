"""Per-rank simulation runtime ("executor").

Replaces the reference's process/greenlet machinery (`training.py:47-137`,
`executor.py:16-96`, `algorithm_factory.py:12-61`): instead of one process per GPU group
plus a server process, each rank (one process per GPU, torchrun-style env) hosts

* a server replica (deterministic: same selection, same aggregation result everywhere),
* one cohort worker for the clients this rank owns in the round (round-robin over the
  *selected* clients: `selected[rank::world]` — balanced even under partial participation),
* the device-resident dataset, model layout and `CohortTrainer`.

Per round: local clients train in waves → uploads are encoded by the client endpoint and
consumed by the local server replica (on-device, zero copy) → one all-reduce merges all
ranks → finalize → next round's broadcast is already resident. Metrics per round go to
`metrics.jsonl` (rounds/s and comm bytes/round, the BASELINE metric).
"""

from __future__ import annotations

import copy
import dataclasses
import functools
import json
import math
import os
import time

import torch

from .data.datasets import create_dataset_collection, get_spec
from .engine.memory import DEVICE_LOCK, plan_capacity
from .engine.trainer import CohortTrainer, HyperParameter
from .method import CentralizedAlgorithmFactory
from .options import config_options
from .options import scoped as scoped_options
from .models.zoo import build_model, stored_image_channels
from .parallel.comm import Comm, get_comm, init_distributed
from .practitioner import create_practitioners
from .sampler import get_partition
from .utils.logging import get_logger
from .utils.tracing import Watchdog, round_timeout, trace


def resolve_dtype(config, device) -> torch.dtype:
    """Compute dtype of activations and of the parameter views the kernels read.

    `auto` follows the reference's own switch: `use_amp: false` (its default,
    `conf/global.yaml:7`) trains in fp32 — on the GPU the GEMMs then run as split-bf16 MFMA
    with fp32 storage and accumulation (csrc/conv_f32.hip) — and `use_amp: true` selects the
    bf16 fast mode. An explicit `compute_dtype` (bf16 / fp32) overrides both."""
    name = (config.compute_dtype or "auto").lower()
    if name == "auto":
        return torch.bfloat16 if (device.type == "cuda" and config.use_amp) else torch.float32
    return {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32,
            "float32": torch.float32}[name]


def _with_run_options(fn):
    """Run a Session method under the run's `runtime_options:` (options.scoped): they apply while
    the session builds, trains or evaluates, and never leak into another session."""

    @functools.wraps(fn)
    def wrapped(self, *a, **kw):
        with scoped_options(self._run_opts):
            return fn(self, *a, **kw)

    return wrapped


class Session:
    def __init__(self, config, practitioners=None, comm: Comm | None = None):
        self.config = copy.deepcopy(config)
        self._run_opts = config_options(self.config)  # (A/B switches, options.py)
        self._build(practitioners, comm)

    @_with_run_options
    def _build(self, practitioners, comm):
        cfg = self.config
        if not CentralizedAlgorithmFactory.has_algorithm(cfg.distributed_algorithm):
            raise ValueError(f"unknown distributed_algorithm {cfg.distributed_algorithm!r}; registered: "
                             f"{sorted(CentralizedAlgorithmFactory.config)}")
        self.comm = comm or get_comm()
        self.device = self.comm.device
        self.is_main = self.comm.rank == 0
        self.compute_dtype = resolve_dtype(cfg, self.device)
        torch.manual_seed(cfg.seed)
        spec = get_spec(cfg.dataset_name, cfg.dataset_kwargs)
        self.dc = create_dataset_collection(cfg.dataset_name, cfg.dataset_kwargs, cfg.seed, self.device,
                                            self.compute_dtype,
                                            image_channels=stored_image_channels(cfg.model_name, spec))
        if cfg.merge_validation_to_training_set:
            # (before the partition: the clients' shards are drawn from the merged training split)
            self.dc.merge_validation_into_train(cfg.seed)
        if practitioners is None:
            labels = self.dc.train.labels  # (graph: labels of the training nodes)
            practitioners = create_practitioners(cfg, labels)
        else:
            # reference algorithm_factory.py:15-23: worker ids = rank of practitioner id
            practitioners = sorted(practitioners, key=lambda p: p.id)
            for wid, p in enumerate(practitioners):
                p.set_worker_id(wid)
            cfg.worker_number = len(practitioners)
        if cfg.dataset_sampling == "iid" and self.dc.graph is None and not cfg.merge_validation_to_training_set:
            # Validation phase for keep-best-model selection (reference aggregation_worker.py:28-35)
            self.dc.split_validation(cfg.seed)
            vparts = get_partition("iid", self.dc.validation_labels(), len(practitioners), seed=cfg.seed + 1)
            key = self.dc.spec.name + "/validation"
            for p, part in zip(practitioners, vparts):
                if not p.has_dataset(key):
                    p.set_sampler(key, self.dc.validation_indices[part])
        self.practitioners = {p.worker_id: p for p in practitioners}
        self.model = build_model(cfg.model_name, self.dc.spec, cfg.model_kwargs)
        self.layout = self.model.layout
        n_sel = int(cfg.algorithm_kwargs.get("random_client_number", cfg.worker_number) or cfg.worker_number)
        n_sel = min(n_sel, cfg.worker_number)
        per_rank = math.ceil(n_sel / self.comm.world)
        if not cfg.optimizer_name:
            cfg.optimizer_name = "Adam" if self.dc.spec.kind == "graph" else "SGD"
        self.hyper = HyperParameter.from_config(cfg)
        if self.dc.spec.kind == "graph":
            capacity = per_rank  # halo exchange needs every client of the rank resident at once
        else:
            # `limited_resource` (reference aggregation_worker.py:124-130 spills the worker's model
            # cache to disk): here the rank gives client cohorts a quarter of the HBM budget it
            # otherwise would (more, smaller waves); client state never leaves the device
            capacity = plan_capacity(per_rank, self.layout, self.model, self.dc, self.hyper, self.device,
                                     self.compute_dtype, explicit=cfg.cohort_size,
                                     fraction=0.2 if cfg.limited_resource else 0.8)
        self.trainer = CohortTrainer(self.model, self.dc, self.hyper, self.device, self.compute_dtype, capacity)
        self.trainer.debug = bool(cfg.debug)
        algo = cfg.distributed_algorithm
        self.server = CentralizedAlgorithmFactory.create_server(
            algo, {"config": cfg, "session": self}, dict(cfg.endpoint_kwargs.get("server", {})))
        self.worker = CentralizedAlgorithmFactory.create_client(
            algo, {"config": cfg, "session": self}, dict(cfg.endpoint_kwargs.get("worker", {})))
        self.server.endpoint.bind(self.layout, self.device, cfg.seed)
        self.worker.endpoint.bind(self.layout, self.device, cfg.seed)
        if self.server.algorithm is not None:
            self.server.algorithm.bind(cfg, self.layout, self.device, self.comm, self.server)
        self.metrics: list[dict] = []
        self.bytes_up_total = 0
        self.bytes_down_total = 0
        get_logger().info(
            "session: algo=%s model=%s params=%d workers=%d ranks=%d capacity/rank=%d device=%s dtype=%s",
            algo, cfg.model_name, self.layout.num_params, cfg.worker_number, self.comm.world, capacity,
            self.device, self.compute_dtype)

    # ------------------------------------------------------------------ helpers
    def local_clients(self, selected: list[int]) -> list[int]:
        return list(selected[self.comm.rank :: self.comm.world])

    def evaluate_tensors(self, rows: torch.Tensor):
        """Sharded test evaluation of M parameter rows (fp32 or compute dtype); returns device
        tensors (loss [M], acc [M]) without synchronising the host."""
        ls, cs, n = self.trainer.evaluate(rows, batch_size=self.config.eval_batch_size or None,
                                          shard=(self.comm.rank, self.comm.world))
        both = torch.stack([ls, cs])
        self.comm.all_reduce_(both)
        both = both / n
        return both[0], both[1]

    def evaluate(self, rows: torch.Tensor):
        """Sharded test evaluation of M parameter rows; returns (loss [M], acc [M]) lists."""
        loss, acc = self.evaluate_tensors(rows)
        both = torch.stack([loss, acc]).cpu()
        return both[0].tolist(), both[1].tolist()

    def sync(self) -> None:
        if self.device.type == "cuda":
            with DEVICE_LOCK:  # (not inside another task thread's graph capture)
                torch.cuda.synchronize(self.device)

    # ---------------------------------------------------------------------- run
    @_with_run_options
    def run(self) -> dict:
        cfg = self.config
        server, worker = self.server, self.worker
        t_start = time.perf_counter()
        if cfg.resume_from:
            theta_recv = self.load_checkpoint(cfg.resume_from)
        else:
            init = server._before_start()
            theta_recv, down = server.send_result(init)
            if not cfg.distribute_init_parameters:
                down = 0  # no M1 message: clients start from their own init (AggregationWorker)
            self.bytes_down_total += down
            server.last_recorded = None  # the round-0 (init) stat is not a round row
        while not server._stopped():
            theta_recv = self.run_one_round(theta_recv)
            if cfg.checkpoint_every and (server.round_number - 1) % cfg.checkpoint_every == 0:
                self.save_checkpoint(theta_recv)
        self.sync()
        total = time.perf_counter() - t_start
        if hasattr(server, "_write_epoch_stat"):
            server._write_epoch_stat(self)
        server._server_exit()
        worker._after_training()
        get_logger().info("training use %s seconds", total)
        if self.is_main:
            os.makedirs(cfg.save_dir, exist_ok=True)
            # reference dumps config.pkl (`server/server.py:57-60`); JSON here (analysis.session)
            with open(os.path.join(cfg.save_dir, "config.json"), "wt", encoding="utf8") as f:
                json.dump(dataclasses.asdict(cfg), f, default=str, indent=1)
            with open(os.path.join(cfg.save_dir, "metrics.jsonl"), "wt", encoding="utf8") as f:
                for m in self.metrics:
                    f.write(json.dumps(m) + "\n")
        result = {"performance": server.performance_stat, "metrics": self.metrics,
                  "bytes_up": self.bytes_up_total, "bytes_down": self.bytes_down_total, "seconds": total,
                  "save_dir": cfg.save_dir}
        algo = server.algorithm
        if algo is not None and hasattr(algo, "shapley_values"):
            result["sv"] = algo.shapley_values
            result["sv_S"] = getattr(algo, "shapley_values_S", {})
        return result

    # ------------------------------------------------------------- checkpoints
    def save_checkpoint(self, theta_recv: torch.Tensor, path: str | None = None) -> str | None:
        """Resumable state after a finished round: global θ (as held by the server
        and as received by the clients), round counter, per-round records, early-stop state,
        next round's selection, and the method's own state (`state_dict` hooks). Plain tensors /
        numbers only, so `torch.load(weights_only=True)` reads it back."""
        if not self.is_main:
            return None
        server = self.server
        path = path or os.path.join(self.config.save_dir, "checkpoint.pt")
        state = {
            "version": 1,
            "round_number": server.round_number,
            "global_parameter": server.global_parameter.detach().cpu(),
            "theta_recv": theta_recv.detach().cpu(),
            "stat": {int(k) if isinstance(k, int) else str(k): v for k, v in server.performance_stat.items()},
            "server": server.state_dict(),
            "worker": self.worker.state_dict(),
            "bytes_up": self.bytes_up_total,
            "bytes_down": self.bytes_down_total,
            "metrics": [{k: v for k, v in m.items() if isinstance(v, (int, float, str))} for m in self.metrics],
        }
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)
        return path

    def load_checkpoint(self, path: str) -> torch.Tensor:
        state = torch.load(path, map_location="cpu", weights_only=True)
        server = self.server
        server.global_parameter = state["global_parameter"].to(self.device)
        server._stat.update(state["stat"])
        server.load_state_dict(state["server"])
        server._round_number = int(state["round_number"])
        self.worker.load_state_dict(state["worker"])
        self.bytes_up_total = int(state["bytes_up"])
        self.bytes_down_total = int(state["bytes_down"])
        self.metrics = list(state["metrics"])
        get_logger().info("resumed from %s at round %d", path, server.round_number)
        return state["theta_recv"].to(self.device)

    # ------------------------------------------------------------------- round
    def _failed_clients(self, r: int, selected: list[int]) -> list[int]:
        """Deterministic client-failure injection (`algorithm_kwargs.failure_rate`, SURVEY
        §5.3): a failed client neither trains nor uploads; the server sees it as skipped."""
        p = float(self.config.algorithm_kwargs.get("failure_rate", 0.0) or 0.0)
        if p <= 0:
            return []
        g = torch.Generator().manual_seed((self.config.seed + 7) * 1_000_033 + r)
        drop = torch.rand(len(selected), generator=g) < p
        return [c for c, d in zip(selected, drop.tolist()) if d]

    def _mark(self, marks: list, name: str) -> None:
        if self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            marks.append((name, ev))
        else:
            marks.append((name, time.perf_counter()))

    @staticmethod
    def _phase_times(marks: list) -> dict:
        out = {}
        for (_, a), (name, b) in zip(marks, marks[1:]):
            out[name] = (a.elapsed_time(b) / 1e3) if hasattr(a, "elapsed_time") else (b - a)
        return out

    @_with_run_options
    def run_one_round(self, theta_recv: torch.Tensor) -> torch.Tensor:
        """One FL round under the round watchdog (utils/tracing.py), inside a roctx range."""
        with Watchdog(round_timeout(self.config), f"round {self.server.round_number}"), \
                trace(f"round {self.server.round_number}"):
            return self._run_one_round(theta_recv)

    def _run_one_round(self, theta_recv: torch.Tensor) -> torch.Tensor:
        server, worker = self.server, self.worker
        if hasattr(server, "run_round"):  # methods with their own round structure (sign-SGD)
            return server.run_round(self, theta_recv)
        r = server.round_number
        t0 = time.perf_counter()
        marks: list = []
        self._mark(marks, "start")
        selected = list(server.selected)
        failed = self._failed_clients(r, selected)
        active = [c for c in selected if c not in set(failed)]
        local = self.local_clients(active)
        self.round_active = active  # (client -> rank map of the round: fed_gnn halo exchange)
        if server.algorithm is not None:
            server.algorithm.expected_kind = (worker.upload_kind() if hasattr(worker, "upload_kind") else
                                              "delta" if getattr(worker, "_send_parameter_diff", True) else "parameter")
        up0 = worker.endpoint.bytes_sent
        with trace("train"):
            for msg in worker.run_round(r, theta_recv, local):
                server._process_worker_data(msg)
            skipped = sorted(set(range(self.config.worker_number)) - set(active))
            if skipped:
                server._process_worker_data(None, worker_ids=skipped)
        up_local = worker.endpoint.bytes_sent - up0
        self._mark(marks, "train_s")
        with trace("aggregate"):
            result = server._aggregate_worker_data()
        self._mark(marks, "aggregate_s")
        with trace("eval_broadcast"):
            theta_recv, down = server.send_result(result)
        self._mark(marks, "eval_broadcast_s")
        up = self._sum_scalar(up_local)
        if self.config.debug:
            self._debug_check(r, server.global_parameter)
        extra = {"failed_clients": len(failed)} if failed else {}
        self.record_round(r, t0, active, up, down, marks=marks, **extra)
        return theta_recv

    def _debug_check(self, r: int, theta: torch.Tensor) -> None:
        """`debug` mode (reference `debug` flag): synchronise and scan the global
        model for NaN/Inf after every round (the reference asserts on NaN in aggregation)."""
        self.sync()
        if theta is not None and not bool(torch.isfinite(theta).all()):
            bad = (~torch.isfinite(theta)).nonzero().flatten()[:8].tolist()
            raise FloatingPointError(f"round {r}: non-finite global parameters at flat indices {bad}")

    def _sum_scalar(self, v: int) -> int:
        if not self.comm.is_distributed:
            return int(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.device)
        self.comm.all_reduce_(t)
        return int(t.item())

    def record_round(self, r, t0, selected, up, down, marks=None, **extra) -> dict:
        if self.config.extra.get("sync_round_timing", True):
            self.sync()
        wall = time.perf_counter() - t0
        if marks and self.config.extra.get("sync_round_timing", True):
            extra.update(self._phase_times(marks))
        self.bytes_up_total += up
        self.bytes_down_total += down
        rec = getattr(self.server, "last_recorded", None)
        stat = {}
        if rec is not None:
            r, stat = rec
            self.server.last_recorded = None
        row = {"round": r, "wall_s": wall, "rounds_per_s": 1.0 / max(wall, 1e-9), "selected_clients": len(selected),
               "comm_bytes_up": up, "comm_bytes_down": down, "comm_bytes_total": up + down,
               "gpus": self.comm.world, "synthetic": bool(self.dc.synthetic), **stat, **extra}
        self.metrics.append(row)
        get_logger().info("round %s done in %.3fs (up %.1f MiB, down %.1f MiB)", r, wall, up / 2**20, down / 2**20)
        return row
