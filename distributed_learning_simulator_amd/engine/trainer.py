"""Cohort trainer: K clients of one rank advance local SGD in lock-step.

Replaces the reference's per-client `cyy_torch_toolbox` Trainer that ran clients one at a
time inside a process (`executor.py:17` semaphore ⇒ serial clients; `worker/worker.py:86`
`trainer.train()`). Here every kernel launch covers all K resident clients:

* a whole round's batch schedule (indices [S, K, B], valid counts, lr, first-step flags) is
  built once and uploaded, so the step loop never synchronises with the host;
* epochs are aligned across clients (an epoch is max_k(batches_k) lock-step steps; a client
  with fewer batches idles with `active=0`), which makes per-epoch hooks (FedOBD stage 2
  aggregates after every epoch, `fed_obd/worker.py:43`) well defined for the whole cohort;
* ragged batches are handled by per-client valid counts (BN statistics, CE and weight
  gradients only see real samples);
* the optimiser is one fused launch over the flat [K, P] buffers.

Semantics pinned (external-library behaviour): SGD with torch semantics
(momentum buffer initialised with the first gradient), optimiser state reset at every
round unless `reuse_learning_rate` (reference `util/model.py:6-23`), CosineAnnealingLR with
T_max = local epochs, stepped per epoch.
"""

from __future__ import annotations

import contextlib
import gc
import math
from dataclasses import dataclass

import torch

from ..models.layers import RunCtx
from ..ops import fl
from ..ops import functional as Fn
from ..utils.tracing import trace
from .hooks import ExecutorHookPoint, HookRegistry, StopExecutingException
from ..options import OPTIONS
from .memory import DEVICE_LOCK, GC_LOCK
from .params import BoundParams, CohortBuffers, FusedSGD


@dataclass
class HyperParameter:
    epoch: int = 1
    batch_size: int = 64
    learning_rate: float = 0.01
    learning_rate_scheduler_name: str | None = None
    weight_decay: float = 0.0
    momentum: float = 0.9
    dampening: float = 0.0
    nesterov: bool = False
    optimizer_name: str = "SGD"

    @classmethod
    def from_config(cls, config) -> "HyperParameter":
        return cls(
            epoch=config.epoch, batch_size=config.batch_size, learning_rate=config.learning_rate,
            learning_rate_scheduler_name=config.learning_rate_scheduler_name,
            weight_decay=config.weight_decay,
            momentum=config.momentum if config.optimizer_name.upper() == "SGD" else 0.0,
            dampening=config.dampening, nesterov=config.nesterov, optimizer_name=config.optimizer_name,
        )

    def lr_at_epoch(self, e: int, total: int) -> float:
        name = (self.learning_rate_scheduler_name or "").lower()
        if name == "cosineannealinglr":
            return 0.5 * self.learning_rate * (1 + math.cos(math.pi * e / max(total, 1)))
        if name == "steplr":
            return self.learning_rate * (0.1 ** (e // max(total // 3, 1)))
        return self.learning_rate


@dataclass
class RoundSchedule:
    idx: torch.Tensor  # [S, K, B] int32 (padded with a valid index)
    counts: torch.Tensor  # [S, K] int32
    active: torch.Tensor  # [S, K] bool
    first: torch.Tensor  # [S, K] bool
    lr: torch.Tensor  # [S, K] fp32
    epoch_end: list[int]  # step index after which epoch e ends
    steps: int
    K: int
    # [S, K, B + 4] int32: idx | count | active | first | lr (fp32 bits) — one row per step, the
    # single copy a graph-replayed step needs (see CohortTrainer._train_graphed)
    packed: torch.Tensor | None = None
    client_ids: torch.Tensor | None = None  # [K] int64 (device): dropout masks follow the client
    seed: int = 0
    # per step: n such that exactly rows [0, n) are active (host ints), or K when the active rows
    # are not a prefix — a ragged step (an epoch's last steps, where only the clients with the
    # largest shards still have a batch) then runs those n rows only (OPTIONS.ragged_steps)
    active_rows: list[int] | None = None


class _StepGraph:
    """One captured lock-step training step of a K-client cohort: every sub-cohort stream,
    forward + backward + optimizer, replayed as a single HIP graph launch. Inputs come from a
    static slot (one D2D copy per step); per-client loss/accuracy sums accumulate in static
    buffers that the host drains at epoch ends."""

    def __init__(self, K: int, B: int, device):
        self.slot = torch.zeros((K, B + 4), dtype=torch.int32, device=device)
        self.loss = torch.zeros(K, dtype=torch.float32, device=device)
        self.correct = torch.zeros_like(self.loss)
        self.samples = torch.zeros_like(self.loss)
        self.graph = None
        self.eager_steps = 0
        self.full = True  # (the full cohort's step: never evicted for a ragged one)
        self.key = None  # (its CohortTrainer._graphs key)


def _nullctx():
    return contextlib.nullcontext()


class TrainStats:
    def __init__(self, epochs: int, K: int, device):
        self.loss_sum = torch.zeros((epochs, K), dtype=torch.float32, device=device)
        self.correct = torch.zeros((epochs, K), dtype=torch.float32, device=device)
        self.samples = torch.zeros((epochs, K), dtype=torch.float32, device=device)

    def epoch_metrics(self, e: int):
        n = self.samples[e].clamp(min=1)
        return self.loss_sum[e] / n, self.correct[e] / n


class CohortTrainer:
    def __init__(self, model, dataset_collection, hyper: HyperParameter, device, compute_dtype,
                 capacity: int):
        self.model = model
        self.dc = dataset_collection
        self.hyper = hyper
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        self.capacity = capacity
        self.layout = model.layout
        self.buffers = CohortBuffers(self.layout, capacity, self.device, compute_dtype, hyper.optimizer_name)
        self.debug = False  # `debug` config: per-step NaN/Inf scan (synchronises every step)
        self.num_streams = int(OPTIONS.streams)  # concurrent sub-cohorts on GPU
        self._stream_pool: list = []
        # HIP-graph replay of whole training steps (OPTIONS.graphs): a ResNet-18 step is
        # ≈400 launches per sub-cohort, which at the 8-GPU per-rank load (13 clients) costs more
        # host time than the GPU needs to run them
        self.use_graphs = bool(OPTIONS.graphs)
        self._graphs: dict = {}
        self.max_graphs = int(OPTIONS.max_graphs)
        # pre-split weight planes (buffers.split) are read by the convolutions only inside a
        # graphed training run: refreshed from θ when it starts and after epoch hooks, kept
        # current by the SGD kernel in between (no other θ writer runs there)
        self._split_live = False
        self._seg_tables: dict = {}  # (fused SGD: complement span tables by stepped-weight set)
        self.hooks = HookRegistry()
        self.adam_step_count = torch.zeros(capacity, dtype=torch.float32, device=self.device)
        self.graph = dataset_collection.graph

    # -------------------------------------------------------------- hook API (X4)
    def append_named_hook(self, point, name, fn):
        self.hooks.append_named_hook(point, name, fn)

    def remove_named_hook(self, name):
        self.hooks.remove_named_hook(name)

    # ----------------------------------------------------------------- state load
    def load_global(self, theta_g: torch.Tensor, K: int) -> None:
        """Every resident client row k < K starts from θ_g (M1/M5 receive + load)."""
        shadow = self.buffers.shadow[:K] if self.buffers.shadow is not None else None
        fl.broadcast_rows(self.buffers.theta[:K], theta_g.to(self.device), shadow)
        if self.hooks.has_hook(ExecutorHookPoint.AFTER_LOAD_MODEL):
            self.hooks.exec(ExecutorHookPoint.AFTER_LOAD_MODEL, theta=self.buffers.theta[:K])

    def load_rows(self, theta_rows: torch.Tensor) -> None:
        K = theta_rows.shape[0]
        self.buffers.theta[:K].copy_(theta_rows)
        if self.buffers.shadow is not None:
            self.buffers.shadow[:K].copy_(theta_rows)
        if self.hooks.has_hook(ExecutorHookPoint.AFTER_LOAD_MODEL):
            self.hooks.exec(ExecutorHookPoint.AFTER_LOAD_MODEL, theta=self.buffers.theta[:K])

    def reset_optimizer(self, K: int) -> None:
        self.buffers.state1[:K].zero_()
        if self.buffers.state2 is not None:
            self.buffers.state2[:K].zero_()
        self.adam_step_count[:K].zero_()

    # ------------------------------------------------------------------ schedule
    def build_schedule(self, shards: list[torch.Tensor], epochs: int, seed: int,
                       epoch_offset: int = 0, total_epochs: int | None = None,
                       lr_override: float | None = None, first_epoch_resets: bool = True,
                       min_steps_per_epoch: int = 1, client_ids: list[int] | None = None) -> RoundSchedule:
        """Per-client shuffles are keyed by (seed, CLIENT id, epoch) so a client sees the same
        batches whichever rank/wave/row hosts it."""
        B = self.hyper.batch_size
        K = len(shards)
        total_epochs = total_epochs or epochs
        per_epoch_steps = [max(min_steps_per_epoch, max((s.numel() + B - 1) // B for s in shards))
                           for _ in range(epochs)]
        S = sum(per_epoch_steps)
        idx = torch.zeros((S, K, B), dtype=torch.int32)
        counts = torch.zeros((S, K), dtype=torch.int32)
        lr = torch.zeros((S, K), dtype=torch.float32)
        first = torch.zeros((S, K), dtype=torch.bool)
        epoch_end = []
        s0 = 0
        for e in range(epochs):
            lr_e = lr_override if lr_override is not None else self.hyper.lr_at_epoch(e + epoch_offset, total_epochs)
            for k, shard in enumerate(shards):
                n = shard.numel()
                if n == 0:
                    continue
                key = client_ids[k] if client_ids is not None else k
                g = torch.Generator().manual_seed((seed * 1_000_003 + key * 7919 + e * 104729) & 0x7FFFFFFF)
                perm = shard[torch.randperm(n, generator=g)]
                nb = (n + B - 1) // B
                padded = torch.cat([perm, perm[:1].expand(nb * B - n)]) if nb * B > n else perm
                idx[s0 : s0 + nb, k] = padded.view(nb, B).to(torch.int32)
                c = torch.full((nb,), B, dtype=torch.int32)
                c[-1] = n - (nb - 1) * B
                counts[s0 : s0 + nb, k] = c
                lr[s0 : s0 + nb, k] = lr_e
            s0 += per_epoch_steps[e]
            epoch_end.append(s0)
        active = counts > 0
        n_act = active.sum(1)
        prefix = active == (torch.arange(K).view(1, K) < n_act.view(S, 1))
        active_rows = [int(n) if bool(ok) else K for n, ok in zip(n_act.tolist(), prefix.all(1).tolist())]
        # torch.optim.SGD initialises the momentum buffer with the first gradient
        seen = torch.zeros(K, dtype=torch.bool)
        for s in range(S):
            if first_epoch_resets:
                first[s] = active[s] & ~seen
            seen |= active[s]
        dev = self.device
        packed = None
        if self._graphs_enabled():
            packed = torch.cat([idx, counts[..., None], active.to(torch.int32)[..., None],
                                first.to(torch.int32)[..., None], lr.view(torch.int32)[..., None]], dim=2).to(dev)
        ids = torch.tensor(client_ids if client_ids is not None else list(range(K)), dtype=torch.int64, device=dev)
        return RoundSchedule(idx.to(dev), counts.to(dev), active.to(dev), first.to(dev), lr.to(dev),
                             epoch_end, S, K, packed, ids, int(seed), active_rows)

    # --------------------------------------------------------------------- train
    def forward_loss(self, K: int, x, labels, valid, shared: bool = False, grad_rows=None, row0: int = 0,
                     client_ids=None, step_seed: int = 0, sgd=None):
        """shared=True: all K clients use parameter row 0 (synchronous-gradient methods such as
        sign-SGD, where every client holds the same model); per-client gradients still land in
        separate rows of `grad_rows` (default grad[row0:row0+K])."""
        b = self.buffers
        grad = grad_rows if grad_rows is not None else b.grad[row0 : row0 + K]
        # weight planes: per-client rows, or the shared row's planes read by all K clients (rep = K)
        split = (b.split[:1] if shared else b.split[row0 : row0 + K]) if self._split_live else None
        params = BoundParams(self.layout, b.compute[:1] if shared else b.compute[row0 : row0 + K], grad, K=K,
                             split=split, sgd=None if shared else sgd)
        ctx = RunCtx(params, valid, training=True, client_ids=client_ids, seed=step_seed)
        logits = self.model.forward(x, ctx)
        loss, correct = Fn.cross_entropy(logits, labels, valid)
        return loss, correct

    @torch.no_grad()
    def evaluate_clients(self, K: int, shards: list[torch.Tensor], dataset=None,
                         batch_size: int | None = None) -> torch.Tensor:
        """Accuracy of each resident client's CURRENT model (row k) on its own index shard of
        `dataset` (default: the test split, where the Validation phase lives) — one batched
        forward per batch position, client = leading dim, ragged shards via valid counts."""
        ds = dataset or self.dc.test
        B = batch_size or self.hyper.batch_size
        sizes = [int(s.numel()) for s in shards]
        nmax = max(sizes) if sizes else 0
        correct = torch.zeros(K, dtype=torch.float32, device=self.device)
        if nmax == 0:
            return correct
        idx = torch.zeros(K, nmax, dtype=torch.long)
        for k, s in enumerate(shards):
            if s.numel():
                idx[k, : s.numel()] = s
                idx[k, s.numel():] = s[0]
        idx = idx.to(self.device)
        size_t = torch.tensor(sizes, dtype=torch.int32, device=self.device)
        params = BoundParams(self.layout, self.buffers.compute[:K], None, K=K)
        for b0 in range(0, nmax, B):
            b1 = min(nmax, b0 + B)
            valid = (size_t - b0).clamp(0, b1 - b0).to(torch.int32)
            x = ds.gather(idx[:, b0:b1])
            y = ds.gather_labels(idx[:, b0:b1])
            ctx = RunCtx(params, valid, training=False)
            _, c = Fn.cross_entropy(self.model.forward(x, ctx), y, valid)
            correct += c
        return correct / size_t.clamp(min=1).float()

    def _gather(self, ds, idx):
        if self.model.input_kind == "graph":
            return self.graph.batch(idx)
        return ds.gather(idx)

    def fused_sgd(self, K: int, lr, active, first, row0: int = 0) -> FusedSGD | None:
        """This step's FusedSGD handle (the wgrad kernels step their weights), or None where the
        flat step must see every gradient: Adam, bf16 compute (shadow rows), no live planes."""
        b = self.buffers
        h = self.hyper
        if not (OPTIONS.fused_sgd and self._split_live and b.shadow is None and b.split is not None
                and h.optimizer_name.lower() != "adam" and self.device.type == "cuda"):
            return None
        r = slice(row0, row0 + K)
        return FusedSGD(b.theta[r], b.state1[r], b.split[r], lr, active, first, h.weight_decay, h.momentum,
                        h.dampening, h.nesterov)

    def _seg_table(self, done: frozenset) -> torch.Tensor:
        """[n, 2] int64 (first float4, count ≤ 2048) spans of the row outside the `done` weights."""
        t = self._seg_tables.get(done)
        if t is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("fused SGD: span table first built inside a graph capture")
            index = self.layout.index()
            cut = sorted((index[n].offset // 4, (index[n].offset + index[n].numel) // 4) for n in done)
            spans, pos = [], 0
            for a, e in cut + [(self.layout.padded_size // 4, self.layout.padded_size // 4)]:
                if a > pos:
                    spans.append((pos, a))
                pos = max(pos, e)
            rows = [(i, min(2048, e - i)) for a, e in spans for i in range(a, e, 2048)]
            t = torch.tensor(rows if rows else [(0, 0)], dtype=torch.int64).to(self.device)
            self._seg_tables[done] = t
        return t

    def optimizer_step(self, K: int, lr, active, first, row0: int = 0, fused: FusedSGD | None = None) -> None:
        b = self.buffers
        h = self.hyper
        r = slice(row0, row0 + K)
        shadow = b.shadow[r] if b.shadow is not None else None
        if fused is not None and fused.done:
            fl.sgd_step_seg(b.theta[r], b.grad[r], b.state1[r], fused.lr, fused.active, fused.first, h.weight_decay,
                            h.momentum, h.dampening, h.nesterov, b.split[r], self._seg_table(frozenset(fused.done)))
            return
        if h.optimizer_name.lower() == "adam":
            self.adam_step_count[r] += active.float()
            fl.adam_step(b.theta[r], b.grad[r], b.state1[r], b.state2[r], lr, active,
                         self.adam_step_count[r], weight_decay=h.weight_decay, shadow=shadow)
        else:
            fl.sgd_step(b.theta[r], b.grad[r], b.state1[r], lr, active, first, h.weight_decay,
                        h.momentum, h.dampening, h.nesterov, shadow,
                        b.split[r] if self._split_live else None)

    # ------------------------------------------------------------------ streams
    def _sub_cohorts(self, K: int) -> list[tuple[int, int]]:
        """Row ranges trained concurrently on separate HIP streams. Sub-cohorts (2 by default)
        overlap each other's kernel tails and small launches (BN coefficients, reductions).
        Measured at fp32 (scripts/ab_streams.sh): rank 0's 13-client share of an 8-rank round
        1 stream 821 ms, 2 streams 743 ms, 3 streams 790 ms; the 100-client round 2 streams
        5.23 s, 3 streams 5.28 s."""
        n = self.num_streams if self.device.type == "cuda" else 1
        n = max(1, min(n, K // 4))
        if n == 1:
            return [(0, K)]
        bounds = [K * i // n for i in range(n + 1)]
        return [(bounds[i], bounds[i + 1]) for i in range(n)]

    def _streams(self, n: int) -> list:
        while len(self._stream_pool) < n:
            self._stream_pool.append(torch.cuda.Stream(device=self.device))
        return self._stream_pool[:n]

    def _graphs_enabled(self) -> bool:
        """Graph replay covers the image models' plain training step (no per-step hooks, no
        debug scans); text/graph models keep the eager path."""
        return (self.use_graphs and self.device.type == "cuda" and self.model.input_kind == "image"
                and not self.debug)

    def train(self, schedule: RoundSchedule, executor=None, stats: TrainStats | None = None,
              epoch_base: int = 0) -> TrainStats:
        K = schedule.K
        ds = self.dc.train
        stats = stats or TrainStats(len(schedule.epoch_end), K, self.device)
        e = 0
        parts = self._sub_cohorts(K)
        if self.hooks.has_hook(ExecutorHookPoint.OPTIMIZER_STEP) or self.model.input_kind == "graph":
            parts = [(0, K)]  # step hooks see the whole cohort; graph halos couple the clients
        elif (schedule.packed is not None and self._graphs_enabled()
              and not self.hooks.has_hook(ExecutorHookPoint.AFTER_BATCH)):
            return self._train_graphed(schedule, parts, executor, stats, epoch_base)
        multi = len(parts) > 1
        streams = self._streams(len(parts)) if multi else [None]
        main = torch.cuda.current_stream(self.device) if multi else None

        def fork():
            for st in streams:
                st.wait_stream(main)

        def join():
            for st in streams:
                main.wait_stream(st)

        self.hooks.exec(ExecutorHookPoint.BEFORE_EXECUTE, executor=executor)
        # pre-split weight planes in eager runs too (Transformer / text models), when nothing but
        # this loop's optimizer steps writes θ between two forwards
        split = self.buffers.split
        if (split is not None and not self.hooks.has_hook(ExecutorHookPoint.OPTIMIZER_STEP)
                and not self.hooks.has_hook(ExecutorHookPoint.AFTER_BATCH) and self.model.input_kind != "graph"):
            fl.split_rows(self.buffers.theta[:K], split[:K])
            self._split_live = True
        else:
            split = None
        if multi:
            fork()
        ragged = self._ragged_ok()
        try:
            for s in range(schedule.steps):
                n = self._step_rows(schedule, s) if ragged else K
                sp = parts if n == K else [(a, min(b, n)) for a, b in parts if a < n]
                for (a, b), st in zip(sp, streams):
                    ctx = torch.cuda.stream(st) if multi else _nullctx()
                    with ctx, trace(f"step {s} rows {a}:{b}"):
                        self._train_step(schedule, ds, s, e, a, b, stats, executor)
                if self.hooks.has_hook(ExecutorHookPoint.AFTER_BATCH):
                    if multi:
                        join()
                    self.hooks.exec(ExecutorHookPoint.AFTER_BATCH, executor=executor, step=s)
                    if multi:
                        fork()
                if s + 1 == schedule.epoch_end[e]:
                    if self.hooks.has_hook(ExecutorHookPoint.AFTER_EPOCH):
                        if multi:
                            join()
                        self.hooks.exec(ExecutorHookPoint.AFTER_EPOCH, executor=executor, epoch=epoch_base + e + 1,
                                        stats=stats, local_epoch=e)
                        if split is not None:  # (an epoch hook may rewrite θ rows)
                            fl.split_rows(self.buffers.theta[:K], split[:K])
                        if multi:
                            fork()
                    e += 1
        except StopExecutingException:
            pass
        finally:
            self._split_live = False
        if multi:
            join()
        self.hooks.exec(ExecutorHookPoint.AFTER_EXECUTE, executor=executor, stats=stats)
        return stats

    def _ragged_ok(self) -> bool:
        """Ragged steps may skip their inactive rows: no per-step hook sees the whole cohort."""
        return (bool(OPTIONS.ragged_steps) and not self.hooks.has_hook(ExecutorHookPoint.OPTIMIZER_STEP)
                and not self.hooks.has_hook(ExecutorHookPoint.AFTER_BATCH) and self.model.input_kind != "graph")

    @staticmethod
    def _step_rows(schedule, s: int) -> int:
        return schedule.active_rows[s] if schedule.active_rows is not None else schedule.K

    def _train_step(self, schedule, ds, s, e, a, b, stats, executor) -> None:
        K = b - a
        idx = schedule.idx[s, a:b]
        x = self._gather(ds, idx)
        labels = ds.gather_labels(idx) if self.model.input_kind != "graph" else self.graph.labels_for(idx)
        valid = schedule.counts[s, a:b]
        ids = schedule.client_ids[a:b] if schedule.client_ids is not None else None
        hooked = self.hooks.has_hook(ExecutorHookPoint.OPTIMIZER_STEP)
        fused = None if hooked else self.fused_sgd(K, schedule.lr[s, a:b], schedule.active[s, a:b],
                                                    schedule.first[s, a:b], row0=a)
        loss, correct = self.forward_loss(K, x, labels, valid, row0=a, client_ids=ids,
                                          step_seed=(schedule.seed * 7919 + s * 104_729) & 0x7FFFFFFF, sgd=fused)
        loss.sum().backward()
        if self.debug and not bool(torch.isfinite(loss).all()):  # synchronising NaN scan
            bad = [a + i for i in (~torch.isfinite(loss)).nonzero().flatten().tolist()]
            raise FloatingPointError(f"step {s}: non-finite loss for cohort rows {bad}")
        with torch.no_grad():
            vf = valid.float()
            stats.loss_sum[e, a:b] += loss.detach() * vf
            stats.correct[e, a:b] += correct
            stats.samples[e, a:b] += vf
            if hooked:
                self.hooks.exec(ExecutorHookPoint.OPTIMIZER_STEP, executor=executor, step=s,
                                lr=schedule.lr[s], active=schedule.active[s], first=schedule.first[s],
                                valid=valid, K=K)
            else:
                self.optimizer_step(K, schedule.lr[s, a:b], schedule.active[s, a:b], schedule.first[s, a:b], row0=a,
                                    fused=fused)

    # ------------------------------------------------------------- graph replay
    def _slot_step(self, sg: _StepGraph, ds, a: int, b: int) -> None:
        """One training step of rows [a, b) reading its inputs from the static slot."""
        B = self.hyper.batch_size
        slot = sg.slot[a:b]
        idx = slot[:, :B]
        valid = slot[:, B].contiguous()
        active = slot[:, B + 1].contiguous().bool()
        first = slot[:, B + 2].contiguous().bool()
        lr = slot[:, B + 3].contiguous().view(torch.float32)
        x = self._gather(ds, idx)
        labels = ds.gather_labels(idx)
        fused = self.fused_sgd(b - a, lr, active, first, row0=a)
        loss, correct = self.forward_loss(b - a, x, labels, valid, row0=a, sgd=fused)
        loss.sum().backward()
        with torch.no_grad():
            vf = valid.float()
            sg.loss[a:b] += loss.detach() * vf
            sg.correct[a:b] += correct
            sg.samples[a:b] += vf
            self.optimizer_step(b - a, lr, active, first, row0=a, fused=fused)

    def release_graphs(self) -> None:
        """Destroy this trainer's step graphs now, under the device lock (a finished session's
        graphs left to the cyclic garbage collector could be destroyed from another task thread in
        the middle of that thread's capture, which HIP aborts on)."""
        if not self._graphs:
            return
        with DEVICE_LOCK:
            torch.cuda.synchronize(self.device)
            for sg in self._graphs.values():
                sg.graph = None
            self._graphs.clear()

    def _step_graph(self, n: int, parts, full: bool = True, keep=()) -> _StepGraph | None:
        """The step graph of an n-row cohort split into `parts` (created empty; captured on its
        second use). Each captured graph owns a private pool sized for its step; n varies with
        failures / last waves / uneven rank shares / ragged epoch ends, so at most `max_graphs`
        are kept (a dropped graph's pool returns to the driver before the next capture), least
        recently used first out — except that a ragged step (`full` False) never evicts a
        full-cohort graph nor a graph in `keep` (the ones this round already uses): then it gets
        None, and the caller runs it on a graph of more rows (the extra rows masked)."""
        B = self.hyper.batch_size
        key = (n, B, tuple(parts))
        sg = self._graphs.get(key)
        if sg is not None:  # (most recently used last)
            self._graphs[key] = self._graphs.pop(key)
            return sg
        while len(self._graphs) >= max(self.max_graphs, 1):
            victim = next((k for k, g in self._graphs.items() if all(g is not u for u in keep)
                           and (full or not g.full)), None)
            if victim is None:
                if full:  # (the caller's own round holds every graph: the oldest goes)
                    victim = next(iter(self._graphs))
                else:
                    return None
            old = self._graphs.pop(victim)
            old.graph = None
            del old
            with DEVICE_LOCK:
                torch.cuda.synchronize(self.device)
                torch.cuda.empty_cache()
        sg = self._graphs[key] = _StepGraph(n, B, self.device)
        sg.full, sg.key = full, key
        return sg

    def _run_step_graph(self, sg: _StepGraph, parts, ds) -> None:
        """One step of the rows in `parts` from sg's slot: eager on first use, captured on the
        second — capture records without executing, so it is replayed right away — replayed after."""
        streams = self._streams(len(parts))

        def run_parts():
            cur = torch.cuda.current_stream(self.device)
            for st in streams:
                st.wait_stream(cur)
            for (a, b), st in zip(parts, streams):
                with torch.cuda.stream(st):
                    self._slot_step(sg, ds, a, b)
            for st in streams:
                cur.wait_stream(st)

        if sg.graph is not None:
            sg.graph.replay()
        elif sg.eager_steps < 1:
            run_parts()
            sg.eager_steps += 1
        else:
            # one capture at a time per process, and no device-wide synchronisation of another
            # task thread inside it (engine.memory.DEVICE_LOCK)
            with DEVICE_LOCK, GC_LOCK:
                # the eager step's cached blocks go back to the driver so the graph's private pool
                # can take them (else activation memory is held twice)
                torch.cuda.synchronize(self.device)
                torch.cuda.empty_cache()
                g = torch.cuda.CUDAGraph()
                # no cyclic GC while capturing: a collected cycle holding an older session's graph
                # or tensors would free device memory inside the capture (HIP aborts);
                # torch.cuda.graph collects once on entry
                gc_was_enabled = gc.isenabled()
                gc.disable()
                try:
                    # thread-local capture: RCCL's watchdog thread (and other task threads' launches
                    # on their own streams) keep running while this one captures
                    with torch.cuda.graph(g, capture_error_mode="thread_local"):
                        run_parts()
                finally:
                    if gc_was_enabled:
                        gc.enable()
            sg.graph = g
            g.replay()

    def _train_graphed(self, schedule: RoundSchedule, parts, executor, stats: TrainStats,
                       epoch_base: int) -> TrainStats:
        """Same step sequence as `train`, each step one HIP-graph replay (`_run_step_graph`): the
        full cohort's graph, or — a ragged step, where only rows [0, n) have a batch
        (OPTIONS.ragged_steps) — the graph of those n rows, split over their own sub-cohorts.
        Every later step, in this and later rounds, is one slot copy + one graph launch."""
        K = schedule.K
        ds = self.dc.train
        ragged = self._ragged_ok()
        used: dict[int, _StepGraph] = {}  # rows → graph used this round (epoch-end stats)
        self.hooks.exec(ExecutorHookPoint.BEFORE_EXECUTE, executor=executor)
        split = self.buffers.split
        if split is not None:
            fl.split_rows(self.buffers.theta[:K], split[:K])
            self._split_live = True
        e = 0
        try:
            for s in range(schedule.steps):
                n = self._step_rows(schedule, s) if ragged else K
                if n > 0:
                    sg = used.get(n)
                    if sg is None:
                        sg = self._step_graph(n, parts if n == K else self._sub_cohorts(n), full=n == K,
                                              keep=tuple(used.values()))
                        if sg is None:
                            # (the graph budget holds the full cohort's and this round's ragged
                            # graphs: the smallest of them with >= n rows runs it, rows past n
                            # inactive — their slot rows carry no batch)
                            n = min(m for m in used if m >= n)
                            sg = used[n]
                        else:
                            used[n] = sg
                            sg.loss.zero_()
                            sg.correct.zero_()
                            sg.samples.zero_()
                    self._graphs[sg.key] = self._graphs.pop(sg.key)  # (most recently used last)
                    sg.slot.copy_(schedule.packed[s, :n])
                    self._run_step_graph(sg, parts if n == K else self._sub_cohorts(n), ds)
                if s + 1 == schedule.epoch_end[e]:
                    for m, g in used.items():
                        stats.loss_sum[e, :m] += g.loss
                        stats.correct[e, :m] += g.correct
                        stats.samples[e, :m] += g.samples
                        g.loss.zero_()
                        g.correct.zero_()
                        g.samples.zero_()
                    if self.hooks.has_hook(ExecutorHookPoint.AFTER_EPOCH):
                        self.hooks.exec(ExecutorHookPoint.AFTER_EPOCH, executor=executor, epoch=epoch_base + e + 1,
                                        stats=stats, local_epoch=e)
                        if split is not None:  # (an epoch hook may rewrite θ rows: FedOBD stage 2)
                            fl.split_rows(self.buffers.theta[:K], split[:K])
                    e += 1
        except StopExecutingException:
            pass
        finally:
            self._split_live = False
        self.hooks.exec(ExecutorHookPoint.AFTER_EXECUTE, executor=executor, stats=stats)
        return stats

    # ------------------------------------------------------------------ evaluate
    @torch.no_grad()
    def evaluate(self, theta_rows: torch.Tensor, dataset=None, batch_size: int | None = None,
                 max_images: int | None = None, shard: tuple[int, int] = (0, 1), indices: torch.Tensor | None = None):
        """Evaluate M models (theta_rows [M,P] fp32 or [P]) on `dataset` (default: the Test
        phase — `dc.test_indices` of the test split when a validation half was carved out).
        BN uses batch statistics of each eval batch (reference: running stats disabled).
        The test set is cut into batches; each batch is a virtual client, so one launch
        covers many batches (and many models). `shard=(rank, world)` evaluates only this
        rank's share of the batches. Returns (loss_sum [M], correct [M], n_total)."""
        if theta_rows.dim() == 1:
            theta_rows = theta_rows.unsqueeze(0)
        if dataset is None:
            ds = self.dc.test
            if indices is None:
                indices = self.dc.test_indices
        else:
            ds = dataset
        if self.model.input_kind == "graph":
            return self.graph.evaluate(self, theta_rows, shard)
        M = theta_rows.shape[0]
        B = batch_size or self.hyper.batch_size
        max_images = int(max_images or OPTIONS.eval_max_images)
        n = ds.n if indices is None else int(indices.numel())
        nb = (n + B - 1) // B
        flat = torch.arange(nb * B, device=self.device) % n
        if indices is not None:
            flat = indices.to(self.device)[flat]
        idx = flat.view(nb, B)
        counts = torch.full((nb,), B, dtype=torch.int32, device=self.device)
        counts[-1] = n - (nb - 1) * B
        rank, world = shard
        lo, hi = nb * rank // world, nb * (rank + 1) // world
        compute = theta_rows.to(self.compute_dtype)
        # fp32 on the GPU: the models' (hi, lo) weight planes, so the evaluation's convolutions run
        # the split-plane LDS-DMA GEMMs (the BatchNorms then emit activation planes, as in training);
        # every virtual client (model m, batch b) reads model m's planes (rep = batches per launch)
        split = None
        if (self.buffers.split is not None and self.model.input_kind == "image" and compute.dtype == torch.float32
                and compute.is_cuda):
            compute = compute.contiguous()
            split = torch.empty((M, 2, compute.shape[1]), dtype=torch.bfloat16, device=self.device)
            fl.split_rows(compute, split)
        g = max(1, min(nb, max_images // max(B * M, 1)))
        starts = list(range(lo, hi, g))
        # launches alternate over the sub-cohort streams (their tails and the small BN / CE
        # kernels overlap); each stream sums into its own accumulators, added in stream order
        ns = max(1, min(self.num_streams if self.device.type == "cuda" else 1, len(starts)))
        streams = self._streams(ns) if ns > 1 else [None]
        if ns > 1:
            cur = torch.cuda.current_stream(self.device)
            for st in streams:
                st.wait_stream(cur)
        accs = []
        for si in range(ns):
            with (torch.cuda.stream(streams[si]) if ns > 1 else _nullctx()):
                accs.append((torch.zeros(M, dtype=torch.float32, device=self.device),
                             torch.zeros(M, dtype=torch.float32, device=self.device)))
        for li, b0 in enumerate(starts):
            si = li % ns
            with (torch.cuda.stream(streams[si]) if ns > 1 else _nullctx()):
                b1 = min(hi, b0 + g)
                gi = idx[b0:b1]
                x = ds.gather(gi)
                y = ds.gather_labels(gi)
                c = counts[b0:b1]
                if M > 1:
                    x = _repeat_leading(x, M)
                    y = y.repeat(M, 1)
                    c = c.repeat(M)
                params = BoundParams(self.layout, compute, None, K=M * (b1 - b0), split=split)
                ctx = RunCtx(params, c, training=False)
                logits = self.model.forward(x, ctx)
                loss, correct = Fn.cross_entropy(logits, y, c)
                w = c.float()
                accs[si][0].add_((loss * w).view(M, -1).sum(1))
                accs[si][1].add_(correct.view(M, -1).sum(1))
        if ns > 1:
            for st in streams:
                cur.wait_stream(st)
        loss_tot, corr_tot = accs[0]
        for la, ca in accs[1:]:
            loss_tot = loss_tot + la
            corr_tot = corr_tot + ca
        return loss_tot, corr_tot, n


def _repeat_leading(x, M):
    if isinstance(x, tuple):
        return tuple(_repeat_leading(t, M) for t in x)
    return x.repeat(M, *([1] * (x.dim() - 1)))
