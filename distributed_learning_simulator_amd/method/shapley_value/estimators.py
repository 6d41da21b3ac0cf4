"""Per-round client-contribution estimators (the external `cyy_torch_algorithm.shapely_value`
surface the reference uses: ctor `(players, last_round_metric)`, `set_metric_function`,
`compute(round_number)`, attributes `shapley_values`, `shapley_values_S`;
`shapley_value_algorithm.py:36-52`).

All estimators evaluate utilities in BATCHES: `batch_metric_fn(list[frozenset]) -> list[float]`
turns many subset models into one client-batched evaluation (each subset model is a
"virtual client" of the eval cohort). A scalar `set_metric_function(fn)` is
accepted for API parity (then subsets are evaluated one at a time).

* GTGShapleyValue — GTG-Shapley (Liu et al. 2022): guided Monte-Carlo permutations (one
  permutation starting with each player per iteration), between-round truncation
  (|v(N) − v(∅)| < eps ⇒ all zeros) and within-round truncation (|v(N) − v(S)| < eps ⇒
  marginal 0), convergence on the relative change of the running means. The n
  permutations of an iteration advance position by position, so every position is ONE
  batched evaluation of ≤ n subset models with exact truncation semantics.
* MultiRoundShapleyValue — exact per-round Shapley over all 2^n subsets (Song et al. 2019).
* HierarchicalShapleyValue — two-level: exact SV over `part_number` groups, then exact SV
  within each group, group value distributed proportionally (config-only in the reference:
  `conf/hierarchical_sv/mnist.yaml`; semantics are this framework's definition).
v(∅) is the previous round's global metric (`shapley_value_algorithm.py:40-42`).
"""

from __future__ import annotations

import itertools
import math
import random
import time
from typing import Callable, Iterable

from ...utils.logging import get_logger


class _Base:
    def __init__(self, players: Iterable[int], last_round_metric: float = 0.0, **kwargs):
        self.players = sorted(players)
        self.last_round_metric = float(last_round_metric)
        self.shapley_values: dict = {}
        self.shapley_values_S: dict = {}
        self._cache: dict[frozenset, float] = {}
        self._batch_fn: Callable | None = None
        self.kwargs = kwargs
        self.evaluations = 0
        self.evaluations_per_round: dict[int, int] = {}  # round -> utilities evaluated (cache misses)
        self.iterations_last = 0

    def set_metric_function(self, fn: Callable) -> None:
        self._batch_fn = lambda subsets: [fn(s) for s in subsets]

    def set_batch_metric_function(self, fn: Callable) -> None:
        self._batch_fn = fn

    def reset_players(self, players, last_round_metric):
        self.players = sorted(players)
        self.last_round_metric = float(last_round_metric)
        self._cache.clear()

    def values(self, subsets: list[frozenset]) -> list[float]:
        todo = []
        for s in subsets:
            if not s:
                continue
            if s not in self._cache and s not in todo:
                todo.append(s)
        if todo:
            vals = self._batch_fn(todo)
            self.evaluations += len(todo)
            for s, v in zip(todo, vals):
                self._cache[s] = float(v)
        return [self.last_round_metric if not s else self._cache[s] for s in subsets]

    def _finish(self, sv: dict) -> None:
        self.shapley_values = sv
        self.shapley_values_S = {p: v for p, v in sv.items() if v > 0}


def exact_shapley(players: list, value_fn) -> dict:
    """value_fn(list[frozenset]) -> list[float]; evaluates all 2^n subsets in one batch."""
    n = len(players)
    subsets = [frozenset(c) for r in range(n + 1) for c in itertools.combinations(players, r)]
    vals = dict(zip(subsets, value_fn(subsets)))
    fact = [math.factorial(i) for i in range(n + 1)]
    sv = {}
    for p in players:
        others = [q for q in players if q != p]
        tot = 0.0
        for r in range(len(others) + 1):
            w = fact[r] * fact[n - r - 1] / fact[n]
            for c in itertools.combinations(others, r):
                s = frozenset(c)
                tot += w * (vals[s | {p}] - vals[s])
        sv[p] = tot
    return sv


class MultiRoundShapleyValue(_Base):
    def compute(self, round_number: int) -> None:
        if len(self.players) > 14:
            raise ValueError("exact multi-round Shapley is limited to <= 14 players; use GTG")
        self._cache.clear()
        self._finish(exact_shapley(self.players, self.values))


class GTGShapleyValue(_Base):
    def __init__(self, players, last_round_metric=0.0, eps: float = 0.001, round_trunc_threshold: float = 0.001,
                 max_iterations: int = 30, min_iterations: int = 3, converge_threshold: float = 0.05, seed: int = 0,
                 parallel_iterations: int | None = None, **kwargs):
        super().__init__(players, last_round_metric, **kwargs)
        self.eps = eps
        self.round_trunc_threshold = round_trunc_threshold
        self.max_iterations = max_iterations
        self.min_iterations = min_iterations
        self.converge_threshold = converge_threshold
        self.seed = seed
        # iterations whose permutations advance together: one utility batch per position covers
        # them all (≤ parallel_iterations·n subset models). Results equal the one-iteration-at-a-
        # time order exactly (same permutations, convergence checked per iteration afterwards);
        # iterations past the converged one are evaluated but discarded. Default: just enough
        # iterations to fill one utility batch (`eval_batch` subset models), so large player
        # counts (one iteration = n permutations) waste nothing.
        self.parallel_iterations = parallel_iterations
        self.eval_batch = 32
        self.converged_last = None

    def _marginals(self, perms: list[list], v0: float, vN: float) -> list[list[tuple]]:
        """Position-by-position lock-step over `perms` with within-round truncation: one batched
        utility evaluation per position. Returns per permutation [(player, marginal), ...]."""
        n = len(self.players)
        v_prev = [v0] * len(perms)
        out: list[list[tuple]] = [[] for _ in perms]
        for j in range(n):
            live = [abs(vN - v_prev[i]) >= self.eps for i in range(len(perms))]
            self.values([frozenset(perm[: j + 1]) for i, perm in enumerate(perms) if live[i] and j + 1 < n])
            for i, perm in enumerate(perms):
                if live[i]:
                    v = self._cache[frozenset(perm[: j + 1])] if j + 1 < n else vN
                else:
                    v = v_prev[i]  # within-round truncation: marginal 0
                out[i].append((perm[j], v - v_prev[i]))
                v_prev[i] = v
        return out

    def compute(self, round_number: int) -> None:
        self._cache.clear()
        players = self.players
        n = len(players)
        v0 = self.last_round_metric
        e0 = self.evaluations
        vN = self.values([frozenset(players)])[0]
        if abs(vN - v0) < self.round_trunc_threshold:
            get_logger().info("GTG: between-round truncation (|v(N)-v0| = %.5f)", abs(vN - v0))
            self.evaluations_per_round[round_number] = self.evaluations - e0
            self.iterations_last = 0
            self.converged_last = "between_round_truncation"
            self._finish({p: 0.0 for p in players})
            return
        rng = random.Random(self.seed * 1_000_003 + round_number)
        sums = {p: 0.0 for p in players}
        counts = {p: 0 for p in players}
        prev_means: dict | None = None
        means = dict(sums)
        it = 0
        done = False
        par = self.parallel_iterations or max(1, -(-int(self.eval_batch) // max(n, 1)))
        t0 = time.perf_counter()
        while not done and it < self.max_iterations:
            g = min(par, self.max_iterations - it)
            perms = []
            for _ in range(g):
                for first in players:  # guided sampling: each player leads one permutation
                    rest = [p for p in players if p != first]
                    rng.shuffle(rest)
                    perms.append([first] + rest)
            marg = self._marginals(perms, v0, vN)
            for t in range(g):  # iterations in order: convergence exactly as if run one by one
                it += 1
                block = marg[t * n : (t + 1) * n]
                for j in range(n):  # (position, permutation) order of the sequential loop
                    for contrib in block:
                        p, d = contrib[j]
                        sums[p] += d
                        counts[p] += 1
                means = {p: sums[p] / max(counts[p], 1) for p in players}
                change = float("inf")
                if prev_means is not None:
                    denom = sum(abs(v) for v in means.values()) / n + 1e-12
                    change = sum(abs(means[p] - prev_means[p]) for p in players) / n / denom
                get_logger().info("GTG round %s: iteration %d, %d evaluations, change %.4f, %.1fs",
                                  round_number, it, self.evaluations, change, time.perf_counter() - t0)
                if it >= self.min_iterations and change < self.converge_threshold:
                    done = True
                    break
                prev_means = means
        get_logger().info("GTG round %s: %d iterations, %d subset evaluations", round_number, it, self.evaluations)
        self.evaluations_per_round[round_number] = self.evaluations - e0
        self.iterations_last = it
        # True: the mean change fell under converge_threshold; False: stopped at max_iterations
        self.converged_last = done
        self._finish(means)


class HierarchicalShapleyValue(_Base):
    def __init__(self, players, last_round_metric=0.0, part_number: int = 2, **kwargs):
        super().__init__(players, last_round_metric, **kwargs)
        self.part_number = max(1, int(part_number))

    def compute(self, round_number: int) -> None:
        self._cache.clear()
        players = self.players
        parts = [players[i :: self.part_number] for i in range(self.part_number)]
        parts = [p for p in parts if p]
        groups = list(range(len(parts)))

        def group_values(subsets):
            return self.values([frozenset(q for g in s for q in parts[g]) for s in subsets])

        gsv = exact_shapley(groups, group_values)
        sv = {}
        for g, members in enumerate(parts):
            inner = exact_shapley(members, self.values)
            tot = sum(inner.values())
            for m in members:
                sv[m] = gsv[g] * (inner[m] / tot) if abs(tot) > 1e-12 else gsv[g] / len(members)
        self._finish(sv)
