"""Shapley estimators (GTG-Shapley, exact multi-round, hierarchical) against exact values on
small games, and the lock-step batching of GTG iterations against the one-at-a-time order
(SURVEY §4 test plan: "GTG vs exact Shapley on ≤6 players")."""

import math

import pytest
import torch

from distributed_learning_simulator_amd.method.shapley_value.estimators import (
    GTGShapleyValue, HierarchicalShapleyValue, MultiRoundShapleyValue, exact_shapley)
from distributed_learning_simulator_amd.ops import ref

W = {0: 1.0, 1: 2.0, 2: 3.0, 3: 4.0, 4: 5.0}


def _concave(subsets):
    return [math.sqrt(sum(W[p] for p in s)) / 4.0 for s in subsets]


def _additive(subsets):
    return [0.1 + sum(0.05 * W[p] for p in s) for s in subsets]


def _gtg(fn, **kw):
    est = GTGShapleyValue(players=list(W), last_round_metric=fn([frozenset()])[0], **kw)
    calls = []

    def batch(subsets):
        calls.append(len(subsets))
        return fn(subsets)

    est.set_batch_metric_function(batch)
    est.compute(round_number=1)
    return est, calls


@pytest.mark.parametrize("par", [2, 4, 7])
def test_gtg_lockstep_iterations_equal_sequential(par):
    seq, calls_seq = _gtg(_concave, parallel_iterations=1, eps=0.01)
    bat, calls_bat = _gtg(_concave, parallel_iterations=par, eps=0.01)
    assert bat.shapley_values == seq.shapley_values  # bitwise: same permutations, same order
    assert len(calls_bat) < len(calls_seq)  # fewer, larger utility batches
    assert max(calls_bat) > max(calls_seq)


def test_gtg_additive_game_is_exact():
    est, _ = _gtg(_additive, eps=0.0)
    for p, v in est.shapley_values.items():
        assert v == pytest.approx(0.05 * W[p], abs=1e-12)


def test_gtg_converges_to_exact_shapley():
    exact = exact_shapley(list(W), _concave)
    est, _ = _gtg(_concave, eps=0.0, max_iterations=300, converge_threshold=0.0, parallel_iterations=16)
    scale = max(abs(v) for v in exact.values())
    for p in W:
        assert abs(est.shapley_values[p] - exact[p]) < 0.03 * scale
    # efficiency: Σ SV = v(N) − v(∅) holds for every permutation sample
    assert sum(est.shapley_values.values()) == pytest.approx(_concave([frozenset(W)])[0] - _concave([frozenset()])[0])


def test_multiround_is_exact_and_hierarchical_is_efficient():
    mr = MultiRoundShapleyValue(players=list(W), last_round_metric=_concave([frozenset()])[0])
    mr.set_batch_metric_function(_concave)
    mr.compute(round_number=1)
    exact = exact_shapley(list(W), _concave)
    for p in W:
        assert mr.shapley_values[p] == pytest.approx(exact[p])
    hi = HierarchicalShapleyValue(players=list(W), last_round_metric=_concave([frozenset()])[0], part_number=2)
    hi.set_batch_metric_function(_concave)
    hi.compute(round_number=1)
    total = _concave([frozenset(W)])[0] - _concave([frozenset()])[0]
    assert sum(hi.shapley_values.values()) == pytest.approx(total)


def test_between_round_truncation():
    est = GTGShapleyValue(players=[0, 1, 2], last_round_metric=0.5, round_trunc_threshold=0.01)
    est.set_batch_metric_function(lambda subsets: [0.5 + 1e-4 for _ in subsets])
    est.compute(round_number=3)
    assert est.shapley_values == {0: 0.0, 1: 0.0, 2: 0.0} and est.evaluations == 1


def test_mix_rows_oracle():
    x = torch.randn(6, 64)
    w = torch.rand(3, 6)
    out = ref.mix_rows(x, w, torch.float32)
    torch.testing.assert_close(out, (w.double() @ x.double()).float())
    assert ref.mix_rows(x, w, torch.bfloat16).dtype == torch.bfloat16
