"""Per-submodule parameter-change report between consecutive model loads.

Reference `analysis/module_diff.py:8-44`: a trainer hook that snapshots every parameterised
sub-module before execution and, after each model load, logs `module <name> has diff <‖Δ‖₂>`
for sub-modules whose change exceeds `delta`. Here a model is one flat row θ[P] of the
cohort layout, so a "sub-module" is the set of layout entries sharing a `module` path and
the norms are one segmented reduction over the row (no per-module concat/copy).

Usage with the worker hooks: `ModuleDiff(layout).attach(trainer.hooks)` logs after every
`load_global` (hook point AFTER_LOAD_MODEL), or call `update(theta_row)` directly.
"""

from __future__ import annotations

import torch

from ..engine.params import ParamLayout
from ..utils.logging import get_logger


class ModuleDiff:
    def __init__(self, layout: ParamLayout, delta: float | None = 0.1):
        self.layout = layout
        self.delta = delta
        self.modules: list[str] = []
        seg = []
        for e in layout.entries:
            mod = e.module or e.name.rsplit(".", 1)[0]
            if mod not in self.modules:
                self.modules.append(mod)
            seg.append((e.offset, e.numel, self.modules.index(mod)))
        ids = torch.full((layout.padded_size,), len(self.modules), dtype=torch.long)
        for off, n, m in seg:
            ids[off : off + n] = m
        self._ids = ids
        self._prev: torch.Tensor | None = None

    def norms(self, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
        """‖a−b‖₂ per module (a, b: flat rows of this layout)."""
        d = (a.float() - b.float()).pow(2)
        ids = self._ids.to(d.device)[: d.numel()]
        out = torch.zeros(len(self.modules) + 1, dtype=torch.float64, device=d.device)
        out.index_add_(0, ids, d.double())
        return out[:-1].sqrt()

    def update(self, theta_row: torch.Tensor) -> dict[str, float]:
        """Compare with the previous snapshot; log and return modules whose change > delta."""
        cur = theta_row.detach().reshape(-1).clone()
        changed: dict[str, float] = {}
        if self._prev is not None:
            for name, v in zip(self.modules, self.norms(self._prev, cur).tolist()):
                if self.delta is not None and v <= self.delta:
                    continue
                changed[name] = v
                get_logger().info("module %s has diff %s", name, v)
        self._prev = cur
        return changed

    def attach(self, hooks, point=None, row: int = 0) -> None:
        """Register on a HookRegistry: the hook receives `theta=` (the [K,P] parameter buffer)."""
        from ..engine.hooks import ExecutorHookPoint

        point = point or ExecutorHookPoint.AFTER_LOAD_MODEL
        hooks.append_named_hook(point, "module_diff", lambda theta=None, **_: self.update(theta[row])
                                if theta is not None else None)
