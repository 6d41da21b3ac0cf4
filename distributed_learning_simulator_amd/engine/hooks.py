"""Named hook points of the cohort trainer.

Reference hook points used by the method code: `AFTER_BATCH`, `AFTER_EPOCH`
(kwargs `epoch`, `executor`), `AFTER_EXECUTE`, `OPTIMIZER_STEP` (replaces the step,
`worker/gradient_worker.py:34-36`). API: `append_named_hook(point, name, fn)`,
`remove_named_hook(name)`, `disable_hook(name)`, `has_hook(point)`.
"""

from __future__ import annotations

from enum import Enum, auto
from typing import Callable


class ExecutorHookPoint(Enum):
    BEFORE_EXECUTE = auto()
    BEFORE_EPOCH = auto()
    BEFORE_BATCH = auto()
    AFTER_FORWARD = auto()
    OPTIMIZER_STEP = auto()
    AFTER_BATCH = auto()
    AFTER_EPOCH = auto()
    AFTER_EXECUTE = auto()
    AFTER_LOAD_MODEL = auto()  # kwargs `theta` ([K,P] rows just loaded); analysis.module_diff


class StopExecutingException(Exception):
    """Raised by a hook to end training early (`aggregation_worker.py:101`)."""


class HookRegistry:
    def __init__(self) -> None:
        self._hooks: dict[ExecutorHookPoint, list[tuple[str, Callable]]] = {p: [] for p in ExecutorHookPoint}
        self._disabled: set[str] = set()

    def append_named_hook(self, point: ExecutorHookPoint, name: str, fn: Callable) -> None:
        self._hooks[point].append((name, fn))

    def remove_named_hook(self, name: str) -> None:
        for p in self._hooks:
            self._hooks[p] = [(n, f) for n, f in self._hooks[p] if n != name]

    def disable_hook(self, name: str) -> None:
        self._disabled.add(name)

    def enable_hook(self, name: str) -> None:
        self._disabled.discard(name)

    def has_hook(self, point: ExecutorHookPoint) -> bool:
        return any(n not in self._disabled for n, _ in self._hooks[point])

    def exec(self, point: ExecutorHookPoint, **kwargs):
        result = None
        for name, fn in list(self._hooks[point]):
            if name in self._disabled:
                continue
            r = fn(**kwargs)
            if r is not None:
                result = r
        return result
