"""roctx ranges and the per-round watchdog (SURVEY §5.1 tracing, §5.3 failure detection).

Tracing. With `DLS_ROCTX=1`, `trace("name")` pushes a roctx range. On ROCm `torch.cuda.nvtx`
is backed by roctx, so the ranges show up in `rocprofv3 --marker-trace --kernel-trace`
(scripts/gpu.sh marker) around the simulator's phases: round, train (per cohort), aggregate,
broadcast + evaluation. Without the variable, `trace` is a no-op context manager (no driver
calls on the hot path).

Watchdog. A round that does not finish within `round_timeout_s` (config `extra.round_timeout_s`
or `DLS_ROUND_TIMEOUT`, seconds; off by default) is treated as hung: a peer died mid-collective,
or a kernel never completed. The watchdog thread then:
- writes every thread's Python stack to stderr (faulthandler), so the log names the hang;
- exits the process with status 75.
The launcher (parallel/launch.py) sees the non-zero status and terminates the other ranks: a
clean job abort instead of waiting out the collective timeout. Collective timeouts themselves
are bounded by `DLS_COLLECTIVE_TIMEOUT` (parallel/comm.py).
"""

from __future__ import annotations

import contextlib
import faulthandler
import os
import sys
import threading
import time

WATCHDOG_EXIT = 75

_ROCTX = os.environ.get("DLS_ROCTX", "0") == "1"


def roctx_enabled() -> bool:
    return _ROCTX


@contextlib.contextmanager
def trace(name: str):
    if not _ROCTX:
        yield
        return
    import torch

    if not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


class Watchdog:
    """`with Watchdog(seconds, what): ...` — dumps stacks and exits if the body overruns."""

    def __init__(self, timeout_s: float | None, what: str = "round", on_fire=None):
        self.timeout_s = float(timeout_s) if timeout_s else 0.0
        self.what = what
        self._timer: threading.Timer | None = None
        self._on_fire = on_fire
        self.t0 = 0.0

    def _fire(self) -> None:
        dt = time.perf_counter() - self.t0
        sys.stderr.write(f"[watchdog] {self.what} exceeded {self.timeout_s:.0f}s (running {dt:.0f}s): "
                         f"assuming a hang (dead peer / stuck collective); stacks follow, exiting "
                         f"{WATCHDOG_EXIT}\n")
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        sys.stderr.flush()
        if self._on_fire is not None:  # tests
            self._on_fire()
            return
        os._exit(WATCHDOG_EXIT)

    def __enter__(self):
        if self.timeout_s > 0:
            self.t0 = time.perf_counter()
            self._timer = threading.Timer(self.timeout_s, self._fire)
            self._timer.daemon = True
            self._timer.start()
        return self

    def __exit__(self, *exc):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        return False


def round_timeout(config) -> float:
    v = os.environ.get("DLS_ROUND_TIMEOUT")
    if v:
        return float(v)
    return float((getattr(config, "extra", None) or {}).get("round_timeout_s", 0) or 0)
