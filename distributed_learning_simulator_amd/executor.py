"""Common base of the server and worker roles.

Reference `executor.py:16-96`: `ExecutorContext` (a process-wide gevent semaphore so only one
executor runs at a time, and the executor's name stamped into the process/thread name for
logging), `Executor` (deep-copied config, `save_dir = <config.save_dir>/<name with _>`,
`_get_device` picks a GPU with enough free memory for the previous peak under a cross-process
lock, `_release_device_lock` records `allocated_bytes.all.peak`).

Cohort form: a rank runs ONE worker object (all its resident clients) and one server replica
side by side on ONE device chosen at `torch.distributed` init (LOCAL_RANK ↔ GPU), so there is
nothing to time-multiplex and no device lock. What remains is the shared identity / output
directory / device accessors and the peak-memory record (used by the memory planner that
sizes the cohort: `engine.memory.plan_capacity`).
"""

from __future__ import annotations

import os

import torch


class Executor:
    def __init__(self, config, name: str, session=None):
        self.config = config
        self.name = name
        self.session = session
        self._peak_bytes: int | None = None

    @property
    def save_dir(self) -> str:
        return os.path.join(self.config.save_dir, self.name.replace(" ", "_"))

    @property
    def device(self) -> torch.device:
        if self.session is not None:
            return self.session.device
        return torch.device("cpu")

    def record_peak_memory(self) -> int:
        """Reference `_release_device_lock` bookkeeping: peak bytes allocated on the device."""
        dev = self.device
        if dev.type == "cuda":
            self._peak_bytes = int(torch.cuda.max_memory_allocated(dev))
        else:
            self._peak_bytes = 0
        return self._peak_bytes

    @property
    def peak_bytes(self) -> int | None:
        return self._peak_bytes

    # resumable state (Session.save_checkpoint / load_checkpoint): tensors and plain numbers
    # only; subclasses with state that outlives a round extend these
    def state_dict(self) -> dict:
        return {}

    def load_state_dict(self, state: dict) -> None:
        pass
