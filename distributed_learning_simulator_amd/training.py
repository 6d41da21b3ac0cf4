"""Experiment entry points: `train(config, practitioners=None)` and
`get_training_result(task_id, timeout)`.

Reference `training.py:82-169`: `train` deep-copies the config, checks the open-file limit,
adds a file log handler, runs server + worker process groups and returns the result
synchronously (or a task id when `practitioners` is given — concurrent tasks,
`test/test_concurrent.py`); `get_training_result` merges results and remaps Shapley values
from worker ids to practitioner ids.

Here one call = one `Session` per rank. Under torchrun (WORLD_SIZE>1) every rank calls
`train` and rank 0's result is returned. Concurrent tasks run in background threads of the
calling process, each with its own Session, single-rank communicator, HIP stream and
`save_dir/task_<id>` output directory; HIP-graph captures and device-wide synchronisation are
serialised across those threads (engine.memory.DEVICE_LOCK). Tested against serial runs in
tests/test_concurrent.py (the reference's `test/test_concurrent.py:11-46`).
"""

from __future__ import annotations

import copy
import os
import resource
import threading
import uuid
from concurrent.futures import Future, ThreadPoolExecutor
from concurrent.futures import TimeoutError  # noqa: A004 (distinct from builtin on 3.10)

from .parallel.comm import Comm, init_distributed
from .session import Session
from .utils.logging import add_file_handler, get_logger, remove_handler

_tasks: dict[int, dict] = {}
_pool: ThreadPoolExecutor | None = None
_lock = threading.Lock()


def _check_limits() -> None:
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if soft <= 1024 and hard > soft:  # reference training.py:89-95 refuses; we raise the soft limit
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (min(hard, 65536), hard))
        except (ValueError, OSError):
            get_logger().warning("open file limit %s is low", soft)


def _run(config, practitioners=None, comm: Comm | None = None) -> dict:
    session = Session(config, practitioners=practitioners, comm=comm)
    try:
        return session.run()
    finally:
        # (concurrent tasks: no step graph of this session may outlive it into the garbage collector)
        trainer = getattr(session, "trainer", None)
        if trainer is not None and hasattr(trainer, "release_graphs"):
            trainer.release_graphs()


def _run_task(config, practitioners, comm: Comm) -> dict:
    """A concurrent task's thread: its own HIP stream, so its kernels, allocator traffic and
    waits never serialise against another task's (kernel workspaces are keyed by stream, and
    graph captures are serialised process-wide by engine.memory.DEVICE_LOCK)."""
    if comm.device.type == "cuda":
        import torch

        torch.cuda.set_device(comm.device)
        with torch.cuda.stream(torch.cuda.Stream(comm.device)):
            return _run(config, practitioners, comm)
    return _run(config, practitioners, comm)


def train(config, practitioners=None) -> dict | int | None:
    config = copy.deepcopy(config)
    _check_limits()
    if practitioners is None:
        comm = init_distributed()
        handler = add_file_handler(config.log_file) if config.log_file and comm.rank == 0 else None
        try:
            result = _run(config, comm=comm)
        finally:
            if handler is not None:
                remove_handler(handler)
        return result if comm.rank == 0 else None
    global _pool
    with _lock:
        if _pool is None:
            _pool = ThreadPoolExecutor(max_workers=int(os.environ.get("DLS_MAX_CONCURRENT_TASKS", "8")))
    task_id = uuid.uuid4().int
    # each task writes under its own directory (the reference names a task's executors
    # "worker <id> of <task>", executor.py:60-67): concurrent tasks of one config never share files
    config.save_dir = os.path.join(config.save_dir or "session", f"task_{task_id:032x}")
    comm = Comm(0, 1, init_distributed().device)
    fut: Future = _pool.submit(_run_task, config, list(practitioners), comm)
    _tasks[task_id] = {"future": fut, "practitioner_ids": sorted(p.id for p in practitioners), "config": config}
    return task_id


def get_training_result(task_id: int, timeout: float | None = None) -> dict | None:
    task = _tasks.get(task_id)
    if task is None:
        return None
    fut: Future = task["future"]
    try:
        result = fut.result(timeout=timeout)
    except TimeoutError:
        return None
    del _tasks[task_id]
    if "sv" in result:
        # reference training.py:156-167: worker_id -> practitioner_id
        ids = task["practitioner_ids"]
        for key in ("sv", "sv_S"):
            if key in result:
                result[key] = {rnd: {ids[int(w)]: v for w, v in vals.items()} for rnd, vals in result[key].items()}
    return result
