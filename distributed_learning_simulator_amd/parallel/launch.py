"""One-process-per-GPU launcher (reference `training.py:105-125` `TorchProcessPool` +
`config.py:22` `parallel_number = len(get_devices())`).

`python simulator.py ...` / `python bench.py --gpus N` call `spawn_ranks(N, ...)` BEFORE anything
touches the GPU: the parent starts N fresh child processes (`subprocess.Popen`, not fork/exec of
an initialised process) running the same script with the torchrun environment
(RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT), waits for
them, and exits with their status. Each child becomes one rank of the RCCL (xGMI) process
group; rank 0 prints the results. A child that fails makes the parent stop the others (a
clean abort instead of peers blocking in a collective until the RCCL timeout — SURVEY §5.3).
Under an external launcher (WORLD_SIZE already set) nothing is spawned.
"""

from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
import uuid

# children inherit this; it makes a second spawn from a child impossible
_CHILD_FLAG = "DLS_LAUNCHED_RANK"


def visible_gpus() -> int:
    """Number of visible GPUs without initialising the HIP runtime in this process
    (`torch.cuda.device_count()` only enumerates)."""
    if os.environ.get("DLS_FORCE_CPU", "0") == "1":
        return 0
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # pragma: no cover - torch without a device runtime
        return 0


def under_launcher() -> bool:
    return "WORLD_SIZE" in os.environ or _CHILD_FLAG in os.environ


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list[str] | None = None, script: str | None = None,
                poll_s: float = 0.2, extra_env: dict | None = None) -> int:
    """Run `python script argv` as n ranks; returns the worst exit code (0 = all ok)."""
    script = script or os.path.abspath(sys.argv[0])
    argv = list(sys.argv[1:] if argv is None else argv)
    port = int(os.environ.get("MASTER_PORT", "0")) or free_port()
    procs: list[subprocess.Popen] = []
    base = dict(os.environ)
    base.setdefault("DLS_RUN_ID", str(uuid.uuid4()))
    base.setdefault("DLS_RUN_TIME", time.strftime("%Y-%m-%d_%H_%M_%S"))
    base.update(extra_env or {})
    for r in range(n):
        env = dict(base)
        env.update(RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR=env.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=str(port))
        env[_CHILD_FLAG] = "1"
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL peer buffers)
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env,
                                      start_new_session=False))
    worst = 0
    try:
        alive = set(range(n))
        while alive:
            for r in sorted(alive):
                rc = procs[r].poll()
                if rc is None:
                    continue
                alive.discard(r)
                if rc != 0:
                    worst = rc if worst == 0 else worst
                    # one rank died: the others would block in their next collective
                    for o in alive:
                        if procs[o].poll() is None:
                            procs[o].send_signal(signal.SIGTERM)
            if alive:
                time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        raise
    finally:
        for p in procs:
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()
    return worst
