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


def _kfd_gpus() -> int | None:
    """GPUs this process may open, from the KFD topology (sysfs, no driver call): nodes whose
    gfx_target_version is non-zero (CPU nodes report 0) AND whose DRM render node is present
    and accessible here (a container sees the host's whole topology but only its own
    /dev/dri/renderD* devices). None when the topology is not readable."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(root)
    except OSError:
        return None
    n = 0
    for node in nodes:
        props = {}
        try:
            with open(os.path.join(root, node, "properties")) as fh:
                for line in fh:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
        except OSError:
            continue
        try:
            if int(props.get("gfx_target_version", "0")) == 0:
                continue
            minor = int(props.get("drm_render_minor", "-1"))
        except ValueError:
            continue
        if minor >= 0 and os.access(f"/dev/dri/renderD{minor}", os.R_OK | os.W_OK):
            n += 1
    return n


def _env_visible(n: int) -> int:
    """Apply HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES to n devices."""
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids)) if ids else 0
    return n


def visible_gpus() -> int:
    """Number of visible GPUs WITHOUT initialising the HIP runtime in this process (the parent
    spawns the rank processes afterwards: nothing may touch the GPU before). Read from the KFD
    sysfs topology and the *_VISIBLE_DEVICES masks; if sysfs is unreadable, counted by a
    short-lived child process, never by torch.cuda in this one (which falls back to
    hipGetDeviceCount when amdsmi discovery fails)."""
    if os.environ.get("DLS_FORCE_CPU", "0") == "1":
        return 0
    n = _kfd_gpus()
    if n is not None:
        return _env_visible(n)
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=300)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else 0
    except Exception:  # pragma: no cover - no python / torch in the child
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
