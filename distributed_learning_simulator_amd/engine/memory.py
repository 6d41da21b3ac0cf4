"""Static memory planner: how many clients a rank keeps resident at once (the cohort).

Reference `executor.py:69-93` / `training.py:103` pack executors onto GPUs dynamically: the
first executor in a process takes a cross-process lock, picks the GPU with enough free memory
for its previous peak and releases the lock after the first batch. With all
of a rank's clients advancing together, the equivalent decision is made once, up front:

  per_client = optimizer/parameter state (θ, grad, momentum[, Adam v], bf16 shadow or the fp32
               GEMMs' pre-split weight planes: P_pad each)
             + activation peak of one client's training step (measured by a probe step)
  capacity   = min(clients this rank hosts, ⌊budget / per_client⌋),  budget = fraction × free HBM

Clients beyond the capacity are trained in successive waves through the same buffers.
On MI355X (288 GB HBM3E) a ResNet-18/CIFAR client costs ≈0.2 GB, so 100 clients fit in one
wave; ResNet-50/ImageNet at batch 128 costs ≈20 GB of activations and runs in waves.
"""

from __future__ import annotations

import gc
import math
import threading

import torch

from ..utils.logging import get_logger

# Device-wide operations that must not overlap a HIP-graph capture running on another thread of
# this process (concurrent training tasks, training.train(config, practitioners)): the capture
# itself with the allocator trims around it, device-wide synchronisation and the activation
# probe (whose peak-memory counters are device-global). Re-entrant; uncontended in a
# one-session process.
DEVICE_LOCK = threading.RLock()

# Held by every cyclic garbage collection, from its start to its end, in whatever thread it runs:
# a capture takes it too (inside DEVICE_LOCK), so a collection another task thread started before
# the capture — which can yield the GIL inside a finaliser and free device memory later —
# finishes first. (gc.disable() only stops new collections from starting.)
GC_LOCK = threading.RLock()


def _gc_phase(phase: str, info: dict) -> None:
    if phase == "start":
        GC_LOCK.acquire()
    else:
        GC_LOCK.release()


gc.callbacks.append(_gc_phase)


def state_bytes_per_client(layout, compute_dtype, optimizer: str) -> int:
    P = layout.padded_size
    n = 3 * 4 * P  # theta, grad, state1
    if optimizer.lower() == "adam":
        n += 4 * P
    if compute_dtype != torch.float32:
        n += torch.tensor([], dtype=compute_dtype).element_size() * P
    elif optimizer.lower() != "adam":
        n += 4 * P  # pre-split (hi, lo) bf16 weight planes of the fp32 GEMMs (CohortBuffers.split)
    return n


def probe_activation_bytes(model, dc, hyper, device, compute_dtype) -> int:
    """Activation memory of ONE client's training step at the configured batch size: the
    bytes autograd keeps for the backward (every distinct tensor saved by the forward, counted
    through `saved_tensors_hooks`, so the figure does not depend on allocator state), plus the
    largest single saved tensor twice over for the backward's transient gradients."""
    from .trainer import CohortTrainer

    if device.type != "cuda":
        return 0
    trainer = CohortTrainer(model, dc, hyper, device, compute_dtype, 1)
    B = hyper.batch_size
    n = dc.train.n if hasattr(dc.train, "n") else B
    idx = (torch.arange(B, device=device) % max(n, 1)).view(1, B)
    x = trainer._gather(dc.train, idx)
    y = dc.train.gather_labels(idx)
    valid = torch.full((1,), B, dtype=torch.int32, device=device)
    seen: dict[int, int] = {}

    def pack(t):
        if t.device.type == "cuda":
            seen[t.untyped_storage().data_ptr()] = t.untyped_storage().nbytes()
        return t

    # the step as training runs it: with the weight planes live, BatchNorms also emit activation
    # planes (kept by the convs' autograd contexts, outside saved_tensors: the allocator's peak
    # over the step is taken as well, and the larger figure wins)
    if trainer.buffers.split is not None:
        from ..ops import fl

        fl.split_rows(trainer.buffers.theta[:1], trainer.buffers.split[:1])
        trainer._split_live = True
    torch.cuda.synchronize(device)
    base = torch.cuda.memory_allocated(device)
    torch.cuda.reset_peak_memory_stats(device)
    try:
        with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
            loss, _ = trainer.forward_loss(1, x, y, valid)
        loss.sum().backward()
    finally:
        trainer._split_live = False
    torch.cuda.synchronize(device)
    peak = torch.cuda.max_memory_allocated(device) - base
    # parameter / gradient rows are state (counted by state_bytes_per_client), not activations
    b = trainer.buffers
    state = {t.untyped_storage().data_ptr() for t in (b.theta, b.grad, b.state1, b.state2, b.shadow, b.split)
             if t is not None}
    acts = [nb for ptr, nb in seen.items() if ptr not in state]
    saved = sum(acts)
    biggest = max(acts, default=0)
    del trainer, x, y, loss
    return int(max(saved + 2 * biggest, peak))


def plan_capacity(wanted: int, layout, model, dc, hyper, device, compute_dtype,
                  fraction: float = 0.80, explicit: int = 0) -> int:
    """Cohort size for this rank. `explicit` > 0 (config `cohort_size`) wins."""
    if explicit:
        return max(1, min(wanted, explicit))
    if device.type != "cuda" or wanted <= 1:
        return max(1, wanted)
    state = state_bytes_per_client(layout, compute_dtype, hyper.optimizer_name)
    with DEVICE_LOCK:
        act = probe_activation_bytes(model, dc, hyper, device, compute_dtype)
    per_client = state + int(act * 1.15)  # allocator slack
    free, _total = torch.cuda.mem_get_info(device)
    cap = max(1, min(wanted, int(math.floor(fraction * free / max(per_client, 1)))))
    get_logger().info("memory plan: %.1f MiB state + %.1f MiB activations per client, %.1f GiB free "
                      "-> %d of %d clients resident per wave", state / 2**20, act / 2**20, free / 2**30, cap, wanted)
    return cap
