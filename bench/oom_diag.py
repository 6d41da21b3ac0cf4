"""Where does a wave's memory go? Runs a bench.py workload (default: sign-SGD ResNet-50, the wave
that runs out of memory) with the CUDA caching allocator's history recorder on from the first
trained wave, and at the first out-of-memory error prints the live allocations grouped by the
innermost frame of this package that made them (bytes, count, largest), then stops.

    python bench/oom_diag.py [--top 40] [-- bench.py arguments]
"""

from __future__ import annotations

import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarize(snapshot: dict, top: int) -> None:
    groups: dict = defaultdict(lambda: [0, 0, 0])
    total = 0
    for seg in snapshot.get("segments", []):
        for blk in seg.get("blocks", []):
            if blk.get("state") != "active_allocated":
                continue
            size = int(blk.get("size", 0))
            total += size
            key = "(allocated before recording)"
            frames = blk.get("frames") or []
            pkg = [f for f in frames if "distributed_learning_simulator_amd" in f.get("filename", "")]
            if pkg:
                f = pkg[0]
                key = f"{os.path.relpath(f['filename'], ROOT)}:{f['line']} {f['name']}"
            elif frames:
                f = frames[0]
                key = f"{f.get('filename', '?')}:{f.get('line', '?')} {f.get('name', '?')}"
            g = groups[key]
            g[0] += size
            g[1] += 1
            g[2] = max(g[2], size)
    print(f"[oom_diag] live allocations: {total / 2**30:.1f} GiB in {sum(g[1] for g in groups.values())} blocks",
          flush=True)
    for key, (b, n, mx) in sorted(groups.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"[oom_diag] {b / 2**30:8.2f} GiB  n={n:6d}  max={mx / 2**20:9.1f} MiB  {key}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    args = ap.parse_args()
    bench_args = [a for a in args.rest if a != "--"] or ["--workload", "signsgd_resnet50", "--steps", "1",
                                                          "--warmup", "0", "--log-level", "INFO"]
    import torch

    from distributed_learning_simulator_amd.engine import trainer as trainer_mod

    orig = trainer_mod.CohortTrainer.forward_loss
    state = {"recording": False}

    def forward_loss(self, K, *a, **kw):
        if not state["recording"]:
            torch.cuda.memory._record_memory_history(enabled="all", context="alloc", stacks="python",
                                                     max_entries=500000)
            state["recording"] = True
            print(f"[oom_diag] recording from the first wave ({K} clients); "
                  f"{torch.cuda.memory_allocated() / 2**30:.1f} GiB allocated", flush=True)
        try:
            return orig(self, K, *a, **kw)
        except torch.OutOfMemoryError:
            print(f"[oom_diag] out of memory in the forward of a {K}-client wave", flush=True)
            summarize(torch.cuda.memory._snapshot(), args.top)
            raise SystemExit(0)

    trainer_mod.CohortTrainer.forward_loss = forward_loss
    # the backward allocates too: catch an OOM there through the worker's wave loop
    import distributed_learning_simulator_amd.worker.gradient_worker as gw

    orig_steps = gw.GradientWorker._steps

    def steps(self, *a, **kw):
        try:
            return orig_steps(self, *a, **kw)
        except torch.OutOfMemoryError:
            print("[oom_diag] out of memory outside the forward", flush=True)
            summarize(torch.cuda.memory._snapshot(), args.top)
            raise SystemExit(0)

    gw.GradientWorker._steps = steps
    sys.argv = ["bench.py"] + bench_args
    import runpy

    runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")


if __name__ == "__main__":
    main()
