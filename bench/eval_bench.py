"""Utility-evaluation throughput: M subset models (ResNet-18, fp32) evaluated on the full
CIFAR-10-shaped 10k test split, exactly as GTG-Shapley's batch metric function runs them
(`method/shapley_value/__init__.py` batch_metric → Session.evaluate_tensors → CohortTrainer.evaluate).

    python bench/eval_bench.py [--M 32] [--iters 3] [--max-images 8192]

Prints one JSON line: ms per M-model chunk, ms per model, images/s and the useful forward
TFLOP/s (1.11 GFLOP per 32x32 ResNet-18 forward).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

FWD_GFLOP_RESNET18_CIFAR = 1.114  # 2 x 0.557 GMAC


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=32)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--max-images", type=int, default=8192)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--no-planes", action="store_true", help="A/B: evaluate without weight planes")
    args = ap.parse_args()

    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
    from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
    from distributed_learning_simulator_amd.models.zoo import build_model

    dev = torch.device("cuda:0")
    dc = create_dataset_collection("CIFAR10", {"n_train": 512, "n_test": args.n_test}, 0, dev, torch.float32,
                                   image_channels=8)
    model = build_model("ResNet18", dc.spec)
    tr = CohortTrainer(model, dc, HyperParameter(epoch=1, batch_size=64), dev, torch.float32, capacity=1)
    if args.no_planes:
        tr.buffers.split = None
    g = torch.Generator().manual_seed(0)
    rows = torch.stack([model.layout.init_flat(g) for _ in range(args.M)]).to(dev)

    def run():
        return tr.evaluate(rows, max_images=args.max_images)

    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        loss, corr, n = run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters
    imgs = args.M * n
    print(json.dumps({"bench": "eval_resnet18_fp32", "M": args.M, "n_test": n, "planes": not args.no_planes,
                      "max_images": args.max_images, "ms_per_chunk": dt * 1e3, "ms_per_model": dt * 1e3 / args.M,
                      "images_per_s": imgs / dt, "fwd_tflops": imgs * FWD_GFLOP_RESNET18_CIFAR / dt / 1e3,
                      "acc_mean": float((corr / n).mean())}), flush=True)


if __name__ == "__main__":
    main()
