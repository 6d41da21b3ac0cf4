"""Utility-evaluation throughput: M subset models (ResNet-18, fp32) evaluated on the full
CIFAR-10-shaped 10k test split, exactly as GTG-Shapley's batch metric function runs them
(`method/shapley_value/__init__.py` batch_metric → Session.evaluate_tensors → CohortTrainer.evaluate).

    python bench/eval_bench.py [--M 32] [--iters 3] [--max-images 4096 ...] [--streams 2 ...]

Prints one JSON line per (max_images, streams) setting — timed in interleaved rounds, best of
`--rounds` — with ms per M-model chunk, ms per model, images/s and the useful forward TFLOP/s
(1.11 GFLOP per 32x32 ResNet-18 forward).
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
    ap.add_argument("--max-images", type=int, nargs="+", default=[4096])
    ap.add_argument("--streams", type=int, nargs="+", default=[2])
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--fused", type=int, nargs="+", default=[1],
                    help="1: bn1 applied in conv2's halo loader (options.bn_fused_halo), 0: unfused")
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--no-planes", action="store_true", help="A/B: evaluate without weight planes")
    ap.add_argument("--halo-mode", type=int, nargs="+", default=[-1],
                    help="conv_halo_set_mode: -1 shape rule, 1 every supported shape (the 4x4 l4 convs too)")
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

    from distributed_learning_simulator_amd import options

    from distributed_learning_simulator_amd.ops import hip

    settings = [(mi, st, fu, hm) for mi in args.max_images for st in args.streams for fu in args.fused
                for hm in args.halo_mode]
    best = {}
    out = {}
    for _ in range(args.rounds):
        for mi, st, fu, hm in settings:
            tr.num_streams = st
            options.update(bn_fused_halo=bool(fu))
            hip._C.conv_halo_set_mode(hm)
            tr.evaluate(rows, max_images=mi)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                loss, corr, n = tr.evaluate(rows, max_images=mi)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.iters
            if dt < best.get((mi, st, fu, hm), float("inf")):
                best[(mi, st, fu, hm)] = dt
                out[(mi, st, fu, hm)] = (n, float((corr / n).mean()))
    hip._C.conv_halo_set_mode(-1)
    for (mi, st, fu, hm), dt in best.items():
        n, acc = out[(mi, st, fu, hm)]
        imgs = args.M * n
        print(json.dumps({"bench": "eval_resnet18_fp32", "M": args.M, "n_test": n, "planes": not args.no_planes,
                          "max_images": mi, "streams": st, "bn_fused_halo": bool(fu), "halo_mode": hm, "ms_per_chunk": dt * 1e3, "ms_per_model": dt * 1e3 / args.M,
                          "images_per_s": imgs / dt, "fwd_tflops": imgs * FWD_GFLOP_RESNET18_CIFAR / dt / 1e3,
                          "acc_mean": acc}), flush=True)


if __name__ == "__main__":
    main()
