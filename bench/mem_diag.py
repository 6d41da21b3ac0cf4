"""Memory diagnostic: the planner's one-client activation probe against the measured peak of a
K-client training step (per-client and shared-model forms), so a wave-size plan can be checked
before a long run. Prints one JSON line per (mode, K).

    python bench/mem_diag.py --model Resnet50 --dataset ImageNet --batch 128 --K 1 2 4
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="Resnet50")
    ap.add_argument("--dataset", default="ImageNet")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--K", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--shared", type=int, default=1, help="1: all clients read parameter row 0 (sign-SGD)")
    ap.add_argument("--planes", type=int, default=1, help="1: weight planes live (split-plane GEMMs)")
    ap.add_argument("--scale", type=float, default=0.002, help="dataset_kwargs scale (procedural above the limit)")
    args = ap.parse_args()
    from distributed_learning_simulator_amd.data.datasets import create_dataset_collection, get_spec
    from distributed_learning_simulator_amd.engine.memory import probe_activation_bytes, state_bytes_per_client
    from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
    from distributed_learning_simulator_amd.models.zoo import build_model, stored_image_channels
    from distributed_learning_simulator_amd.ops import build, fl

    build.build()
    dev = torch.device("cuda", 0)
    spec = get_spec(args.dataset, {"scale": args.scale})
    dc = create_dataset_collection(args.dataset, {"scale": args.scale}, 0, dev, torch.float32,
                                   image_channels=stored_image_channels(args.model, spec))
    model = build_model(args.model, dc.spec)
    hyper = HyperParameter(epoch=1, batch_size=args.batch, learning_rate=0.001)
    probe = probe_activation_bytes(model, dc, hyper, dev, torch.float32)
    state = state_bytes_per_client(model.layout, torch.float32, "SGD")
    print(json.dumps({"probe_act_mib": probe / 2**20, "state_mib": state / 2**20}), flush=True)
    for K in args.K:
        torch.cuda.empty_cache()
        tr = CohortTrainer(model, dc, hyper, dev, torch.float32, K)
        theta = model.layout.init_flat(torch.Generator().manual_seed(0)).to(dev)
        tr.load_global(theta, K)
        if args.planes and tr.buffers.split is not None:
            fl.split_rows(tr.buffers.theta[:K], tr.buffers.split[:K])
            tr._split_live = True
        n = dc.train.n
        idx = (torch.arange(K * args.batch, device=dev) % n).view(K, args.batch)
        x = tr._gather(dc.train, idx)
        y = dc.train.gather_labels(idx)
        valid = torch.full((K,), args.batch, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        loss, correct = tr.forward_loss(K, x, y, valid, shared=bool(args.shared))
        fwd_peak = torch.cuda.max_memory_allocated() - base
        loss.sum().backward()
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated() - base
        print(json.dumps({"K": K, "scale": args.scale, "base_mib": base / 2**20, "materialized": dc.train.materialized,
                          "shared": args.shared, "planes": args.planes, "fwd_peak_mib": fwd_peak / 2**20,
                          "step_peak_mib": peak / 2**20, "per_client_mib": peak / K / 2**20,
                          "probe_ratio": peak / K / max(probe, 1)}), flush=True)
        # (`correct` too: any live output keeps the whole graph, and the convolutions' activations
        # live in its contexts)
        del tr, x, y, loss, correct


if __name__ == "__main__":
    main()
