"""Headline benchmark: FL rounds/s (+ comm bytes/round) — FedAvg, 100 clients, ResNet-18,
CIFAR-10-shaped synthetic non-IID data, random-init weights (BASELINE.json config 2;
`conf/large_scale/fed_avg/cifar10.yaml` hyper-parameters: 5 local epochs, batch 64, SGD lr 0.1
with cosine schedule).

One step = one full FL round: every selected client trains its local epochs (lock-step cohort
on the rank's GPU), uploads are aggregated (fused weighted reduction + RCCL all-reduce across
ranks), the global model is evaluated on the (rank-sharded) test split and broadcast.
The 100 clients are dealt round-robin over the N ranks, so total work is fixed: strong scaling.

  python bench.py --gpus N --steps K --warmup W
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N --steps K --warmup W
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--algo", default="fed_avg", choices=["fed_avg", "fed_obd"])
    ap.add_argument("--model", default="ResNet18")
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--epoch", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--cohort", type=int, default=0)
    args = ap.parse_args()

    if args.backend == "torch":
        os.environ["DLS_BACKEND"] = "torch"
    os.environ.setdefault("DLS_LOG_LEVEL", "WARNING")

    import torch
    import torch.distributed as dist

    from distributed_learning_simulator_amd.config import config_from_dict
    from distributed_learning_simulator_amd.parallel.comm import init_distributed
    from distributed_learning_simulator_amd.session import Session

    if torch.cuda.is_available() and args.backend == "hip":
        from distributed_learning_simulator_amd.ops import build

        if int(os.environ.get("RANK", "0")) == 0:
            build.build()
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            # wait for rank 0's (no-op or incremental) build before other ranks import
            while not os.path.exists(build.TARGET):
                time.sleep(1)

    comm = init_distributed()
    algo_kwargs = {}
    endpoint_kwargs = {}
    if args.algo == "fed_obd":
        algo_kwargs = {"second_phase_epoch": 1, "dropout_rate": 0.3, "random_client_number": args.clients}
        endpoint_kwargs = {"server": {"weight": 0.001}, "worker": {"weight": 0.001}}
    rounds = args.warmup + args.steps
    cfg = config_from_dict({
        "distributed_algorithm": args.algo, "dataset_name": "CIFAR10", "model_name": args.model,
        "worker_number": args.clients, "round": rounds + 1000, "epoch": args.epoch, "batch_size": args.batch,
        "optimizer_name": "SGD", "learning_rate": 0.1, "learning_rate_scheduler_name": "CosineAnnealingLR",
        "dataset_sampling": "random_label_iid", "dataset_sampling_kwargs": {"sampled_class_number": 5},
        "algorithm_kwargs": algo_kwargs, "endpoint_kwargs": endpoint_kwargs,
        "save_models": False, "log_level": "WARNING", "cohort_size": args.cohort,
        "save_dir": os.path.join("/tmp", f"dls_bench_{os.getpid()}"),
    })
    sess = Session(cfg, comm=comm)
    server = sess.server
    init = server._before_start()
    theta, _ = server.send_result(init)

    def barrier_sync():
        if comm.world > 1:
            comm.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        theta = sess.run_one_round(theta)
    barrier_sync()
    t0 = time.perf_counter()
    m0 = len(sess.metrics)
    for _ in range(args.steps):
        theta = sess.run_one_round(theta)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if comm.world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    rows = sess.metrics[m0:]
    bytes_per_round = sum(r["comm_bytes_total"] for r in rows) / max(len(rows), 1)
    acc = rows[-1].get("test_accuracy") if rows else None
    if comm.rank == 0:
        ms = elapsed / args.steps * 1000.0
        out = {
            "metric": "FL rounds/sec (FedAvg, 100 clients, ResNet-18, CIFAR-10-shaped)",
            "value": args.steps / elapsed,
            "unit": "rounds/s",
            "n_gpus": comm.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16" if sess.compute_dtype == torch.bfloat16 else "fp32",
            "data": "synthetic (CIFAR-10-shaped, random_label_iid non-IID shards, random-init weights)",
            "comm_bytes_per_round": bytes_per_round,
            "test_accuracy_last_round": acc,
            "images_per_s": args.clients * args.epoch * (50000 // args.clients) / (elapsed / args.steps),
            "config": {
                "model": args.model, "algo": args.algo, "clients": args.clients, "local_epochs": args.epoch,
                "global_batch": args.batch * args.clients, "per_client_batch": args.batch, "seq_len": None,
                "parallelism": f"client-dp{comm.world}", "backend": args.backend,
            },
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
