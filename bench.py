"""Headline benchmark: FL rounds/s (+ comm bytes/round) — FedAvg, 100 clients, ResNet-18,
CIFAR-10-shaped synthetic non-IID data, random-init weights (BASELINE.json config 2;
`conf/large_scale/fed_avg/cifar10.yaml` hyper-parameters: 5 local epochs, batch 64, SGD lr 0.1
with cosine schedule).

The other BASELINE.json configs are selectable with `--workload` (same JSON contract):
  fedavg_resnet18     (default) config 2 above
  fedavg_densenet40   the reference's own `conf/large_scale/fed_avg/cifar10.yaml` (DenseNet-40)
  fedobd_transformer  config 3: FedOBD, 100 clients (50 per round), Transformer-base (d 512, 8 heads,
                      6 layers, FFN 2048), AG-News-shaped; stage 1 timed, stage 2 reported apart
  fedobd_imdb         `conf/large_scale/fed_obd/imdb.yaml` verbatim (d 100, 2 layers, L 300,
                      second_phase_epoch 10): block dropout 0.3 + NNADQ 1e-4
  signsgd_resnet50    config 4: sign-SGD, 128 clients, ResNet-50, ImageNet-shaped (batch 128; one
                      round = one local epoch of 1-bit majority-vote steps over a scaled ImageNet shard)
  signsgd_densenet40  the reference's own `conf/sign_sgd/cifar10.yaml` (DenseNet-40, 10 workers, batch 64,
                      SGD 0.1 cosine): one round = `--epoch` epochs of vote steps (the config's 100 epochs
                      in one round is 7.9k steps; vote steps/s is the comparable figure)
  gtg_resnet18        config 5: GTG-Shapley, 32 clients, ResNet-18, 5 local epochs, full test split
  fedavg_mlp_mnist    config 1: FedAvg, 4 clients, MLP, MNIST-shaped (the CPU plumbing check)

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
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


# The reference publishes no numbers. Its execution model — clients trained one
# after another per GPU in eager PyTorch fp32, fp64 server average — re-created with stock
# PyTorch-ROCm (bench/torch_reference_baseline.py) and measured on one MI355X, in rounds/s for
# the default (headline) config, the reference's own DenseNet-40 config, the FedOBD
# Transformer-base config and sign-SGD ResNet-50; profiles/r2_torch_eager_reference_baseline_*.json.
# With N GPUs the reference would deal the clients over N processes: N x this rate at best.
REFERENCE_STYLE_ROUNDS_PER_S = {"fedavg_resnet18": 0.05827, "fedavg_densenet40": 0.03161,
                                # training only (no block dropout / NNADQ): a lower bound on its time
                                "fedobd_transformer": 0.01587,
                                # 128 sequential client gradients per step, 8 vote steps per round
                                "signsgd_resnet50": 0.01621}


def vs_baseline(args, value: float, n_gpus: int, fp32: bool):
    ref = REFERENCE_STYLE_ROUNDS_PER_S.get(args.workload)
    default_cfg = (args.algo == "fed_avg" and args.clients == 100 and args.epoch == 5 and args.batch == 64
                   and not args.emulate_world and (args.model == "ResNet18" or args.workload != "fedavg_resnet18"))
    if ref is None or not fp32 or not default_cfg:
        return None
    if args.workload == "signsgd_resnet50":
        # the eager baseline was measured at 10 % shards (8 vote steps per round): a round of
        # `shard_scale` holds ~shard_scale / 0.1 times as many vote steps
        ref = ref * 0.1 / float(args.shard_scale)
    return value / (ref * n_gpus)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="fedavg_resnet18",
                    choices=["fedavg_resnet18", "fedavg_densenet40", "fedobd_transformer", "fedobd_imdb",
                             "signsgd_resnet50", "signsgd_densenet40", "gtg_resnet18", "fedavg_mlp_mnist"])
    ap.add_argument("--algo", default="fed_avg", choices=["fed_avg", "fed_obd", "fed_obd_sq"],
                    help="fedavg_resnet18: fed_avg or fed_obd; fedobd_*: fed_obd (NNADQ uploads, the default) or "
                         "fed_obd_sq (stochastic 255-level quantisation, method/fed_obd/__init__.py)")
    ap.add_argument("--model", default="ResNet18")
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--epoch", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--cohort", type=int, default=0)
    ap.add_argument("--log-level", default="WARNING", help="simulator log level (INFO shows GTG progress)")
    ap.add_argument("--no-stage2", action="store_true", help="FedOBD workloads: skip timing the second phase")
    ap.add_argument("--amp", action="store_true",
                    help="bf16 fast mode (use_amp: true). Default: fp32, the reference's precision "
                         "(conf/global.yaml use_amp: false) — split-bf16 MFMA GEMMs, fp32 storage/accumulate")
    ap.add_argument("--shard-scale", type=float, default=0.1,
                    help="signsgd_resnet50: fraction of ImageNet dealt to the 128 clients (1.0 = full shards, "
                         "10k images per client, 79 vote steps per round)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="diagnostic: time rank 0's share of an N-rank round alone on one GPU "
                         "(collectives are no-ops; not the benchmark contract)")
    args = ap.parse_args()
    if args.emulate_world and args.workload != "fedavg_resnet18":
        ap.error("--emulate-world supports the fedavg_resnet18 workload only")

    from distributed_learning_simulator_amd.parallel import launch

    if args.gpus > 1 and not launch.under_launcher():
        # one rank per GPU, spawned before anything touches the GPU; rank 0 prints the line
        sys.exit(launch.spawn_ranks(args.gpus))
    if args.backend == "torch":
        os.environ["DLS_BACKEND"] = "torch"
    os.environ.setdefault("DLS_LOG_LEVEL", args.log_level)

    import torch
    import torch.distributed as dist

    from distributed_learning_simulator_amd.config import config_from_dict
    from distributed_learning_simulator_amd.parallel.comm import init_distributed, shutdown
    from distributed_learning_simulator_amd.session import Session

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1 and not torch.cuda.is_available():
        # CPU ranks share the host: split the intra-op threads instead of oversubscribing
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // world_env))

    if torch.cuda.is_available() and args.backend == "hip":
        from distributed_learning_simulator_amd.ops import build

        if int(os.environ.get("RANK", "0")) == 0:
            build.build()
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            # every rank waits until the in-tree binary is linked from THESE sources (rank 0's
            # no-op or incremental build writes the content-hash stamp last), so no rank can
            # import a stale .so while rank 0 replaces it
            build.wait_current()

    comm = init_distributed()
    emulated = args.emulate_world > 1
    if emulated:
        from distributed_learning_simulator_amd.parallel.comm import EmulatedRankComm

        assert comm.world == 1, "--emulate-world runs as a single process"
        comm = EmulatedRankComm(0, args.emulate_world, comm.device)
    rounds = args.warmup + args.steps
    wl = workload_config(args, rounds)
    cfg = config_from_dict(wl["config"])
    sess = Session(cfg, comm=comm)
    server = sess.server
    init = server._before_start()
    theta, _ = server.send_result(init)

    def progress(tag):
        # one stderr line per round keeps long runs visibly alive (gpurun's silence watchdog)
        if comm.rank == 0:
            row = sess.metrics[-1] if sess.metrics else {}
            retries = torch.cuda.memory_stats().get("num_alloc_retries", 0) if torch.cuda.is_available() else 0
            print(f"[bench] {tag} round {row.get('round')} {row.get('wall_s', 0):.2f}s (allocator retries {retries})",
                  file=sys.stderr, flush=True)

    def barrier_sync():
        if comm.world > 1:
            comm.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    # heartbeat: long rounds (GTG utilities, ResNet-50) stay visibly alive on stderr
    t_start = time.perf_counter()

    def beat():
        while True:
            time.sleep(60)
            if comm.rank == 0:
                print(f"[bench] alive {time.perf_counter() - t_start:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    for _ in range(args.warmup):
        theta = sess.run_one_round(theta)
        progress("warmup")
    barrier_sync()
    t0 = time.perf_counter()
    m0 = len(sess.metrics)
    for _ in range(args.steps):
        theta = sess.run_one_round(theta)
        progress("timed")
    barrier_sync()
    elapsed = time.perf_counter() - t0
    # the timed rounds' metrics rows, taken before any stage-2 round appends its own (FedOBD:
    # per-round comm bytes / phases / accuracy describe stage 1 only; stage 2 is reported apart)
    rows = sess.metrics[m0:]
    stage2 = None
    if wl.get("stage2") and not args.no_stage2:
        # FedOBD: the timed rounds above are stage 1; the whole second phase (all clients,
        # `second_phase_epoch` epochs, aggregation after every epoch) is timed on its own
        m1 = len(sess.metrics)
        t1 = time.perf_counter()
        while not server._stopped():
            theta = sess.run_one_round(theta)
            progress("stage2")
        barrier_sync()
        s2 = sess.metrics[m1:]
        stage2 = {"seconds": time.perf_counter() - t1, "epochs": len(s2),
                  "clients": cfg.worker_number,
                  "comm_bytes": sum(r["comm_bytes_total"] for r in s2),
                  "comm_bytes_per_epoch": sum(r["comm_bytes_total"] for r in s2) / max(len(s2), 1),
                  "test_accuracy": s2[-1].get("test_accuracy") if s2 else None}
    if comm.world > 1 and not emulated:
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if stage2 is not None:
            t[0] = stage2["seconds"]
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            stage2["seconds"] = float(t.item())
    bytes_per_round = sum(r["comm_bytes_total"] for r in rows) / max(len(rows), 1)
    acc = rows[-1].get("test_accuracy") if rows else None
    if comm.rank == 0:
        ms = elapsed / args.steps * 1000.0
        out = {
            "metric": wl["metric"],
            "value": args.steps / elapsed,
            "unit": "rounds/s",
            "n_gpus": 1 if emulated else comm.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": vs_baseline(args, args.steps / elapsed, comm.world, sess.compute_dtype != torch.bfloat16),
            "baseline": ("reference-style PyTorch eager fp32 on MI355X, sequential clients "
                         "(bench/torch_reference_baseline.py), x n_gpus"
                         if args.workload in REFERENCE_STYLE_ROUNDS_PER_S else None),
            "dtype": "bf16" if sess.compute_dtype == torch.bfloat16 else "fp32",
            # fp32: activations/weights/gradients fp32; GEMMs as split-bf16 (hi+lo) MFMA with fp32
            # accumulation (≤1e-5 relative vs fp64, tests/test_kernels_f32_gpu.py)
            "matmul": "bf16 MFMA" if sess.compute_dtype == torch.bfloat16 else "split-bf16x3 MFMA, fp32 accumulate",
            "data": wl["data"],
            "comm_bytes_per_round": bytes_per_round,
            "test_accuracy_last_round": acc,
            # mean per-round phase split (HIP-event timed, Session.run_one_round)
            "phase_s": {k: sum(r.get(k, 0.0) for r in rows) / max(len(rows), 1)
                        for k in ("train_s", "aggregate_s", "eval_broadcast_s") if rows and k in rows[0]},
            # (emulated: this rank trains 1/N of the round's samples)
            "samples_per_s": wl["samples_per_round"](sess) / (comm.world if emulated else 1) / (elapsed / args.steps),
            "config": {
                "model": cfg.model_name, "algo": cfg.distributed_algorithm, "clients": cfg.worker_number,
                "local_epochs": cfg.epoch, "global_batch": cfg.batch_size * cfg.worker_number,
                "per_client_batch": cfg.batch_size, "seq_len": wl.get("seq_len"),
                "parallelism": f"emulated-rank0-of-{comm.world}" if emulated else f"client-dp{comm.world}",
                "backend": args.backend, "workload": args.workload, **wl.get("config_extra", {}),
            },
        }
        if stage2 is not None:
            out["stage2"] = stage2
        if torch.cuda.is_available():
            # device memory of this rank: peak allocated, and how often the caching allocator had to
            # free its cache and retry an allocation (a synchronising stall)
            ms = torch.cuda.memory_stats()
            out["memory"] = {"peak_allocated_gb": round(ms.get("allocated_bytes.all.peak", 0) / 2**30, 2),
                             "alloc_retries": int(ms.get("num_alloc_retries", 0))}
        if "extra" in wl:
            out.update(wl["extra"](sess, elapsed / args.steps))
        print(json.dumps(out), flush=True)
    # tear the process group down on every rank (an exiting rank with a live gloo/RCCL group
    # aborts in the communicator's destructor)
    shutdown()


def workload_config(args, rounds: int) -> dict:
    common = {"round": rounds + 1000, "save_models": False, "log_level": args.log_level, "cohort_size": args.cohort,
              "use_amp": bool(args.amp),
              "save_dir": os.path.join("/tmp", f"dls_bench_{os.getpid()}")}

    def shard_samples(sess):
        # samples trained per round: every client's shard × local epochs, scaled by the share of
        # clients a round selects (FedOBD stage 1: random_client_number of worker_number)
        name = sess.dc.spec.name
        total = sum(p.dataset_size(name) for p in sess.practitioners.values()) * sess.config.epoch
        n = sess.config.algorithm_kwargs.get("random_client_number")
        if n is not None and int(n) < sess.config.worker_number:
            total = total * int(n) / sess.config.worker_number
        return total

    if args.workload == "fedavg_mlp_mnist":
        # BASELINE.json config 1: the plumbing check (runs on the CPU executor as well)
        cfg = {"distributed_algorithm": "fed_avg", "dataset_name": "MNIST", "model_name": "MLP", "worker_number": 4,
               "epoch": 1, "batch_size": 64, "optimizer_name": "SGD", "learning_rate": 0.01,
               "dataset_sampling": "iid"}
        return {"config": {**cfg, **common}, "metric": "FL rounds/sec (FedAvg, 4 clients, MLP, MNIST-shaped)",
                "data": "synthetic (MNIST-shaped, iid shards, random-init weights)", "samples_per_round": shard_samples}
    if args.workload == "fedavg_resnet18":
        algo_kwargs, endpoint_kwargs = {}, {}
        if args.algo == "fed_obd":
            algo_kwargs = {"second_phase_epoch": 1, "dropout_rate": 0.3, "random_client_number": args.clients}
            endpoint_kwargs = {"server": {"weight": 0.001}, "worker": {"weight": 0.001}}
        cfg = {"distributed_algorithm": args.algo, "dataset_name": "CIFAR10", "model_name": args.model,
               "worker_number": args.clients, "epoch": args.epoch, "batch_size": args.batch,
               "optimizer_name": "SGD", "learning_rate": 0.1, "learning_rate_scheduler_name": "CosineAnnealingLR",
               "dataset_sampling": "random_label_iid", "dataset_sampling_kwargs": {"sampled_class_number": 5},
               "algorithm_kwargs": algo_kwargs, "endpoint_kwargs": endpoint_kwargs}
        model = "ResNet-18" if args.model == "ResNet18" else args.model
        algo = "FedOBD" if args.algo == "fed_obd" else "FedAvg"
        metric = f"FL rounds/sec ({algo}, {args.clients} clients, {model}, CIFAR-10-shaped)"
        data = "synthetic (CIFAR-10-shaped, random_label_iid non-IID shards, random-init weights)"
        return {"config": {**cfg, **common}, "metric": metric, "data": data, "samples_per_round": shard_samples}
    if args.workload == "fedavg_densenet40":
        # the reference's own large-scale FedAvg config, verbatim (conf/large_scale/fed_avg/cifar10.yaml):
        # DenseNet-40, 100 clients, 5 local epochs, batch 64, SGD lr 0.1 cosine, iid sampling
        # (⇒ keep-best-by-validation uploads, reference aggregation_worker.py:28-29)
        cfg = {"distributed_algorithm": "fed_avg", "dataset_name": "CIFAR10", "model_name": "densenet40",
               "worker_number": args.clients, "epoch": args.epoch, "batch_size": args.batch, "optimizer_name": "SGD",
               "learning_rate": 0.1, "learning_rate_scheduler_name": "CosineAnnealingLR"}
        return {"config": {**cfg, **common}, "samples_per_round": shard_samples,
                "metric": f"FL rounds/sec (FedAvg, {args.clients} clients, DenseNet-40, CIFAR-10-shaped)",
                "data": "synthetic (CIFAR-10-shaped, iid shards, random-init weights)"}
    if args.workload in ("fedobd_transformer", "fedobd_imdb"):
        # stage-1 rounds are the timed steps; stage 2 (second_phase_epoch epochs over all clients)
        # is run to the end afterwards and reported under "stage2"
        sq = args.algo == "fed_obd_sq"
        obd = {"distributed_algorithm": "fed_obd_sq" if sq else "fed_obd", "worker_number": 100, "epoch": 5,
               "batch_size": 64,
               "optimizer_name": "SGD", "learning_rate": 0.01, "learning_rate_scheduler_name": "CosineAnnealingLR",
               "algorithm_kwargs": {"second_phase_epoch": 10, "dropout_rate": 0.3, "random_client_number": 50},
               "endpoint_kwargs": {"server": {"weight": 0.0001}, "worker": {"weight": 0.0001}},
               **common, "round": rounds}
        if args.workload == "fedobd_imdb":
            # the reference's conf/large_scale/fed_obd/imdb.yaml verbatim (d_model 100, 5 heads, 2 layers)
            cfg = {**obd, "dataset_name": "imdb", "model_name": "TransformerClassificationModel",
                   "dataset_kwargs": {"max_len": 300},
                   "model_kwargs": {"d_model": 100, "nhead": 5, "num_encoder_layer": 2, "max_len": 300}}
            return {"config": cfg, "stage2": True, "samples_per_round": shard_samples, "seq_len": 300,
                    "metric": "FL rounds/sec (FedOBD stage 1, 100 clients / 50 per round, Transformer, imdb-shaped)",
                    "data": "synthetic (imdb-shaped token sequences, max_len 300, iid shards, random-init weights)"}
        # BASELINE.json config 3: Transformer-base (d_model 512, 8 heads, 6 layers, FFN 2048) on
        # AG-News-shaped data (4 classes, max_len 128), the reference's FedOBD hyper-parameters
        cfg = {**obd, "dataset_name": "AG_NEWS", "model_name": "TransformerClassificationModel",
               "dataset_kwargs": {"max_len": 128},
               "model_kwargs": {"d_model": 512, "nhead": 8, "num_encoder_layer": 6, "dim_feedforward": 2048,
                                "max_len": 128}}
        return {"config": cfg, "stage2": True, "samples_per_round": shard_samples, "seq_len": 128,
                "config_extra": {"d_model": 512, "nhead": 8, "layers": 6, "ffn": 2048,
                                 "upload_quantiser": "stochastic-255" if sq else "NNADQ"},
                "metric": ("FL rounds/sec (FedOBD" + ("-SQ" if sq else "") +
                           " stage 1, 100 clients / 50 per round, Transformer-base, AG-News-shaped)"),
                "data": "synthetic (AG-News-shaped token sequences, max_len 128, iid shards, random-init weights)"}
    if args.workload == "signsgd_densenet40":
        # conf/sign_sgd/cifar10.yaml verbatim but for `epoch` (--epoch; the config's 100 epochs make
        # one 7.9k-step round): every step is one 1-bit majority vote over the 10 clients
        cfg = {"distributed_algorithm": "sign_SGD", "dataset_name": "CIFAR10", "model_name": "densenet40",
               "worker_number": 10, "epoch": args.epoch, "batch_size": 64, "optimizer_name": "SGD",
               "learning_rate": 0.1, "learning_rate_scheduler_name": "CosineAnnealingLR",
               "distribute_init_parameters": False}

        def dn_extra(sess, s_per_round):
            name = sess.dc.spec.name
            B = sess.config.batch_size
            n = max((p.dataset_size(name) + B - 1) // B for p in sess.practitioners.values()) * sess.config.epoch
            return {"vote_steps_per_round": n, "ms_per_vote_step": s_per_round / n * 1e3,
                    "vote_steps_per_s": n / s_per_round,
                    "reference_round_s_estimate": 100 / sess.config.epoch * s_per_round}

        return {"config": {**cfg, **common}, "samples_per_round": shard_samples, "extra": dn_extra,
                "metric": "FL rounds/sec (sign-SGD, 10 clients, DenseNet-40, CIFAR-10-shaped)",
                "data": "synthetic (CIFAR-10-shaped, iid shards, random-init weights)"}
    if args.workload == "signsgd_resnet50":
        scale = float(args.shard_scale)
        cfg = {"distributed_algorithm": "sign_SGD", "dataset_name": "ImageNet", "model_name": "Resnet50",
               "dataset_kwargs": {"scale": scale}, "worker_number": 128, "epoch": 1, "batch_size": 128,
               "optimizer_name": "SGD", "learning_rate": 0.001, "momentum": 0.0, "distribute_init_parameters": False}

        def vote_steps(sess):
            name = sess.dc.spec.name
            B = sess.config.batch_size
            return max(1, max((p.dataset_size(name) + B - 1) // B for p in sess.practitioners.values()))

        def extra(sess, s_per_round):
            # a round is one local epoch of synchronous steps; every step is one 1-bit majority vote
            # over all 128 clients (reference gradient_worker.py:86-91 exchanges per optimizer step)
            n = vote_steps(sess) * sess.config.epoch
            return {"vote_steps_per_round": n, "ms_per_vote_step": s_per_round / n * 1e3,
                    "vote_steps_per_s": n / s_per_round,
                    "wire": ("1 bit/param/client accounted each way (packed sign words); the cross-rank vote "
                             "all-reduce carries 16-bit counts (fp16, exact up to 2048 clients)")}

        pct = f"{scale * 100:g}%"
        return {"config": {**cfg, **common}, "metric": "FL rounds/sec (sign-SGD, 128 clients, ResNet-50, ImageNet-shaped)",
                # `scale` of ImageNet dealt to 128 clients (0.1: 1,000 images each, 8 steps of batch 128 per
                # round; 1.0: the full 1.28M images, 10k per client, 79 steps)
                "data": f"synthetic (ImageNet-shaped 224x224, {pct} scale shards, random-init weights)",
                "samples_per_round": shard_samples, "extra": extra,
                "config_extra": {"shard_scale": scale}}
    # utility v(S) = test accuracy of the subset model on the FULL test split (reference
    # shapley_value_algorithm.py:67-76); 5 local epochs as conf/gtg_sv/cifar10.yaml
    cfg = {"distributed_algorithm": "GTG_shapley_value", "dataset_name": "CIFAR10", "model_name": "ResNet18",
           "worker_number": 32, "epoch": args.epoch, "batch_size": 64, "optimizer_name": "SGD", "learning_rate": 0.1,
           "learning_rate_scheduler_name": "CosineAnnealingLR",
           "dataset_sampling": "random_label_iid", "dataset_sampling_kwargs": {"sampled_class_number": 5}}
    def gtg_extra(sess, s_per_round):
        sv = getattr(sess.server.algorithm, "sv_algorithm", None)
        if sv is None:
            return {}
        ev = sv.evaluations_per_round.get(max(sv.evaluations_per_round, default=0), 0)
        return {"subset_evaluations_last_round": ev, "gtg_iterations_last_round": sv.iterations_last,
                "gtg_converged": getattr(sv, "converged_last", None), "gtg_max_iterations": sv.max_iterations,
                "subset_evaluations_per_s": ev / s_per_round, "utility_images_per_evaluation": sess.dc.spec.n_test}

    return {"config": {**cfg, **common}, "extra": gtg_extra,
            "metric": "FL rounds/sec (GTG-Shapley, 32 clients, ResNet-18, CIFAR-10-shaped)",
            "data": "synthetic (CIFAR-10-shaped, full 10k test split as the utility set, random_label_iid non-IID "
                    "shards, random-init weights)",
            "samples_per_round": shard_samples}


if __name__ == "__main__":
    main()
