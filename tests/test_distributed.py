"""Multi-rank execution on CPU (gloo — the same code path as RCCL on MI355X): results at world
size 2, 4 and 8 must match the single-rank run (client sharding + all-reduce aggregation +
sharded evaluation are exact up to fp32 summation order), for FedAvg (full and partial
participation), FedDropoutAvg, FedPAQ, FedOBD (both phases), federated GNN with the halo
exchange, sign-SGD and GTG-Shapley. Also the self-launching entry point (parallel/launch.py)."""

import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


BASE = {"dataset_name": "MNIST", "model_name": "LeNet5", "worker_number": 8, "round": 2, "epoch": 1,
        "batch_size": 32, "learning_rate": 0.05, "dataset_kwargs": {"scale": 0.03}, "save_models": False,
        "log_level": "WARNING", "seed": 3}


def _cfg(algo, tmp, extra=None):
    from distributed_learning_simulator_amd.config import config_from_dict

    d = dict(BASE, distributed_algorithm=algo, save_dir=tmp)
    for k, v in (extra or {}).items():
        d[k] = v
    return config_from_dict(d)


def _worker(rank, world, port, algo, tmp, extra, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DLS_FORCE_CPU="1")
    torch.set_num_threads(1)
    from distributed_learning_simulator_amd.parallel import comm as commmod
    from distributed_learning_simulator_amd.session import Session

    commmod._COMM = None
    c = commmod.init_distributed(prefer_gpu=False)
    sess = Session(_cfg(algo, tmp, extra), comm=c)
    res = sess.run()
    # numpy pickles by value: a tensor would travel as a shared-memory fd that dies with this process
    q.put((rank, sess.server.global_parameter.cpu().numpy().copy(), res["performance"], res["bytes_up"], res.get("sv")))
    commmod.shutdown()


def _run_world(world, algo, tmp, extra=None):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, algo, tmp, extra, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = [(o[0], torch.from_numpy(o[1]), *o[2:]) for o in out]
    return sorted(out, key=lambda t: t[0])


def _single(algo, tmp, extra=None):
    from distributed_learning_simulator_amd.parallel.comm import Comm
    from distributed_learning_simulator_amd.session import Session

    # same intra-op thread count as the spawned ranks: fp32 reduction order then matches
    nthreads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        s = Session(_cfg(algo, tmp, extra), comm=Comm())
        res = s.run()
    finally:
        torch.set_num_threads(nthreads)
    return s.server.global_parameter, res


CASES = [
    ("fed_avg", None, 2),
    ("fed_avg", None, 4),
    ("fed_avg", None, 8),
    ("fed_avg", {"algorithm_kwargs": {"random_client_number": 5}}, 4),
    ("fed_dropout_avg", {"algorithm_kwargs": {"dropout_rate": 0.3}}, 2),
    ("fed_paq", None, 4),
    ("fed_obd", {"algorithm_kwargs": {"random_client_number": 6, "second_phase_epoch": 2, "dropout_rate": 0.3},
                 "endpoint_kwargs": {"server": {"weight": 0.01}, "worker": {"weight": 0.01}}}, 4),
    ("GTG_shapley_value", {"worker_number": 4}, 2),
    ("GTG_shapley_value", {"worker_number": 4}, 4),
]


@pytest.mark.parametrize("algo,extra,world", CASES)
def test_n_ranks_match_single_rank(tmp_path, algo, extra, world):
    theta1, res1 = _single(algo, str(tmp_path / "s"), extra)
    outs = _run_world(world, algo, str(tmp_path / "d"), extra)
    th0 = outs[0][1]
    for o in outs[1:]:
        torch.testing.assert_close(o[1], th0, rtol=0, atol=0)  # replicas identical
    # quantisation (fed_paq stochastic, fed_obd NNADQ) may flip one step where fp32 client deltas
    # differ in the last bit between cohort compositions
    atol = 2e-3 if algo in ("fed_paq", "fed_obd") else 1e-5
    torch.testing.assert_close(th0, theta1, rtol=1e-4, atol=atol)
    assert outs[0][3] == res1["bytes_up"]
    for k in res1["performance"]:
        assert abs(outs[0][2][k]["test_accuracy"] - res1["performance"][k]["test_accuracy"]) < 1e-6 + 2e-3
    if algo == "GTG_shapley_value":
        sv_n, sv_1 = outs[0][4], res1["sv"]
        assert sv_n.keys() == sv_1.keys()
        for r in sv_1:
            for w in sv_1[r]:
                assert abs(sv_n[r][w] - sv_1[r][w]) < 1e-4


def test_fed_gnn_halo_ranks_match_single_rank(tmp_path):
    extra = {"dataset_name": "Coauthor_CS", "model_name": "TwoGCN", "worker_number": 4, "dataset_kwargs": {"scale": 0.05},
             "optimizer_name": "Adam", "learning_rate": 0.01, "batch_size": 64,
             "algorithm_kwargs": {"share_feature": True}}
    theta1, res1 = _single("fed_gnn", str(tmp_path / "s"), extra)
    outs = _run_world(4, "fed_gnn", str(tmp_path / "d"), extra)
    for o in outs[1:]:
        torch.testing.assert_close(o[1], outs[0][1], rtol=0, atol=0)
    torch.testing.assert_close(outs[0][1], theta1, rtol=1e-4, atol=1e-5)
    assert outs[0][3] == res1["bytes_up"]


@pytest.mark.parametrize("world", [2, 4])
def test_sign_sgd_ranks_match_single_rank(tmp_path, world):
    extra = {"learning_rate": 0.001, "round": 1, "momentum": 0.0, "distribute_init_parameters": False}
    theta1, _ = _single("sign_SGD", str(tmp_path / "s"), extra)
    outs = _run_world(world, "sign_SGD", str(tmp_path / "d"), extra)
    for o in outs[1:]:
        torch.testing.assert_close(o[1], outs[0][1], rtol=0, atol=0)
    # majority votes are integers: identical whatever the client sharding
    torch.testing.assert_close(outs[0][1], theta1, rtol=1e-5, atol=1e-6)


def test_self_launch_spawns_ranks(tmp_path):
    """`python simulator.py ... parallel_number=2` starts 2 ranks by itself (no torchrun)."""
    env = dict(os.environ, DLS_FORCE_CPU="1", PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "simulator.py"), "--config-name", "fed_avg/mnist.yaml",
           "++fed_avg.round=1", "++fed_avg.epoch=1", "++fed_avg.parallel_number=2", "++fed_avg.worker_number=4",
           "++fed_avg.dataset_kwargs.scale=0.03", f"++fed_avg.save_dir={tmp_path}"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "[rank 1]" in r.stderr and "ranks=2" in r.stderr
    rows = [json.loads(line) for line in open(tmp_path / "metrics.jsonl")]
    assert rows[0]["gpus"] == 2


def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` (no torchrun): 2 ranks, ONE JSON line with n_gpus = 2."""
    env = dict(os.environ, DLS_FORCE_CPU="1", PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--workload", "fedavg_mlp_mnist"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [line for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0


@pytest.mark.parametrize("share", [True, False])
def test_fed_gnn_rank_without_clients(tmp_path, share):
    """a rank left without an active client (here 3 clients, 1 selected per round, on
    4 ranks) still runs every collective of the round — halo all-to-alls (share_feature), the
    fed_aas-free embedding-byte all-reduce, FedAvg — with empty contributions: no hang, and the
    result equals the single-rank run."""
    extra = {"dataset_name": "Coauthor_CS", "model_name": "TwoGCN", "worker_number": 3, "dataset_kwargs": {"scale": 0.05},
             "optimizer_name": "Adam", "learning_rate": 0.01, "batch_size": 64,
             "algorithm_kwargs": {"share_feature": share, "random_client_number": 1}}
    theta1, res1 = _single("fed_gnn", str(tmp_path / "s"), extra)
    outs = _run_world(4, "fed_gnn", str(tmp_path / "d"), extra)
    for o in outs[1:]:
        torch.testing.assert_close(o[1], outs[0][1], rtol=0, atol=0)
    torch.testing.assert_close(outs[0][1], theta1, rtol=1e-4, atol=1e-5)
