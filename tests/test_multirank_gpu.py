"""1 rank ≡ 2 ranks ≡ 4 ranks on the GPU.

Two (four) rank processes share the one GPU of the box (gloo carries the collectives: RCCL needs a GPU
per rank; the code path above the communicator is the RCCL one). Each rank trains its half of
the clients with the native kernels; FedAvg reduces the fp64 accumulators across ranks. With
deterministic kernels (split-K chosen per client, ordered folds, no atomics) every client's
update is bitwise the same whichever rank / cohort trains it, so the global model may differ
from the 1-rank run only through the fp64 cross-rank summation order, i.e. not at all after the
fp32 cast except in rare ties.
"""

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = {"distributed_algorithm": "fed_avg", "dataset_name": "CIFAR10", "model_name": "ResNet18", "worker_number": 6,
       "round": 1, "epoch": 1, "batch_size": 32, "learning_rate": 0.01, "dataset_kwargs": {"scale": 0.01},
       "save_models": False, "log_level": "WARNING", "seed": 5}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", DLS_DIST_BACKEND="gloo")
    from distributed_learning_simulator_amd.config import config_from_dict
    from distributed_learning_simulator_amd.parallel import comm as commmod
    from distributed_learning_simulator_amd.session import Session

    commmod._COMM = None
    c = commmod.init_distributed()
    assert c.device.type == "cuda"
    sess = Session(config_from_dict(dict(CFG, save_dir=tmp)), comm=c)
    res = sess.run()
    q.put((rank, sess.server.global_parameter.cpu().numpy().copy(), res["performance"]))
    commmod.shutdown()


@pytest.mark.parametrize("world", [2, 4])
def test_ranks_on_one_gpu_equal_one_rank(hip, tmp_path, world):
    """6 clients dealt round-robin over `world` rank processes (3 / 2 / 1-2 clients each, the
    small-cohort launch rules of an 8-GPU round's per-rank share)."""
    from distributed_learning_simulator_amd.config import config_from_dict
    from distributed_learning_simulator_amd.parallel.comm import Comm
    from distributed_learning_simulator_amd.session import Session

    single = Session(config_from_dict(dict(CFG, save_dir=str(tmp_path / "s"))), comm=Comm(device=torch.device("cuda")))
    single.run()
    ref = single.server.global_parameter.cpu()
    torch.cuda.synchronize()

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path / f"r{r}"), q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0 = torch.from_numpy(out[0][1])
    for r in range(1, world):
        assert torch.equal(g0, torch.from_numpy(out[r][1])), f"server replica {r} diverged"
    diff = (g0 - ref).abs()
    # bitwise up to rare fp64-order ties at the fp32 cast
    assert (diff > 0).float().mean().item() < 1e-5, (diff > 0).sum()
    assert diff.max().item() <= 1e-6 * ref.abs().max().item()
