"""GPU-box check: HIP-graph capture of training steps while an RCCL (nccl backend) process group
is live — its watchdog thread polls the events of issued collectives during the capture. Runs a
1-rank nccl group (the 8-GPU driver run uses the same code path per rank), issues an all-reduce
before every local-training call, and trains with graph replay. Exit 0 = capture coexisted."""

import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
    from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
    from distributed_learning_simulator_amd.models.zoo import build_model

    dc = create_dataset_collection("CIFAR10", {"n_train": 1024, "n_test": 128}, 0, dev, torch.bfloat16,
                                   image_channels=8)
    model = build_model("ResNet18", dc.spec)
    tr = CohortTrainer(model, dc, HyperParameter(epoch=2, batch_size=32, learning_rate=0.01), dev, torch.bfloat16,
                       capacity=4)
    theta0 = model.layout.init_flat(torch.Generator().manual_seed(0)).to(dev)
    shards = [torch.arange(i * 256, (i + 1) * 256) for i in range(4)]
    buf = torch.ones(1 << 20, device=dev)
    for r in range(3):
        dist.all_reduce(buf)  # outstanding RCCL work for the watchdog to poll
        tr.load_global(theta0, 4)
        tr.reset_optimizer(4)
        stats = tr.train(tr.build_schedule(shards, 2, seed=r))
        torch.cuda.synchronize()
        assert torch.isfinite(stats.loss_sum).all()
    assert any(sg.graph is not None for sg in tr._graphs.values()), "no step was graph-replayed"
    dist.barrier()
    dist.destroy_process_group()
    print("rccl + graph capture ok")


if __name__ == "__main__":
    main()
