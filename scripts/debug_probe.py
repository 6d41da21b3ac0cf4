import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_learning_simulator_amd.ops import build
build.build()
from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
from distributed_learning_simulator_amd.models.zoo import build_model
dev = torch.device("cuda", 0)
dc = create_dataset_collection("CIFAR10", {"scale": 0.02}, 0, dev, torch.bfloat16, image_channels=8)
model = build_model("ResNet18", dc.spec)
hyper = HyperParameter(epoch=1, batch_size=64, learning_rate=0.1)
tr = CohortTrainer(model, dc, hyper, dev, torch.bfloat16, 1)
torch.cuda.synchronize()
base = torch.cuda.memory_allocated(dev)
torch.cuda.reset_peak_memory_stats(dev)
idx = torch.arange(64, device=dev).view(1, 64)
x = tr._gather(dc.train, idx)
print("after gather", torch.cuda.memory_allocated(dev) - base, x.shape, x.dtype, x.device)
y = dc.train.gather_labels(idx)
valid = torch.full((1,), 64, dtype=torch.int32, device=dev)
loss, _ = tr.forward_loss(1, x, y, valid)
torch.cuda.synchronize()
print("after fwd", torch.cuda.memory_allocated(dev) - base, "peak", torch.cuda.max_memory_allocated(dev) - base)
loss.sum().backward()
torch.cuda.synchronize()
print("after bwd", torch.cuda.memory_allocated(dev) - base, "peak", torch.cuda.max_memory_allocated(dev) - base)
