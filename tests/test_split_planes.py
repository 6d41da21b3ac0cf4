"""Pre-split (hi, lo) bf16 weight planes of the fp32 GEMMs (CohortBuffers.split,
BoundParams.ws, ops split_rows / sgd_step(split=)): the CPU rule and the view mapping."""

import torch

from distributed_learning_simulator_amd.engine.params import BoundParams
from distributed_learning_simulator_amd.models.zoo import build_model
from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
from distributed_learning_simulator_amd.ops import ref


def test_split_rows_rule_bounds_and_roundtrip():
    torch.manual_seed(0)
    theta = torch.randn(3, 64) * torch.logspace(-6, 3, 64)
    split = torch.zeros((3, 2, 64), dtype=torch.bfloat16)
    ref.split_rows(theta, split)
    hi, lo = split[:, 0].float(), split[:, 1].float()
    assert torch.equal(hi, theta.to(torch.bfloat16).float())  # hi = RNE(x)
    # x - hi - lo: at most half an ulp of lo, i.e. <= 2^-17 |x| (the split-bf16 GEMM's operand error)
    err = (theta.double() - hi.double() - lo.double()).abs()
    assert torch.all(err <= theta.double().abs() * 2.0 ** -16)


def test_sgd_step_refreshes_split_planes():
    torch.manual_seed(1)
    K, P = 2, 48
    theta, grad, mom = torch.randn(K, P), torch.randn(K, P), torch.zeros(K, P)
    split = torch.zeros((K, 2, P), dtype=torch.bfloat16)
    lr = torch.full((K,), 0.1)
    on = torch.ones(K, dtype=torch.bool)
    ref.sgd_step(theta, grad, mom, lr, on, 0.0, 0.9, 0.0, False, on, None, split)
    exp = torch.zeros_like(split)
    ref.split_rows(theta, exp)
    assert torch.equal(split, exp)


def test_bound_params_ws_views_alias_the_hi_plane():
    dc = create_dataset_collection("CIFAR10", {"n_train": 64, "n_test": 32}, 0, torch.device("cpu"), torch.float32,
                                   image_channels=8)
    model = build_model("ResNet18", dc.spec)
    layout = model.layout
    P = layout.padded_size
    K = 2
    theta = layout.init_flat(torch.Generator().manual_seed(0)).repeat(K, 1)
    split = torch.zeros((K, 2, P), dtype=torch.bfloat16)
    ref.split_rows(theta, split)
    params = BoundParams(layout, theta, None, K=K, split=split)
    name = next(n for n in layout.index() if n.endswith("conv2.weight"))
    w, ws = params.w(name), params.ws(name)
    assert ws.shape == w.shape and ws.dtype == torch.bfloat16
    assert ws.data_ptr() == split[:, 0].data_ptr() + layout.index()[name].offset * 2
    assert torch.equal(ws, w.to(torch.bfloat16))
    assert BoundParams(layout, theta, None, K=K).ws(name) is None
