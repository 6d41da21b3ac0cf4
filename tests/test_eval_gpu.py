"""Batched model evaluation on the GPU (the GTG-Shapley utility path).

CohortTrainer.evaluate runs M models x (test batches per launch) virtual clients; with fp32 on
the GPU it hands the split-plane GEMMs each model's (hi, lo) weight planes, shared by the
`rep` virtual clients of that model (csrc/conv_pl.hip / conv_halo.hip `client / rep`).
Checked against the in-kernel-split fp32 path (no planes) and the CPU fp32 oracle.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(device, n_test=700):
    from distributed_learning_simulator_amd.data.datasets import create_dataset_collection
    from distributed_learning_simulator_amd.engine.trainer import CohortTrainer, HyperParameter
    from distributed_learning_simulator_amd.models.zoo import build_model

    dc = create_dataset_collection("CIFAR10", {"n_train": 128, "n_test": n_test}, 0, torch.device(device),
                                   torch.float32, image_channels=8)
    model = build_model("ResNet18", dc.spec)
    tr = CohortTrainer(model, dc, HyperParameter(epoch=1, batch_size=64), torch.device(device), torch.float32,
                       capacity=1)
    g = torch.Generator().manual_seed(1)
    rows = torch.stack([model.layout.init_flat(g) for _ in range(3)])
    return tr, rows


def test_eval_planes_rep_matches_plain_and_cpu(hip):
    from distributed_learning_simulator_amd.ops import hip as H

    tr, rows = _setup("cuda")
    assert tr.buffers.split is not None
    dev_rows = rows.cuda()
    before = dict(H.planes_launches)
    # 3 models x 4 batches per launch (rep = 4), 11 batches: a ragged last launch (rep = 3)
    lp, cp, n = tr.evaluate(dev_rows, max_images=3 * 4 * 64)
    assert H.planes_launches["fwd"] > before.get("fwd", 0), "evaluation did not take the split-plane GEMMs"
    split = tr.buffers.split
    tr.buffers.split = None
    lq, cq, _ = tr.evaluate(dev_rows, max_images=3 * 4 * 64)
    tr.buffers.split = split
    torch.cuda.synchronize()
    # planes and in-kernel split are the same bf16x3 products: equal up to summation order
    assert torch.allclose(lp, lq, rtol=1e-5, atol=1e-5 * n), (lp, lq)
    assert (cp - cq).abs().max().item() <= 2, (cp, cq)
    tc, rows_c = _setup("cpu")
    lc, cc, nc = tc.evaluate(rows_c, max_images=3 * 4 * 64)
    assert nc == n
    assert torch.allclose(lp.cpu(), lc, rtol=2e-4, atol=1e-4 * n), (lp, lc)
    assert (cp.cpu() - cc).abs().max().item() <= 3, (cp, cc)
