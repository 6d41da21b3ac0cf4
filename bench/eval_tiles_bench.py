"""Tile sweep of the plane-GEMM forward (csrc/conv_pl.hip, every conv_nt_pl variant) on large-M
launches of the ResNet-18 layer shapes: `--K` clients x 8192 images per launch, fp32 planes
operands, BN statistics in the epilogue — the strided 3x3 convs, the 1x1 stride-2 shortcuts and
l4. (CohortTrainer.evaluate does not launch these: it runs each 64-image test batch as a virtual
client; the large-M rule it informed serves ResNet-50's 56x56 layers.) Best of `--rounds`.

    python bench/eval_tiles_bench.py [--K 4] [--B 8192] [--iters 5]
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

# (name, H, Ci, Co, k, stride)
SHAPES = [("l2a", 32, 64, 128, 3, 2), ("l2sc", 32, 64, 128, 1, 2), ("l3a", 16, 128, 256, 3, 2),
          ("l3sc", 16, 128, 256, 1, 2), ("l4a", 8, 256, 512, 3, 2), ("l4sc", 8, 256, 512, 1, 2),
          ("l4", 4, 512, 512, 3, 1)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=4)
    ap.add_argument("--B", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip

    dev = torch.device("cuda:0")
    K = args.K
    nv = hip._C.conv_nt_pl_num_variants()
    for name, H, Ci, Co, k, s in SHAPES:
        B = args.B if H < 32 else args.B // 2  # (a client's 32x32x64 planes past 2 GiB run batch-chunked)
        pad = k // 2
        OH = (H + 2 * pad - k) // s + 1
        x = torch.randn(K, B, H, H, Ci, device=dev)
        w = torch.randn(K, Co, k, k, Ci, device=dev) * 0.05
        n = w[0].numel()
        planes = torch.empty((K, 2, n), dtype=torch.bfloat16, device=dev)
        hip.split_rows(w.reshape(K, n).contiguous(), planes)
        ws = planes[:, 0].view(w.shape)
        xp = hip.split_planes(x)
        M = B * OH * OH
        st = torch.empty((K, hip.conv_stats_parts(M), 2, Co), device=dev)
        valid = torch.full((K,), B, dtype=torch.int32, device=dev)
        flops = 2.0 * K * M * Co * k * k * Ci
        best = {}
        try:
            for _ in range(args.rounds):
                for v in [-1] + list(range(nv)):
                    hip._C.conv_nt_pl_set_variant(v)
                    t = timeit(lambda: hip.conv_fwd(x, w, s, pad, w_split=ws, x_planes=xp, stats=st, stats_valid=valid),
                               args.iters)
                    best[v] = min(best.get(v, 1e9), t)
        finally:
            hip._C.conv_nt_pl_set_variant(-1)
        row = {"layer": name, "K": K, "B": B, "default_ms": round(best[-1] * 1e3, 3),
               "ms": {v: round(best[v] * 1e3, 3) for v in range(nv)},
               "tflops": {v: round(flops / best[v] / 1e12, 1) for v in [-1] + list(range(nv))}}
        print(json.dumps(row), flush=True)
        del x, w, planes, xp, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
