"""ResNet-18 layer-1 3x3 conv (32x32, 64 -> 64 channels) on the LDS-halo kernel, per tile variant
(csrc/conv_halo.hip conv_halo_set_variant): forward and the dgrad on the forward tiles (wt), fp32
planes, K clients x batch 64 — ms per launch, TFLOP/s of useful fp32 work, and bitwise agreement
with the default variant.

    python bench/halo_variant_bench.py [--K 50] [--variants -1 4] [--iters 10]
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
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--C", type=int, default=64)
    ap.add_argument("--variants", type=int, nargs="+", default=[-1, 4])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip

    K, B, H, C = args.K, args.B, args.H, args.C
    torch.manual_seed(0)
    x = torch.randn(K, B, H, H, C, device="cuda")
    dy = torch.randn(K, B, H, H, C, device="cuda")
    w = torch.randn(K, C, 3, 3, C, device="cuda") * 0.05
    n = C * 9 * C
    wpl = torch.empty((K, 2, n), dtype=torch.bfloat16, device="cuda")
    hip.split_rows(w.reshape(K, n).contiguous(), wpl)
    ws = wpl[:, 0].unflatten(1, (C, 3, 3, C))
    xp, dyp = hip.split_planes(x), hip.split_planes(dy)
    flops = 2.0 * K * B * H * H * C * 9 * C
    fwd = lambda: hip.conv_fwd(x, w, 1, 1, w_split=ws, x_planes=xp)
    # the training dgrad of a block's first conv: + the identity shortcut's gradient gated by ReLU
    # bits, and the BN-backward partials of the BN below (ResNet-18 layer 1)
    acc = torch.randn(K, B, H, H, C, device="cuda")
    mask = torch.randint(0, 256, (K, B * H * H, C // 8), dtype=torch.uint8, device="cuda")
    bx = torch.randn(K, B * H * H, C, device="cuda")
    mean, rstd = bx.mean(1).contiguous(), (1.0 / (bx.var(1) + 1e-5).sqrt()).contiguous()
    valid = torch.full((K,), B * H * H, dtype=torch.int32, device="cuda")
    part = torch.empty((K, hip.conv_stats_parts(B * H * H), 2, C), device="cuda")
    dgr = lambda: hip.conv_dgrad(dy, w, (H, H), 1, 1, w_split=ws, dy_planes=dyp, wt=True, acc=acc, acc_mask=mask,
                                 bnb=(part, bx, mask, mean, rstd, valid, None))
    ref = {}
    best = {}
    for _ in range(args.rounds):
        for v in args.variants:
            hip._C.conv_halo_set_variant(v)
            yf, yd = fwd(), dgr()
            torch.cuda.synchronize()
            if v == args.variants[0]:
                ref = {"fwd": yf, "dgrad": yd}
            same = torch.equal(yf, ref["fwd"]) and torch.equal(yd, ref["dgrad"])
            tf, td = timeit(fwd, args.iters), timeit(dgr, args.iters)
            b = best.get(v)
            best[v] = (min(tf, b[0]) if b else tf, min(td, b[1]) if b else td, same)
    hip._C.conv_halo_set_variant(-1)
    for v, (tf, td, same) in best.items():
        print(json.dumps({"variant": v, "K": K, "fwd_ms": round(tf * 1e3, 4), "dgrad_ms": round(td * 1e3, 4),
                          "fwd_tflops": round(flops / tf / 1e12, 1), "dgrad_tflops": round(flops / td / 1e12, 1),
                          "bitwise_equal_to_first": same}), flush=True)


if __name__ == "__main__":
    main()
