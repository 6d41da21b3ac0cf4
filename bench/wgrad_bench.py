"""3x3 stride-1 weight gradients of the ResNet-18 / CIFAR layers: the LDS-halo kernel
(csrc/conv_halo_wgrad.hip, every operand mode and both tile heights) against the implicit-GEMM
plane kernel (csrc/conv_pl.hip) — ms per launch and TFLOP/s of useful fp32 work.

    python bench/wgrad_bench.py [--K 50] [--iters 20]
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

LAYERS = [("l1", 32, 64), ("l2", 16, 128), ("l3", 8, 256)]


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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated layers (l1,l2,l3)")
    ap.add_argument("--runs", default="", help="comma-separated run names")
    ap.add_argument("--unroll", default="1,2")
    args = ap.parse_args()
    from distributed_learning_simulator_amd import options
    from distributed_learning_simulator_amd.ops import hip

    K, B = args.K, args.B
    for name, H, C in LAYERS:
        if args.only and name not in args.only.split(","):
            continue
        x = torch.randn(K, B, H, H, C, device="cuda")
        dy = torch.randn(K, B, H, H, C, device="cuda")
        xp, dyp = hip.split_planes(x), hip.split_planes(dy)
        gw = torch.empty((K, C, 3, 3, C), device="cuda")
        coef = torch.stack([torch.rand(K, C, device="cuda") + 0.5, torch.randn(K, C, device="cuda")], -1).contiguous()
        flop = 2.0 * K * B * H * H * C * C * 9
        # the BN backward in the dY loader (dy mode 2): dy_out, the BN's raw input, ReLU bits, (a, d, e)
        R = B * H * H
        dyo = torch.randn(K, R, C, device="cuda")
        xbn = torch.randn(K, R, C, device="cuda")
        mk = torch.randint(0, 256, (K, R * C // 8), dtype=torch.uint8, device="cuda")
        cf3 = torch.randn(K, C, 3, device="cuda").contiguous()
        dxp = torch.empty((K, 2, R, C), dtype=torch.bfloat16, device="cuda")
        bnb = (dyo, xbn, mk, cf3, None, dxp)
        runs = {
            "tn_planes": lambda: hip.conv_wgrad(dy, x, gw, 1, 1, dy_planes=dyp, x_planes=xp),
            "bn_bwd_apply_pass": lambda: hip.bn_bwd_apply_planes(dyo, xbn, mk, cf3, None, dxp),
            "halo_xplanes_dm2": lambda: hip.halo_wgrad(dy, x, gw, x_planes=xp, bn_bwd=bnb),
            "halo_bn_dm2": lambda: hip.halo_wgrad(dy, x, gw, bn=(coef, True, None), bn_bwd=bnb),
            "halo_planes": lambda: hip.halo_wgrad(dy, x, gw, dy_planes=dyp, x_planes=xp),
            "halo_f32": lambda: hip.halo_wgrad(dy, x, gw),
            "halo_bn_dyplanes": lambda: hip.halo_wgrad(dy, x, gw, dy_planes=dyp, bn=(coef, True, None)),
        }
        for small in [int(v) for v in args.unroll.split(",")]:
            with options.override(native={"halo_wgrad_unroll": small}):
                for rn, fn in runs.items():
                    if (rn in ("tn_planes", "bn_bwd_apply_pass") and small != 1) or (args.runs and rn not in args.runs.split(",")):
                        continue
                    t = timeit(fn, args.iters)
                    print(json.dumps({"layer": name, "K": K, "run": rn, "unroll": small if rn != "tn_planes" else None,
                                      "ms": round(t * 1e3, 4), "tflops": round(flop / t / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
