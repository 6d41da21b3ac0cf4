"""Run one GEMM kernel configuration in a loop (a target for rocprofv3 --pmc passes).

    python bench/pl_probe.py --layer l3 --op fwd --variant 1 [--planes] [--K 50] [--iters 20]

`--planes`: the pre-split-operand LDS-DMA kernels (csrc/conv_pl.hip, variant = conv_nt_pl id);
otherwise the register-staged split kernels with pre-split weights (variant = nt_f32 id, -1 =
heuristic). Shapes are bench/kernel_bench.py's ResNet-18 CIFAR layers, batch 64 per client.
"""

from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

import torch  # noqa: E402

from kernel_bench import RESNET18_CIFAR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="l3")
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--planes", action="store_true")
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from distributed_learning_simulator_amd.ops import hip

    name, H, Ci, Co, k, s = next(r for r in RESNET18_CIFAR if r[0] == args.layer)
    K, B, pad = args.K, args.B, k // 2
    OH = (H + 2 * pad - k) // s + 1
    x = torch.randn(K, B, H, H, Ci, device="cuda")
    w = torch.randn(K, Co, k, k, Ci, device="cuda") * 0.05
    dy = torch.randn(K, B, OH, OH, Co, device="cuda")
    n = Co * k * k * Ci
    wpl = torch.empty((K, 2, n), dtype=torch.bfloat16, device="cuda")
    hip.split_rows(w.reshape(K, n).contiguous(), wpl)
    ws = wpl[:, 0].unflatten(1, (Co, k, k, Ci))
    gw = torch.empty(K, Co, k, k, Ci, device="cuda")
    xp = hip.split_planes(x) if args.planes else None
    dyp = hip.split_planes(dy) if args.planes else None
    if args.planes:
        hip._C.conv_nt_pl_set_variant(args.variant)
    else:
        hip.nt_f32_variant = args.variant
    if args.op == "fwd":
        fn = lambda: hip.conv_fwd(x, w, s, pad, w_split=ws, x_planes=xp)  # noqa: E731
    elif args.op == "dgrad":
        fn = lambda: hip.conv_dgrad(dy, w, (H, H), s, pad, w_split=ws, dy_planes=dyp)  # noqa: E731
    else:
        fn = lambda: hip.conv_wgrad(dy, x, gw, s, pad, **({"dy_planes": dyp, "x_planes": xp} if args.planes else {}))  # noqa: E731
    for _ in range(args.iters):
        fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.iters):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / args.iters
    flops = 2.0 * K * B * OH * OH * Co * Ci * k * k
    print(f"{name} {args.op} planes={args.planes} v={args.variant}: {ms:.3f} ms {flops / ms / 1e9:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
