"""Per-layer microbenchmark of sign-SGD's ResNet-50 (ImageNet 224², batch 128 per client, K clients
sharing ONE weight row, fp32 via the split-bf16 plane kernels — the layout
`worker/gradient_worker.py` trains with): fwd / dgrad / wgrad ms and TFLOP/s per unique conv shape,
weighted by how often the shape occurs in the network, plus the BN apply passes at the l1 / l2
shapes. One JSON line per shape and a summary line (modelled conv ms per wave).

    python bench/r50_kernel_bench.py [--K 7] [--B 128] [--iters 5]
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

# (name, H_in, Ci, Co, k, stride, occurrences in ResNet-50)
RESNET50 = [
    ("l1.c1a", 56, 64, 64, 1, 1, 1),
    ("l1.c1", 56, 256, 64, 1, 1, 2),
    ("l1.c2", 56, 64, 64, 3, 1, 3),
    ("l1.c3", 56, 64, 256, 1, 1, 4),  # 3 conv3 + the downsample (64 -> 256, stride 1)
    ("l2.c1a", 56, 256, 128, 1, 1, 1),
    ("l2.c2a", 56, 128, 128, 3, 2, 1),
    ("l2.ds", 56, 256, 512, 1, 2, 1),
    ("l2.c1", 28, 512, 128, 1, 1, 3),
    ("l2.c2", 28, 128, 128, 3, 1, 3),
    ("l2.c3", 28, 128, 512, 1, 1, 4),
    ("l3.c1a", 28, 512, 256, 1, 1, 1),
    ("l3.c2a", 28, 256, 256, 3, 2, 1),
    ("l3.ds", 28, 512, 1024, 1, 2, 1),
    ("l3.c1", 14, 1024, 256, 1, 1, 5),
    ("l3.c2", 14, 256, 256, 3, 1, 5),
    ("l3.c3", 14, 256, 1024, 1, 1, 6),
    ("l4.c1a", 14, 1024, 512, 1, 1, 1),
    ("l4.c2a", 14, 512, 512, 3, 2, 1),
    ("l4.ds", 14, 1024, 2048, 1, 2, 1),
    ("l4.c1", 7, 2048, 512, 1, 1, 2),
    ("l4.c2", 7, 512, 512, 3, 1, 2),
    ("l4.c3", 7, 512, 2048, 1, 1, 3),
]


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
    ap.add_argument("--K", type=int, default=7)
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--nt-variants", default="", help="also time fwd / dgrad on these conv_nt_pl variants")
    ap.add_argument("--tn-variants", default="", help="also time the wgrad on these conv_tn_pl variants")
    args = ap.parse_args()
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip

    K, B, dev = args.K, args.B, "cuda"
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    flops_tot = 0.0
    for name, H, Ci, Co, k, s, n in RESNET50:
        if args.only and name not in args.only.split(","):
            continue
        pad = k // 2
        OH = (H + 2 * pad - k) // s + 1
        x = torch.randn(K, B, H, H, Ci, device=dev)
        w = torch.randn(1, Co, k, k, Ci, device=dev) * 0.05
        dy = torch.randn(K, B, OH, OH, Co, device=dev)
        gw = torch.empty(K, Co, k, k, Ci, device=dev)
        nw = Co * k * k * Ci
        wpl = torch.empty((1, 2, nw), dtype=torch.bfloat16, device=dev)
        hip.split_rows(w.reshape(1, nw).contiguous(), wpl)
        ws = wpl[:, 0].unflatten(1, (Co, k, k, Ci))
        xp, dyp = hip.split_planes(x), hip.split_planes(dy)
        flops = 2.0 * K * B * OH * OH * Co * Ci * k * k
        t_f = timeit(lambda: hip.conv_fwd(x, w, s, pad, w_split=ws, x_planes=xp), args.iters)
        t_d = timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad, w_split=ws, dy_planes=dyp), args.iters)
        t_w = timeit(lambda: hip.conv_wgrad(dy, x, gw, s, pad, dy_planes=dyp, x_planes=xp), args.iters)
        nt = {}
        for v in [int(a) for a in args.nt_variants.split(",") if a]:
            hip._C.conv_nt_pl_set_variant(v)
            try:
                nt[v] = [round(timeit(lambda: hip.conv_fwd(x, w, s, pad, w_split=ws, x_planes=xp), args.iters) * 1e3, 3),
                         round(timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad, w_split=ws, dy_planes=dyp),
                                      args.iters) * 1e3, 3)]
            finally:
                hip._C.conv_nt_pl_set_variant(-1)
        tn = {}
        for v in [int(a) for a in args.tn_variants.split(",") if a]:
            hip._C.conv_tn_pl_set_variant(v)
            try:
                tn[v] = round(timeit(lambda: hip.conv_wgrad(dy, x, gw, s, pad, dy_planes=dyp, x_planes=xp),
                                     args.iters) * 1e3, 3)
            finally:
                hip._C.conv_tn_pl_set_variant(-1)
        for key, t in (("fwd", t_f), ("dgrad", t_d), ("wgrad", t_w)):
            tot[key] += t * n
        flops_tot += 3 * flops * n
        print(json.dumps({"layer": name, "H": H, "Ci": Ci, "Co": Co, "k": k, "s": s, "n": n,
                          "fwd_ms": round(t_f * 1e3, 3), "fwd_tflops": round(flops / t_f / 1e12, 1),
                          "dgrad_ms": round(t_d * 1e3, 3), "dgrad_tflops": round(flops / t_d / 1e12, 1),
                          "wgrad_ms": round(t_w * 1e3, 3), "wgrad_tflops": round(flops / t_w / 1e12, 1),
                          "weighted_ms": round((t_f + t_d + t_w) * n * 1e3, 2),
                          **({"nt_variants_fwd_dgrad_ms": nt} if nt else {}),
                          **({"tn_variants_wgrad_ms": tn} if tn else {})}), flush=True)
        del x, w, dy, gw, wpl, xp, dyp
        torch.cuda.empty_cache()
    ms = sum(tot.values()) * 1e3
    print(json.dumps({"summary": "resnet50 convs per wave", "K": K, "B": B,
                      **{f"{k2}_ms": round(v * 1e3, 2) for k2, v in tot.items()},
                      "conv_ms": round(ms, 2), "tflops": round(flops_tot / max(ms, 1e-9) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
