"""Plane-GEMM tiles at a rank's share of an 8-rank round (6-7 clients per sub-cohort launch): the
ResNet-18 l4 / strided / shortcut convs forward and dgrad on every conv_nt_pl variant — where the
default 128x128 tile leaves most CUs idle. Best of `--rounds`.

    python bench/small_cohort_bench.py [--K 7] [--iters 10]
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
SHAPES = [("l4", 4, 512, 512, 3, 1), ("l4a", 8, 256, 512, 3, 2), ("l3a", 16, 128, 256, 3, 2),
          ("l2a", 32, 64, 128, 3, 2), ("l4sc", 8, 256, 512, 1, 2), ("l3sc", 16, 128, 256, 1, 2)]


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
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip

    dev = torch.device("cuda:0")
    K, B = args.K, args.B
    nv = hip._C.conv_nt_pl_num_variants()
    for name, H, Ci, Co, k, s in SHAPES:
        pad = k // 2
        OH = (H + 2 * pad - k) // s + 1
        x = torch.randn(K, B, H, H, Ci, device=dev)
        w = torch.randn(K, Co, k, k, Ci, device=dev) * 0.05
        n = w[0].numel()
        planes = torch.empty((K, 2, n), dtype=torch.bfloat16, device=dev)
        hip.split_rows(w.reshape(K, n).contiguous(), planes)
        ws = planes[:, 0].view(w.shape)
        xp = hip.split_planes(x)
        dy = torch.randn(K, B, OH, OH, Co, device=dev)
        dyp = hip.split_planes(dy)
        flops = 2.0 * K * B * OH * OH * Co * k * k * Ci
        best = {}
        try:
            for _ in range(args.rounds):
                for v in [-1] + list(range(nv)):
                    hip._C.conv_nt_pl_set_variant(v)
                    for op, fn in (("fwd", lambda: hip.conv_fwd(x, w, s, pad, w_split=ws, x_planes=xp)),
                                   ("dgrad", lambda: hip.conv_dgrad(dy, w, (H, H), s, pad, w_split=ws, dy_planes=dyp))):
                        try:
                            t = timeit(fn, args.iters)
                        except Exception:
                            continue
                        best[(op, v)] = min(best.get((op, v), 1e9), t)
        finally:
            hip._C.conv_nt_pl_set_variant(-1)
        for op in ("fwd", "dgrad"):
            row = {"layer": name, "op": op, "K": K, "ms": {v: round(best[(op, v)] * 1e3, 4) for v in [-1] + list(range(nv))
                                                          if (op, v) in best}}
            row["tflops_default"] = round(flops / best[(op, -1)] / 1e12, 1)
            print(json.dumps(row), flush=True)
        del x, w, planes, xp, dy, dyp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
