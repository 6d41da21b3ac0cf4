"""Transformer-base linears (d 512, FFN 2048, batch 64 × seq 128 per client) on the split-plane
GEMMs (csrc/conv_pl.hip): forward (x planes × weight planes), dgrad (dY planes × k-major weight
planes) and weight gradient (dY planes × X planes), per tile variant — ms per launch and TFLOP/s
of useful fp32 work (2·M·N·K).

    python bench/linear_bench.py [--K 25] [--rows 8192] [--iters 10] [--sweep]
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

SHAPES = [("in_proj", 512, 1536), ("out_proj", 512, 512), ("linear1", 512, 2048), ("linear2", 2048, 512)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def _wsplit(hip, w):
    K = w.shape[0]
    ws = torch.empty((K, 2, w[0].numel()), dtype=torch.bfloat16, device=w.device)
    hip.split_rows(w.reshape(K, -1).contiguous(), ws)
    return ws[:, 0].view(w.shape)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=25)
    ap.add_argument("--rows", type=int, default=64 * 128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--sweep", action="store_true", help="every conv_nt_pl / conv_tn_pl variant")
    ap.add_argument("--only", default="")
    ap.add_argument("--f32-variants", default="", help="fp32-operand paths (register-staged split): conv_nt_f32 variants")
    ap.add_argument("--tn-f32-variants", default="", help="fp32-operand weight gradient: conv_tn_f32 variants")
    args = ap.parse_args()
    from distributed_learning_simulator_amd.ops import hip

    K, N = args.K, args.rows
    C = hip._C
    for name, Fi, Fo in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        x = torch.randn(K, N, Fi, device="cuda")
        w = torch.randn(K, Fo, Fi, device="cuda") * 0.05
        b = torch.randn(K, Fo, device="cuda")
        dy = torch.randn(K, N, Fo, device="cuda")
        ws = _wsplit(hip, w)
        xp, dyp = hip.split_planes(x), hip.split_planes(dy)
        gw, gb = torch.empty(K, Fo, Fi, device="cuda"), torch.empty(K, Fo, device="cuda")
        flop = 2.0 * K * N * Fi * Fo
        nt = [-1] + (list(range(C.conv_nt_pl_num_variants())) if args.sweep else [])
        tn = [-1] + (list(range(C.conv_tn_pl_num_variants())) if args.sweep else [])
        for v in nt:
            C.conv_nt_pl_set_variant(v)
            for op, fn in (("fwd", lambda: hip.linear_fwd(x, w, b, w_split=ws, x_planes=xp)),
                           ("dgrad", lambda: hip.linear_dgrad(dy, w, w_split=ws, dy_planes=dyp))):
                try:
                    t = timeit(fn, args.iters)
                except Exception as e:  # (a variant whose LDS does not fit)
                    print(json.dumps({"layer": name, "op": op, "variant": v, "error": str(e)[:80]}), flush=True)
                    continue
                print(json.dumps({"layer": name, "op": op, "variant": v, "K": K, "rows": N, "ms": round(t * 1e3, 4),
                                  "tflops": round(flop / t / 1e12, 1)}), flush=True)
        C.conv_nt_pl_set_variant(-1)
        for v in tn:
            C.conv_tn_pl_set_variant(v)
            t = timeit(lambda: hip.linear_wgrad(dy, x, gw, None, dy_planes=dyp, x_planes=xp), args.iters)
            print(json.dumps({"layer": name, "op": "wgrad", "variant": v, "K": K, "rows": N, "ms": round(t * 1e3, 4),
                              "tflops": round(flop / t / 1e12, 1)}), flush=True)
        C.conv_tn_pl_set_variant(-1)
        t = timeit(lambda: hip.linear_fwd(x, w, b), args.iters)
        print(json.dumps({"layer": name, "op": "fwd_f32_split_in_loader", "K": K, "ms": round(t * 1e3, 4),
                          "tflops": round(flop / t / 1e12, 1)}), flush=True)
        # the Transformer's fp32-operand users (attention output into out_proj, dqkv into in_proj):
        # x / dY fp32 split in the loader, the weight from its planes
        for v in [int(a) for a in args.f32_variants.split(",") if a]:
            hip.nt_f32_variant = v
            try:
                for op, fn in (("fwd_f32", lambda: hip.linear_fwd(x, w, b, w_split=ws)),
                               ("dgrad_f32", lambda: hip.linear_dgrad(dy, w, w_split=ws))):
                    t = timeit(fn, args.iters)
                    print(json.dumps({"layer": name, "op": op, "nt_f32_variant": v, "ms": round(t * 1e3, 4),
                                      "tflops": round(flop / t / 1e12, 1)}), flush=True)
            finally:
                hip.nt_f32_variant = -1
        for v in [int(a) for a in args.tn_f32_variants.split(",") if a]:
            hip.tn_f32_variant = v
            try:
                t = timeit(lambda: hip.linear_wgrad(dy, x, gw, None), args.iters)
                print(json.dumps({"layer": name, "op": "wgrad_f32", "tn_f32_variant": v, "ms": round(t * 1e3, 4),
                                  "tflops": round(flop / t / 1e12, 1)}), flush=True)
            finally:
                hip.tn_f32_variant = -1
        del x, w, dy, xp, dyp, gw, gb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
