"""Per-kernel microbenchmark on the flagship shapes (ResNet-18 / CIFAR, cohort of K clients,
batch 64 per client): conv fwd / dgrad / wgrad, BN fwd / bwd, SGD — TFLOP/s or TB/s, plus the
same convolutions through PyTorch (MIOpen grouped conv) as a vendor-library reference.

    python bench/kernel_bench.py [--K 100] [--iters 10] [--torch]
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

# (name, H, Cin, Cout, k, stride)  (input spatial H = W)
RESNET18_CIFAR = [
    ("stem", 32, 3, 64, 3, 1),
    ("stem8", 32, 8, 64, 3, 1),  # the stem as the model runs it: images stored zero-padded to 8 channels
    ("l1", 32, 64, 64, 3, 1),
    ("l2a", 32, 64, 128, 3, 2),
    ("l2", 16, 128, 128, 3, 1),
    ("l2sc", 32, 64, 128, 1, 2),
    ("l3a", 16, 128, 256, 3, 2),
    ("l3", 8, 256, 256, 3, 1),
    ("l3sc", 16, 128, 256, 1, 2),
    ("l4a", 8, 256, 512, 3, 2),
    ("l4", 4, 512, 512, 3, 1),
    ("l4sc", 8, 256, 512, 1, 2),
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
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--sweep", action="store_true", help="time every conv_nt tile variant")
    ap.add_argument("--skip-misc", action="store_true", help="conv layers only (no BN/SGD)")
    ap.add_argument("--gl", action="store_true", help="A/B the LDS-DMA large-tile kernel (conv_gl) vs conv_nt")
    ap.add_argument("--f32", action="store_true", help="fp32 tensors: the split-bf16 kernels (csrc/conv_f32.hip)")
    ap.add_argument("--planes", action="store_true",
                    help="fp32: A/B the pre-split-operand LDS-DMA kernels (csrc/conv_pl.hip, every variant) "
                         "against the register-staged split kernels with pre-split weights")
    args = ap.parse_args()
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip, ref

    K, B = args.K, args.B
    dev = "cuda"
    dt = torch.float32 if args.f32 else torch.bfloat16
    nt_attr, tn_attr = ("nt_f32_variant", "tn_f32_variant") if args.f32 else ("nt_variant", "tn_variant")
    n_nt = hip._C.conv_nt_f32_num_variants() if args.f32 else hip._C.conv_nt_num_variants()
    n_tn = hip._C.conv_tn_f32_num_variants() if args.f32 else hip._C.conv_tn_num_variants()
    rows = []
    for name, H, Ci, Co, k, s in RESNET18_CIFAR:
        if args.only and name not in args.only.split(","):
            continue
        pad = k // 2
        OH = (H + 2 * pad - k) // s + 1
        x = torch.randn(K, B, H, H, Ci, device=dev).to(dt)
        w = (torch.randn(K, Co, k, k, Ci, device=dev) * 0.05).to(dt)
        dy = torch.randn(K, B, OH, OH, Co, device=dev).to(dt)
        gw = torch.empty(K, Co, k, k, Ci, device=dev)
        flops = 2.0 * K * B * OH * OH * Co * Ci * k * k
        t_f = timeit(lambda: hip.conv_fwd(x, w, s, pad), args.iters)
        t_d = timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad), args.iters)
        t_w = timeit(lambda: hip.conv_wgrad(dy, x, gw, s, pad), args.iters)
        row = {"layer": name, "H": H, "Ci": Ci, "Co": Co, "k": k, "s": s,
               "fwd_ms": t_f * 1e3, "fwd_tflops": flops / t_f / 1e12,
               "dgrad_ms": t_d * 1e3, "dgrad_tflops": flops / t_d / 1e12,
               "wgrad_ms": t_w * 1e3, "wgrad_tflops": flops / t_w / 1e12}
        if args.gl:
            # interleaved A/B in one process: conv_gl forced on vs forced off (TFLOP/s)
            ab = {"gl": [], "nt": []}
            for _ in range(3):
                for mode, key in ((1, "gl"), (0, "nt")):
                    hip.gl_mode = mode
                    tf_m = timeit(lambda: hip.conv_fwd(x, w, s, pad), args.iters)
                    td_m = timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad), args.iters)
                    ab[key].append((flops / tf_m / 1e12, flops / td_m / 1e12))
            hip.gl_mode = -1
            for key in ab:
                row[f"{key}_fwd_tflops"] = round(max(a for a, _ in ab[key]), 1)
                row[f"{key}_dgrad_tflops"] = round(max(b for _, b in ab[key]), 1)
        if args.f32 and k * k * Ci % 8 == 0 and Ci % 8 == 0:
            # interleaved A/B in one process: weights pre-split into (hi, lo) bf16 planes (what a
            # graphed training step reads, CohortBuffers.split) vs split per workgroup
            n = Co * k * k * Ci
            planes = torch.empty((K, 2, n), dtype=torch.bfloat16, device=dev)
            hip.split_rows(w.reshape(K, n).contiguous(), planes)
            ws = planes[:, 0].unflatten(1, (Co, k, k, Ci))
            ab = {"split": [], "plain": []}
            for _ in range(3):
                for key, wsp in (("split", ws), ("plain", None)):
                    tf_m = timeit(lambda: hip.conv_fwd(x, w, s, pad, w_split=wsp), args.iters)
                    td_m = timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad, w_split=wsp), args.iters)
                    ab[key].append((flops / tf_m / 1e12, flops / td_m / 1e12))
            for key in ab:
                row[f"{key}_fwd_tflops"] = round(max(a for a, _ in ab[key]), 1)
                row[f"{key}_dgrad_tflops"] = round(max(b for _, b in ab[key]), 1)
        if args.planes and Ci % 32 == 0:
            n = Co * k * k * Ci
            wpl = torch.empty((K, 2, n), dtype=torch.bfloat16, device=dev)
            hip.split_rows(w.reshape(K, n).contiguous(), wpl)
            ws = wpl[:, 0].unflatten(1, (Co, k, k, Ci))
            xp, dyp = hip.split_planes(x), hip.split_planes(dy)
            base_f = flops / timeit(lambda: hip.conv_fwd(x, w, s, pad, w_split=ws), args.iters) / 1e12
            base_d = flops / timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad, w_split=ws), args.iters) / 1e12
            if k == 3 and s == 1:  # 3x3 stride 1: the LDS-halo kernel (csrc/conv_halo.hip)
                hip._C.conv_halo_set_mode(1)
                hv = {}
                for v in range(3):
                    hip._C.conv_halo_set_variant(v)
                    tf_h = timeit(lambda: hip.conv_fwd(x, w, s, pad, w_split=ws, x_planes=xp), args.iters)
                    td_h = timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad, w_split=ws, dy_planes=dyp),
                                  args.iters)
                    hv[v] = (round(flops / tf_h / 1e12, 1), round(flops / td_h / 1e12, 1))
                hip._C.conv_halo_set_variant(-1)
                hip._C.conv_halo_set_mode(0)
                row["halo_fwd_dgrad"] = hv
            pv = {}
            for v in [-1] + list(range(hip._C.conv_nt_pl_num_variants())):
                hip._C.conv_nt_pl_set_variant(v)
                tf_v = timeit(lambda: hip.conv_fwd(x, w, s, pad, w_split=ws, x_planes=xp), args.iters)
                td_v = timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad, w_split=ws, dy_planes=dyp), args.iters)
                pv[v] = (round(flops / tf_v / 1e12, 1), round(flops / td_v / 1e12, 1))
            hip._C.conv_nt_pl_set_variant(-1)
            hip._C.conv_halo_set_mode(-1)
            row["split_w_fwd_dgrad"] = (round(base_f, 1), round(base_d, 1))
            row["planes_fwd_dgrad"] = pv
            pw = {}
            for v in [-1] + list(range(hip._C.conv_tn_pl_num_variants())):
                hip._C.conv_tn_pl_set_variant(v)
                tw_v = timeit(lambda: hip.conv_wgrad(dy, x, gw, s, pad, dy_planes=dyp, x_planes=xp), args.iters)
                pw[v] = round(flops / tw_v / 1e12, 1)
            hip._C.conv_tn_pl_set_variant(-1)
            row["planes_wgrad"] = pw
            del xp, dyp, wpl
        if args.sweep:
            # every NT tile configuration on this shape (fwd / dgrad TFLOP/s per variant id)
            sw = {}
            for v in range(n_nt):
                setattr(hip, nt_attr, v)
                tf_v = timeit(lambda: hip.conv_fwd(x, w, s, pad), args.iters)
                td_v = timeit(lambda: hip.conv_dgrad(dy, w, (H, H), s, pad), args.iters)
                sw[v] = (round(flops / tf_v / 1e12, 1), round(flops / td_v / 1e12, 1))
            setattr(hip, nt_attr, -1)
            row["sweep_fwd_dgrad"] = sw
            swt = {}
            for v in range(n_tn):
                setattr(hip, tn_attr, v)
                tw_v = timeit(lambda: hip.conv_wgrad(dy, x, gw, s, pad), args.iters)
                swt[v] = round(flops / tw_v / 1e12, 1)
            setattr(hip, tn_attr, -1)
            row["sweep_wgrad"] = swt
        if args.torch:
            tf = timeit(lambda: ref.conv_fwd(x, w, s, pad), max(2, args.iters // 4))
            row["torch_fwd_ms"] = tf * 1e3
            row["torch_fwd_tflops"] = flops / tf / 1e12
        rows.append(row)
        print(json.dumps({k2: (round(v, 3) if isinstance(v, float) else v) for k2, v in row.items()}), flush=True)
        del x, w, dy, gw
        torch.cuda.empty_cache()
    if args.skip_misc:
        return
    # BN + SGD
    R, C = B * 32 * 32, 64
    x = torch.randn(K, R, C, device=dev).to(dt)
    g = torch.ones(K, C, device=dev).to(dt)
    bb = torch.zeros(K, C, device=dev).to(dt)
    valid = torch.full((K,), R, dtype=torch.int32, device=dev)
    t = timeit(lambda: hip.bn_fwd(x, g, bb, valid, True, x), args.iters)
    nbytes = x.numel() * x.element_size() * 4  # stats read + apply read x,res + write
    print(json.dumps({"kernel": "bn_fwd_relu_res", "rows": R, "C": C, "ms": t * 1e3, "TB/s": nbytes / t / 1e12}))
    y, mean, rstd = hip.bn_fwd(x, g, bb, valid, True, None)
    gg = torch.zeros(K, C, device=dev)
    t = timeit(lambda: hip.bn_bwd(x, x, y, mean, rstd, g, valid, True, gg, gg, True), args.iters)
    nbytes = x.numel() * x.element_size() * 7
    print(json.dumps({"kernel": "bn_bwd_relu", "ms": t * 1e3, "TB/s": nbytes / t / 1e12}))
    del x, y
    P = 11173968
    th = torch.randn(K, P, device=dev)
    gr = torch.randn(K, P, device=dev)
    mo = torch.randn(K, P, device=dev)
    sh = th.to(torch.bfloat16)
    lr = torch.full((K,), 0.1, device=dev)
    act = torch.ones(K, dtype=torch.bool, device=dev)
    t = timeit(lambda: hip.sgd_step(th, gr, mo, lr, act, 0.0, 0.9, 0.0, False, act, sh), args.iters)
    print(json.dumps({"kernel": "sgd_step", "P": P, "ms": t * 1e3, "TB/s": K * P * 22 / t / 1e12}))
    w = torch.rand(K, device=dev)
    t = timeit(lambda: hip.weighted_sum(th, w), args.iters)
    print(json.dumps({"kernel": "weighted_sum", "ms": t * 1e3, "TB/s": K * P * 4 / t / 1e12}))


if __name__ == "__main__":
    main()
