"""A/B of the pixel-major tap-skipping GEMMs (csrc/conv_pl.hip PIX, native option conv_pix) on the
small-image convolutions they serve: ResNet-18 l4 (3x3, 4x4, 512 channels) and the strided l4a / l3a
forwards, at a training cohort (K clients x 64 images, default tiles, planes operands) and at 8192
images per client (forward only: one-pixel tiles; the GTG utility itself launches 64-image test
batches as virtual clients, i.e. the training shapes). Interleaved rounds in one process,
best of `--rounds`; TFLOP/s count every tap (the padded ones too), as bench/kernel_bench.py does.

    python bench/pix_bench.py [--K 50] [--iters 10] [--rounds 3]
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

# (name, K, B, H, Ci, Co, stride, passes)
SHAPES = [
    ("l4", None, 64, 4, 512, 512, 1, "fdw"),
    ("l4a", None, 64, 8, 256, 512, 2, "fw"),
    ("l3a", None, 64, 16, 128, 256, 2, "fw"),
    ("l4_small_cohort", 7, 64, 4, 512, 512, 1, "fdw"),
    ("l4_eval", 4, 8192, 4, 512, 512, 1, "f"),
    ("l4a_eval", 4, 8192, 8, 256, 512, 2, "f"),
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
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for name, K, B, H, Ci, Co, s, passes in SHAPES:
        K = K or args.K
        OH = (H + 2 - 3) // s + 1
        x = torch.randn(K, B, H, H, Ci, device=dev)
        w = torch.randn(K, Co, 3, 3, Ci, device=dev) * 0.05
        n = w[0].numel()
        planes = torch.empty((K, 2, n), dtype=torch.bfloat16, device=dev)
        hip.split_rows(w.reshape(K, n).contiguous(), planes)
        ws = planes[:, 0].view(w.shape)
        xp = hip.split_planes(x)
        dy = torch.randn(K, B, OH, OH, Co, device=dev)
        dyp = hip.split_planes(dy)
        acc = torch.randn_like(x) if "d" in passes else None
        gw = torch.empty_like(w)
        M = B * OH * OH
        st = torch.empty((K, hip.conv_stats_parts(M), 2, Co), device=dev)
        valid = torch.full((K,), B, dtype=torch.int32, device=dev)
        flops = 2.0 * K * M * Co * 9 * Ci
        fns = {
            "f": lambda: hip.conv_fwd(x, w, s, 1, w_split=ws, x_planes=xp, stats=st, stats_valid=valid),
            "d": lambda: hip.conv_dgrad(dy, w, (H, H), s, 1, acc=acc, w_split=ws, dy_planes=dyp),
            "w": lambda: hip.conv_wgrad(dy, x, gw, s, 1, dy_planes=dyp, x_planes=xp),
        }
        best = {}
        for _ in range(args.rounds):
            for pix in (0, 1):
                hip._C.set_native_option("conv_pix", pix)
                for ps in passes:
                    t = timeit(fns[ps], args.iters)
                    best[(ps, pix)] = min(best.get((ps, pix), 1e9), t)
        hip._C.set_native_option("conv_pix", 1)
        row = {"layer": name, "K": K, "B": B, "H": H, "Ci": Ci, "Co": Co, "stride": s}
        for ps in passes:
            key = {"f": "fwd", "d": "dgrad", "w": "wgrad"}[ps]
            t0, t1 = best[(ps, 0)], best[(ps, 1)]
            row[key] = {"ms_off": round(t0 * 1e3, 3), "ms_pix": round(t1 * 1e3, 3),
                        "tflops_off": round(flops / t0 / 1e12, 1), "tflops_pix": round(flops / t1 / 1e12, 1),
                        "speedup": round(t0 / t1, 3)}
        print(json.dumps(row), flush=True)
        del x, w, planes, xp, dy, dyp, acc, gw, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
