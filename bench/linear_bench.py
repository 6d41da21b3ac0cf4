"""Client-batched linear (conv_nt GEMM) timings for the Transformer shapes (d_model 100,
ff 2048, 300 tokens × batch 64 per client): native kernel vs hipBLASLt bmm, and the effect of
an 8-aligned reduction width. Prints one JSON line per shape."""

from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip

    K, N = int(os.environ.get("LB_K", "33")), 64 * 300
    for Fi, Fo in [(100, 300), (100, 100), (100, 2048), (2048, 100), (104, 2048), (112, 2048), (128, 2048)]:
        x = torch.randn(K, N, Fi, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, Fo, Fi, device="cuda") * 0.05).to(torch.bfloat16)
        dy = torch.randn(K, N, Fo, device="cuda").to(torch.bfloat16)
        gw = torch.empty(K, Fo, Fi, device="cuda")
        fl = 2.0 * K * N * Fi * Fo
        t_f = timeit(lambda: hip.linear_fwd(x, w))
        t_d = timeit(lambda: hip.linear_dgrad(dy, w))
        t_w = timeit(lambda: hip.linear_wgrad(dy, x, gw))
        t_blas = timeit(lambda: torch.bmm(x, w.transpose(1, 2)))
        print(json.dumps({"K": K, "N": N, "Fi": Fi, "Fo": Fo, "fwd_ms": round(t_f, 3), "fwd_tflops": round(fl / t_f / 1e9, 1),
                          "dgrad_tflops": round(fl / t_d / 1e9, 1), "wgrad_tflops": round(fl / t_w / 1e9, 1),
                          "bmm_tflops": round(fl / t_blas / 1e9, 1)}), flush=True)
        del x, w, dy, gw


if __name__ == "__main__":
    main()
