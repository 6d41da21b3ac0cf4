#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_kernels_f32_gpu.py -k "halo or planes or pl" || exit 1
timeout -k 10 600 python -u bench/kernel_bench.py --f32 --planes --K 50 --skip-misc --iters 5 --only l1,l2,l3,l4 > gpurun_out/kbench_halo.log 2>&1 || { tail -20 gpurun_out/kbench_halo.log; exit 1; }
timeout -k 10 300 python -u bench/eval_bench.py --M 32 --iters 3 > gpurun_out/eval_planes.log 2>&1 || { tail -20 gpurun_out/eval_planes.log; exit 1; }
bash scripts/gpu.sh bench --steps 3 --warmup 1 || exit 1
grep '^{' gpurun_out/eval_planes.log
