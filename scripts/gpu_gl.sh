#!/bin/bash
# GPU-box: conv_gl numerics, then the conv_gl vs conv_nt A/B on the ResNet-18 layer shapes
# (K=100 and K=13 clients), then a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "conv" --timeout 120 --timeout-method thread \
  > gpurun_out/gl_tests.log 2>&1 || exit $?
timeout -k 10 400 python bench/kernel_bench.py --K 100 --iters 5 --gl --skip-misc > gpurun_out/gl_kbench100.log 2>&1 || exit $?
timeout -k 10 300 python bench/kernel_bench.py --K 13 --iters 10 --gl --skip-misc > gpurun_out/gl_kbench13.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/gl_bench.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/gl_bench.log
exit $rc
