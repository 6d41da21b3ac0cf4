#!/bin/bash
# GPU-box: subset-mixing kernel tests, GTG-Shapley bench round (lock-step GTG iterations + native
# subset mixing), and rank 0's share of the 8-rank FedAvg round emulated on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -x -v -m gpu \
  -k "mix_rows or sgd_and_fl or graph" --timeout 200 --timeout-method thread > gpurun_out/gtg_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload gtg_resnet18 --steps 1 --warmup 1 > gpurun_out/gtg_bench.log 2>&1 || exit $?
for w in 8 4 2; do
  timeout -k 10 300 python bench.py --emulate-world $w --steps 3 --warmup 1 > gpurun_out/emu$w.log 2>&1 || exit $?
done
