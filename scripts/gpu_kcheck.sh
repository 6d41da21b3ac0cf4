#!/bin/bash
# GPU-box: kernel numerics then the per-kernel microbenchmark. Stops on crash/timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x > gpurun_out/kern.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/kern.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench/kernel_bench.py ${KB_ARGS:-} > gpurun_out/kbench.log 2>&1
echo "rc=$?" >> gpurun_out/kbench.log
