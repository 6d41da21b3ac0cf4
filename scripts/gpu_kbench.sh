#!/bin/bash
# GPU-box: per-kernel microbenchmark (optionally with the MIOpen comparison)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench/kernel_bench.py ${KB_ARGS:---torch} > gpurun_out/kbench.log 2>&1
echo "rc=$?" >> gpurun_out/kbench.log
