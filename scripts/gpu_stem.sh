#!/bin/bash
# GPU-box: stem (8-channel) and l1 conv timings at the 8-rank per-rank cohort and at 100 clients.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 13 100; do
  timeout -k 10 300 python bench/kernel_bench.py --K $k --only l1,l2a,l2sc --skip-misc --sweep > gpurun_out/sweep_k$k.log 2>&1 || exit $?
done
