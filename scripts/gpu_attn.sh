#!/bin/bash
# GPU-box: attention numerics, then the FedOBD Transformer bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -x -v -m gpu -k "attention or transformer or linear" --timeout 200 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload fedobd_transformer --steps 2 --warmup 1 > gpurun_out/attn_fedobd.log 2>&1 || exit $?
