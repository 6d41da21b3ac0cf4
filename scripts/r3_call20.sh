#!/bin/bash
# GPU-vs-CPU parameter and loss differences of the ResNet-18 / LeNet / DenseNet session tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
DLS_PRINT_TOL=1 timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_sessions.py -k "resnet18_matches_cpu or lenet5 or densenet40" > gpurun_out/k20_tol.log 2>&1 || { tail -20 gpurun_out/k20_tol.log; exit 1; }
grep -E "TOL|passed|failed" gpurun_out/k20_tol.log
