#!/bin/bash
# GPU-box: full GPU test suite, headline bench, 8-rank per-rank share, sign-SGD bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/check3_tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/check3_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --emulate-world 8 --steps 4 --warmup 1 > gpurun_out/check3_emu8.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload signsgd_resnet50 --steps 2 --warmup 1 > gpurun_out/check3_signsgd.log 2>&1 || exit $?
