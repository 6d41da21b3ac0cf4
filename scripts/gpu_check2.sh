#!/bin/bash
# GPU-box: full GPU test suite, then the headline bench and rank 0's share of the 8-rank round.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/check2_tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/check2_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --emulate-world 8 --steps 3 --warmup 1 > gpurun_out/check2_emu8.log 2>&1 || exit $?
