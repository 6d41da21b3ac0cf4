#!/bin/bash
# Round-6 GPU check: the tests named in $1 (pytest -k expression over the GPU files), then an
# alternating A/B of one option on the headline bench ($2 = VAR, $3 = "values", rest: bench args)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
k=$1; var=$2; vals=$3; shift 3
if [ -n "$k" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_kernels_f32_gpu.py \
    tests/test_gpu_sessions.py tests/test_concurrent.py -m gpu -k "$k" > gpurun_out/r6_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/r6_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$var" ]; then
  bash scripts/ab_env.sh "$var" "$vals" "$@" | tee gpurun_out/r6_ab.txt
fi
