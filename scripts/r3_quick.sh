#!/bin/bash
# targeted GPU tests (pass test ids as arguments)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -30 gpurun_out/quick_tests.log
exit $rc
