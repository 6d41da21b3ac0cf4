#!/bin/bash
# GPU-box check: every gpu-marked test (kernel numerics + e2e sessions), smoke, short bench.
# Stops at the first crash/timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest ${TESTS:-tests/} -x -v -m gpu --timeout 240 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gputests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench1.log
exit $rc
