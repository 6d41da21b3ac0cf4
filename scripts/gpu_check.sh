#!/bin/bash
# GPU-box check: kernel numerics, smoke, short bench. Stops at the first crash/timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/kern.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/kern.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --steps 2 --warmup 1 > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench1.log
exit $rc
