#!/bin/bash
# full GPU suite, driver-shaped headline bench, kernel profile of the headline round
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_full.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_full.log; [ $rc -ne 0 ] && { grep -n "Error\|FAIL" gpurun_out/gpu_tests_full.log | head; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
bash scripts/gpu.sh bench --steps 20 --warmup 5 || exit 1
cp gpurun_out/bench.json gpurun_out/bench_driver_shape.json
bash scripts/gpu.sh prof --steps 3 --warmup 1 || exit 1
