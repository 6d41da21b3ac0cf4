#!/bin/bash
# GPU-box: kernel tests, rocprofv3 kernel stats of one bench round, torch-backend comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-1}
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/kern.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/kern.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench_prof.log 2>&1 || exit $?
if [ "${TORCH_CMP:-1}" = "1" ]; then
  timeout -k 10 900 python bench.py --steps 1 --warmup 1 --backend torch > gpurun_out/bench_torch.log 2>&1
  echo "torch rc=$?" >> gpurun_out/bench_torch.log
fi
exit 0
