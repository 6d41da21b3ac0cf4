#!/bin/bash
# GPU-box: kernel stats of rank 0's share of the 8-rank FedAvg round (emulated on one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/emuprof -o run -- \
  python bench.py --emulate-world 8 --steps 3 --warmup 1 > gpurun_out/emuprof.log 2>&1
rc=$?
rm -f gpurun_out/emuprof/run_kernel_trace.csv
exit $rc
