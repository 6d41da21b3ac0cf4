#!/bin/bash
# GPU-box: kernel stats + INFO log (GTG iteration / evaluation counts) of one GTG bench round.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export DLS_LOG_LEVEL=INFO
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gtgprof -o run -- \
  python bench.py --workload gtg_resnet18 --steps 1 --warmup 1 > gpurun_out/gtgprof.log 2>&1
rc=$?
rm -f gpurun_out/gtgprof/run_kernel_trace.csv
exit $rc
