#!/bin/bash
# GPU-box: rocprofv3 kernel stats of one bench round per workload (trace CSVs dropped: size cap).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WORKLOADS:-fedobd_transformer signsgd_resnet50 gtg_resnet18}; do
  timeout -k 10 ${WL_TIMEOUT:-500} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wlprof_$w -o run -- \
    python bench.py --workload $w --steps 1 --warmup 1 > gpurun_out/wlprof_$w.log 2>&1
  rc=$?
  rm -f gpurun_out/wlprof_$w/run_kernel_trace.csv
  echo "rc=$rc" >> gpurun_out/wlprof_$w.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
