#!/bin/bash
# GPU-box: one short bench.py run per BASELINE workload (each under its own time limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WORKLOADS:-fedobd_transformer gtg_resnet18 signsgd_resnet50}; do
  timeout -k 10 ${WL_TIMEOUT:-400} python bench.py --workload $w --steps ${STEPS:-1} --warmup 1 > gpurun_out/wl_$w.log 2>&1
  rc=$?
  echo "rc=$rc" >> gpurun_out/wl_$w.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
