#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1140 python -u bench.py --workload gtg_resnet18 --steps 1 --warmup 0 --log-level INFO > gpurun_out/gtg.log 2>&1
rc=$?
grep '^{' gpurun_out/gtg.log | tail -1 | tee gpurun_out/gtg.json
exit $rc
