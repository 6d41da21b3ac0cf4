#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --workload signsgd_resnet50 --steps 1 --warmup 1 --log-level INFO > gpurun_out/signsgd.log 2>&1
grep "memory plan\|session:" gpurun_out/signsgd.log | head -3
timeout -k 10 600 python -u bench.py --workload signsgd_resnet50 --steps 1 --warmup 1 --cohort 8 > gpurun_out/signsgd8.log 2>&1 || { tail -3 gpurun_out/signsgd8.log; exit 1; }
grep '^{' gpurun_out/signsgd8.log | tail -1 | tee gpurun_out/signsgd8.json
