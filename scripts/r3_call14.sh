#!/bin/bash
# GTG utility-evaluation kernel profile; sign-SGD ResNet-50 at full ImageNet-shaped shards
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_call12.sh || exit 1
timeout -k 10 700 python -u bench.py --workload signsgd_resnet50 --shard-scale 1.0 --steps 1 --warmup 0 --log-level INFO > gpurun_out/signsgd_full.log 2>&1 || { tail -10 gpurun_out/signsgd_full.log; exit 1; }
grep '^{' gpurun_out/signsgd_full.log | tail -1 | tee gpurun_out/signsgd_full.json | cut -c1-400
