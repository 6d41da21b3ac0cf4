#!/bin/bash
# block outputs written in the forms their readers need (planes only before a downsample block,
# fp32 only before the head): ResNet tests, alternating A/B on the headline round, eval bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_gpu_sessions.py -k "resnet18 or sign_sgd or gtg" tests/test_multirank_gpu.py || exit 1
grep -E "passed|failed" gpurun_out/quick_tests.log | tail -1
bash scripts/ab_env.sh DLS_BLOCK_OUT_PLANES "1 0" --steps 3 --warmup 1 || exit 1
for v in 1 0; do
  DLS_BLOCK_OUT_PLANES=$v timeout -k 10 300 python -u bench/eval_bench.py --M 32 --iters 2 > gpurun_out/k17_eval$v.log 2>&1 || { tail -5 gpurun_out/k17_eval$v.log; exit 1; }
  echo "eval out_planes=$v $(grep '^{' gpurun_out/k17_eval$v.log | tail -1 | cut -c1-200)"
done
