#!/bin/bash
# round-3 GPU batch: tests, evaluation microbench A/B, headline kernel profile, PMC counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu.sh tests || exit 1
timeout -k 10 300 python -u bench/eval_bench.py --M 32 --iters 3 > gpurun_out/eval_planes.log 2>&1 || { tail -20 gpurun_out/eval_planes.log; exit 1; }
timeout -k 10 300 python -u bench/eval_bench.py --M 32 --iters 3 --no-planes > gpurun_out/eval_noplanes.log 2>&1 || { tail -20 gpurun_out/eval_noplanes.log; exit 1; }
grep '^{' gpurun_out/eval_planes.log gpurun_out/eval_noplanes.log
bash scripts/gpu.sh prof --steps 2 --warmup 1 || exit 1
bash scripts/gpu.sh pmcset --steps 1 --warmup 1 || exit 1
timeout -k 10 600 python -u bench.py --workload fedobd_transformer --steps 1 --warmup 1 > gpurun_out/fedobd_tb.log 2>&1 || { tail -20 gpurun_out/fedobd_tb.log; exit 1; }
grep '^{' gpurun_out/fedobd_tb.log | tail -1 > gpurun_out/fedobd_tb.json
