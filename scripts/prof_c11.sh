#!/bin/bash
# Kernel stats of the headline round (one sub-cohort stream) and of the GTG utility evaluation on
# the current tree -> gpurun_out/p_{full,eval}_kernel_stats.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
prof() {  # name, program args...
  local n=$1; shift
  rm -rf gpurun_out/p_$n
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_$n -o run -- \
    python3 -u "$@" > gpurun_out/p_$n.log 2>&1 || { tail -5 gpurun_out/p_$n.log; return 1; }
  cp "$(find gpurun_out/p_$n -name '*kernel_stats.csv' | head -1)" gpurun_out/p_${n}_kernel_stats.csv
  rm -rf gpurun_out/p_$n
  grep '^{' gpurun_out/p_$n.log | tail -1 | cut -c1-200
}
DLS_STREAMS=1 prof full bench.py --steps 2 --warmup 1 &&
prof eval bench/eval_bench.py --iters 1 --rounds 1
