#!/bin/bash
# Secondary BASELINE workloads, one bench.py run each (own time limit, stop at the first failure):
#   scripts/bench_all.sh [WORKLOAD...]  -> gpurun_out/bench_<workload>.json
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
for wl in ${@:-gtg_resnet18 fedobd_transformer signsgd_resnet50 fedavg_densenet40}; do
  case "$wl" in
    gtg_resnet18) args="--steps 1 --warmup 1 --log-level INFO" ;;
    fedobd_transformer) args="--steps 2 --warmup 1 --no-stage2" ;;
    signsgd_resnet50) args="--steps 1 --warmup 1" ;;
    *) args="--steps 1 --warmup 1" ;;
  esac
  timeout -k 10 600 python -u bench.py --workload "$wl" $args > "gpurun_out/bench_$wl.log" 2>&1 || {
    echo "$wl failed"; tail -5 "gpurun_out/bench_$wl.log"; exit 1; }
  grep '^{' "gpurun_out/bench_$wl.log" | tail -1 > "gpurun_out/bench_$wl.json"
  cut -c1-300 "gpurun_out/bench_$wl.json"
done
