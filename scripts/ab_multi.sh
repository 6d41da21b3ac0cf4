#!/bin/bash
# Alternating A/B of several environment settings on one bench workload (same box), twice each:
#   scripts/ab_multi.sh "A=1 B=0" "A=0" ... -- [bench.py args]   -> ms per round per setting
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
sets=()
while [ "$1" != "--" ] && [ $# -gt 0 ]; do sets+=("$1"); shift; done
shift
for i in 1 2; do
  j=0
  for st in "${sets[@]}"; do
    j=$((j+1))
    env $st timeout -k 10 400 python -u ${BENCH_SCRIPT:-bench.py} "$@" > "gpurun_out/abm_${j}_$i.log" 2>&1 || { tail -5 "gpurun_out/abm_${j}_$i.log"; exit 1; }
    echo "[$st] run $i $(grep '^{' "gpurun_out/abm_${j}_$i.log" | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],1))')"
  done
done
