#!/bin/bash
# Alternating A/B of one environment switch on one bench workload (same box):
#   scripts/ab_env.sh VAR "VALUES" [bench.py args...]   -> ms per round for each value, twice
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
var=$1; vals=$2; shift 2
for i in 1 2; do for v in $vals; do
  env "$var=$v" timeout -k 10 400 python -u bench.py "$@" > "gpurun_out/ab_${var}_${v}_$i.log" 2>&1 || exit 1
  echo "$var=$v run $i $(grep '^{' "gpurun_out/ab_${var}_${v}_$i.log" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
