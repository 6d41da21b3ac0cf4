#!/bin/bash
# A/B of the pre-split weight planes (DLS_WSPLIT) on the headline round, alternating on one box
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
for i in 1 2; do for ws in 1 0; do  # DLS_WSPLIT=1: planes on
  DLS_WSPLIT=$ws timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 > gpurun_out/abws_${ws}_$i.log 2>&1 || exit 1
  echo "wsplit $ws run $i $(grep '^{' gpurun_out/abws_${ws}_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
