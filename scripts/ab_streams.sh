#!/bin/bash
# A/B of sub-cohort streams x small-cohort tile rules on rank 0's share of an 8-rank round
# (bench.py --emulate-world 8): ms per round for each (DLS_STREAMS, DLS_F32_SMALLK) pair
#   scripts/ab_streams.sh "STREAMS..." "RULES..."
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
for st in ${1:-3 2 1}; do for rules in ${2:-3 0}; do
  DLS_STREAMS=$st DLS_F32_SMALLK=$rules timeout -k 10 200 python -u bench.py --emulate-world 8 --steps 4 --warmup 1 \
    > gpurun_out/ab_s${st}_r${rules}.log 2>&1 || exit 1
  echo "streams $st rules $rules $(grep '^{' gpurun_out/ab_s${st}_r${rules}.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
