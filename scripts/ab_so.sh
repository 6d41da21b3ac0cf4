#!/bin/bash
# alternating runs of bench.py ARGS on two extension builds: ab_attn/{old,new} each hold one changed
# csrc file ($AB_SRC), the .so and its source stamp, swapped in together -> one line per run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
SO=distributed_learning_simulator_amd/_dls_hip.cpython-310-x86_64-linux-gnu.so
use() { cp ab_attn/$1/$AB_SRC csrc/ && cp ab_attn/$1/$(basename $SO) $SO && cp ab_attn/$1/$(basename $SO).srchash $SO.srchash; }
for r in 1 2; do
  for v in old new; do
    use $v
    timeout -k 10 400 python -u bench.py "$@" > gpurun_out/abso.log 2>&1 || { tail -5 gpurun_out/abso.log; exit 1; }
    echo "$v $* $(grep '^{' gpurun_out/abso.log | tail -1 | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"],1))')"
  done
done
use new
