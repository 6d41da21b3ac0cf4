#!/bin/bash
# alternating runs of bench.py ARGS on several extension builds: ab_attn/<name>/ holds the csrc
# files that differ, the .so and its source stamp, swapped in together. AB_NAMES: build order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
SO=distributed_learning_simulator_amd/_dls_hip.cpython-310-x86_64-linux-gnu.so
use() {
  for f in ab_attn/$1/*.hip; do cp "$f" csrc/; done
  cp ab_attn/$1/$(basename $SO) $SO && cp ab_attn/$1/$(basename $SO).srchash $SO.srchash
}
for r in $(seq ${AB_ROUNDS:-2}); do
  for v in $AB_NAMES; do
    use $v
    timeout -k 10 400 python -u bench.py "$@" > gpurun_out/abso.log 2>&1 || { tail -5 gpurun_out/abso.log; exit 1; }
    echo "$v $(grep '^{' gpurun_out/abso.log | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_per_step"],1), round(d.get("ms_per_vote_step", 0), 1))')"
  done
done
use cur
