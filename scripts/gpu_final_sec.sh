#!/bin/bash
# Final-tree measurements of every BASELINE workload, >= 3 timed rounds each (each its own time
# limit; stop at a failure). PART=a: headline, 8-rank share, DenseNet-40, sign-SGD DenseNet-40,
# GTG utility evaluation; PART=b: sign-SGD ResNet-50, FedOBD Transformer-base (stage 1 + stage 2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
run() {  # name, limit, args...
  local n=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py "$@" > gpurun_out/fin_$n.log 2>&1 || { echo "$n failed"; tail -8 gpurun_out/fin_$n.log; exit 1; }
  grep '^{' gpurun_out/fin_$n.log | tail -1 > gpurun_out/fin_$n.json
  echo "$n $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["ms_per_step"],1), "ms/step", round(d["value"],5), d.get("unit"), d.get("stage2", ""))' gpurun_out/fin_$n.json)"
}
if [ "${PART:-a}" = a ]; then
  run headline 300 --steps 10 --warmup 3
  run emu8 200 --emulate-world 8 --steps 6 --warmup 2
  run densenet40 300 --workload fedavg_densenet40 --steps 3 --warmup 1
  run signsgd_densenet40 300 --workload signsgd_densenet40 --steps 3 --warmup 1
  timeout -k 10 200 python -u bench/eval_bench.py > gpurun_out/fin_eval.log 2>&1 || { tail -5 gpurun_out/fin_eval.log; exit 1; }
  tail -1 gpurun_out/fin_eval.log
else
  # (two warmup rounds: the caching allocator frees its cache and retries once in each of the
  # first two rounds at 243 GB peak, then holds — bench.py reports the retry count)
  run signsgd_resnet50 500 --workload signsgd_resnet50 --steps 3 --warmup 2
  run fedobd_transformer 600 --workload fedobd_transformer --steps 3 --warmup 1
fi
