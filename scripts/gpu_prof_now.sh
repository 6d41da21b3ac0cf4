#!/bin/bash
# GPU-box: current headline bench + rocprofv3 kernel stats of the 100-client FedAvg round and of the
# emulated rank-0 share of an 8-rank round.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/now
export TMPDIR=/tmp
O=gpurun_out/now
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > $O/bench_fedavg.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof100 -o run -- \
  python bench.py --steps 1 --warmup 1 > $O/prof100.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profemu8 -o run -- \
  python bench.py --emulate-world 8 --steps 2 --warmup 1 > $O/profemu8.log 2>&1 || exit $?
