#!/bin/bash
# GPU-box: graph-replay numerics test, then eager vs graph-replayed rounds at 13 and 100 clients.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py -x -v -m gpu -k "graph or resnet" --timeout 200 --timeout-method thread \
  > gpurun_out/graph_tests.log 2>&1 || exit $?
for n in 13 100; do
  for g in 0 1; do
    DLS_GRAPHS=$g timeout -k 10 400 python bench.py --clients $n --steps 2 --warmup 1 > gpurun_out/graphs_c${n}_g${g}.log 2>&1 || exit $?
  done
done
