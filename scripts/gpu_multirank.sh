#!/bin/bash
# GPU-box rehearsal of the multi-rank path on ONE GPU: 2 ranks share the card over gloo
# (RCCL needs a GPU per rank; the driver's 8-GPU run uses RCCL). Checks the N-rank bench JSON.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
DLS_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps ${STEPS:-1} --warmup 1 ${BENCH_ARGS:-} \
  > gpurun_out/multirank.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/multirank.log
exit $rc
