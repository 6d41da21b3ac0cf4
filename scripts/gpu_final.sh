#!/bin/bash
# GPU-box: full GPU suite + smoke, every BASELINE workload on one GPU, rank-0 shares of the 2/4/8-rank
# FedAvg round (emulated), and a 2-rank gloo rehearsal of the torchrun path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
export TMPDIR=/tmp
O=gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > $O/bench_fedavg.log 2>&1 || exit $?
for w in 2 4 8; do
  timeout -k 10 300 python bench.py --emulate-world $w --steps 4 --warmup 1 > $O/bench_emu$w.log 2>&1 || exit $?
done
for wl in signsgd_resnet50 fedobd_transformer gtg_resnet18; do
  timeout -k 10 600 python bench.py --workload $wl --steps 2 --warmup 1 > $O/bench_$wl.log 2>&1 || exit $?
done
DLS_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 > $O/multirank2.log 2>&1 || exit $?
