#!/bin/bash
# GTG-Shapley contribution valuation (counterpart of the reference's gtg_shapley_train.sh).
set -e
cd "$(dirname "$0")/../.."
NGPU=${NGPU:-$(python3 -c "import torch; print(max(torch.cuda.device_count(), 1))")}
python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" --master-addr 127.0.0.1 simulator.py \
  --config-name gtg_sv/mnist.yaml "$@"
