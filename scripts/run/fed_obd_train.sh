#!/bin/bash
# Paper-scale FedOBD runs (counterpart of the reference's fed_obd_train.sh): CIFAR-10/100 and
# IMDB, 100 clients, one rank per GPU. NGPU defaults to every visible GPU.
set -e
cd "$(dirname "$0")/../.."
NGPU=${NGPU:-$(python3 -c "import torch; print(max(torch.cuda.device_count(), 1))")}
RUN="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $NGPU --master-addr 127.0.0.1 simulator.py"
for c in large_scale/fed_obd/cifar10.yaml large_scale/fed_obd/cifar100.yaml large_scale/fed_obd/imdb.yaml; do
  $RUN --config-name "$c"
done
