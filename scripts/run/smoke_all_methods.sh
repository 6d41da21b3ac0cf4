#!/bin/bash
# One-round smoke run of every method family through the CLI (counterpart of the reference's
# test.sh / other_method_test.sh). Runs on the GPU when one is visible, else on the CPU.
# Multi-GPU: prefix each line with `python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1`.
set -e
cd "$(dirname "$0")/../.."
S="python3 ./simulator.py"
# CV
$S --config-name fed_avg/mnist.yaml ++fed_avg.round=1 ++fed_avg.epoch=1 ++fed_avg.worker_number=2 ++fed_avg.debug=True
# NLP
$S --config-name fed_avg/imdb.yaml ++fed_avg.round=1 ++fed_avg.epoch=1 ++fed_avg.worker_number=2 ++fed_avg.dataset_kwargs.scale=0.02
# Graph
$S --config-name fed_gnn/cs.yaml ++fed_gnn.round=1 ++fed_gnn.epoch=1 ++fed_gnn.worker_number=2
# GTG-Shapley
$S --config-name gtg_sv/mnist.yaml ++gtg_sv.round=1 ++gtg_sv.epoch=1 ++gtg_sv.worker_number=2
# FedOBD (two-phase, NNADQ)
$S --config-name fed_obd/cifar10.yaml ++fed_obd.round=1 ++fed_obd.epoch=1 ++fed_obd.worker_number=10 \
   ++fed_obd.algorithm_kwargs.random_client_number=10 ++fed_obd.algorithm_kwargs.second_phase_epoch=1
# FedDropoutAvg / FedPAQ with partial participation
$S --config-name fed_dropout_avg/cifar100.yaml ++fed_dropout_avg.round=1 ++fed_dropout_avg.epoch=1 \
   ++fed_dropout_avg.worker_number=2 ++fed_dropout_avg.algorithm_kwargs.random_client_number=2
$S --config-name fed_paq/cifar100.yaml ++fed_paq.round=1 ++fed_paq.epoch=1 ++fed_paq.worker_number=2 \
   ++fed_paq.algorithm_kwargs.random_client_number=2
# sign-SGD (1-bit majority vote)
$S --config-name sign_sgd/cifar10.yaml ++sign_sgd.round=1 ++sign_sgd.epoch=1 ++sign_sgd.worker_number=4
