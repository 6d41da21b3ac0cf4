#!/bin/bash
# GPU-box: list counters, then PMC counters of the conv kernels on two ResNet-18 layers.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
PMC=${PMC:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES"}
timeout -k 10 600 rocprofv3 --kernel-trace --pmc $PMC --output-format csv -d gpurun_out/pmc -o pmc -- \
  python bench/kernel_bench.py --only ${LAYERS:-l1,l3} --skip-misc --iters 2 --K 100 > gpurun_out/pmc.log 2>&1
echo "rc=$?" >> gpurun_out/pmc.log
