#!/bin/bash
# Stall breakdown of the ResNet-18 layer kernels in isolation (bench/kernel_bench.py --f32
# --planes, 50 clients): one PMC pass -> gpurun_out/pmc_stalls_kb.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmck
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d gpurun_out/pmck -o run -- python3 -u bench/kernel_bench.py --f32 --planes --K 50 --iters 3 --skip-misc \
  --only "${ONLY:-l1,l2,l3,l4}" > gpurun_out/pmck.log 2>&1 || { grep -v '^    @' gpurun_out/pmck.log | tail -5; exit 1; }
python3 scripts/pmc_agg.py gpurun_out/pmck > gpurun_out/pmc_stalls_kb_raw.txt
python3 scripts/pmc_stalls_table.py gpurun_out/pmc_stalls_kb_raw.txt > gpurun_out/pmc_stalls_kb.txt
rm -rf gpurun_out/pmck
head -40 gpurun_out/pmc_stalls_kb.txt
