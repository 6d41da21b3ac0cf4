#!/bin/bash
# Stall breakdown per kernel of bench.py ARGS (one PMC pass): wave cycles parked at s_waitcnt /
# barriers (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY, LDS part SQ_WAIT_INST_LDS), issuing
# (SQ_ACTIVE_INST_ANY), MFMA-busy cycles -> gpurun_out/pmc_stalls.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
# (eager, one stream: counters per dispatch without graph replay — PMC under graph replay crashed)
export DLS_GRAPHS=0 DLS_STREAMS=1
mkdir -p gpurun_out
rm -rf gpurun_out/pmcs
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d gpurun_out/pmcs -o run -- python3 -u bench.py "$@" > gpurun_out/pmcs.log 2>&1 || { tail -5 gpurun_out/pmcs.log; exit 1; }
python3 scripts/pmc_agg.py gpurun_out/pmcs > gpurun_out/pmc_stalls_raw.txt
python3 scripts/pmc_stalls_table.py gpurun_out/pmc_stalls_raw.txt > gpurun_out/pmc_stalls.txt
rm -rf gpurun_out/pmcs
head -30 gpurun_out/pmc_stalls.txt
