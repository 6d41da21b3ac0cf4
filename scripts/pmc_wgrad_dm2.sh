#!/bin/bash
# l1 halo weight gradient with the BN backward in its dY loader (dy mode 2) against the plain
# plane modes and the separate bn_bwd_apply pass: timings, then one stall PMC pass
# -> gpurun_out/wg_dm2.log, gpurun_out/pmc_stalls_wg.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 -u bench/wgrad_bench.py --only l1 --unroll 1 > gpurun_out/wg_dm2.log 2>&1 || { tail -5 gpurun_out/wg_dm2.log; exit 1; }
grep '^{' gpurun_out/wg_dm2.log
rm -rf gpurun_out/pmcw
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d gpurun_out/pmcw -o run -- python3 -u bench/wgrad_bench.py --only l1 --unroll 1 --iters 3 \
  > gpurun_out/pmcw.log 2>&1 || { tail -5 gpurun_out/pmcw.log; exit 1; }
python3 scripts/pmc_agg.py gpurun_out/pmcw > gpurun_out/pmc_stalls_wg_raw.txt
python3 scripts/pmc_stalls_table.py gpurun_out/pmc_stalls_wg_raw.txt > gpurun_out/pmc_stalls_wg.txt
rm -rf gpurun_out/pmcw
head -20 gpurun_out/pmc_stalls_wg.txt
