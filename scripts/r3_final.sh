#!/bin/bash
# final-tree evidence: GPU suite, smoke, driver-shaped headline, kernel profile, PMC summary,
# emulated 8-rank share, secondary workloads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/final_gpu_tests.log; [ $rc -ne 0 ] && { grep -n "Error\|FAIL" gpurun_out/final_gpu_tests.log | head; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
bash scripts/gpu.sh bench --steps 20 --warmup 5 > /dev/null || exit 1
cp gpurun_out/bench.json gpurun_out/final_bench.json; cut -c1-200 gpurun_out/final_bench.json
bash scripts/gpu.sh prof --steps 3 --warmup 1 > /dev/null || exit 1
cp gpurun_out/prof_kernel_stats.csv gpurun_out/final_kernel_stats.csv
bash scripts/gpu.sh pmcset --steps 1 --warmup 1 > /dev/null || exit 1
cp gpurun_out/pmc_summary.csv gpurun_out/final_pmc_summary.csv
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --emulate-world 8 > gpurun_out/final_emu8.log 2>&1 || { tail -5 gpurun_out/final_emu8.log; exit 1; }
grep '^{' gpurun_out/final_emu8.log | tail -1 > gpurun_out/final_emu8.json; cut -c1-200 gpurun_out/final_emu8.json
timeout -k 10 400 python -u bench.py --workload fedavg_densenet40 --steps 1 --warmup 1 > gpurun_out/final_dense.log 2>&1 || { tail -5 gpurun_out/final_dense.log; exit 1; }
grep '^{' gpurun_out/final_dense.log | tail -1 > gpurun_out/final_dense.json; cut -c1-200 gpurun_out/final_dense.json
timeout -k 10 500 python -u bench.py --workload fedobd_transformer --steps 1 --warmup 1 > gpurun_out/final_tfm.log 2>&1 || { tail -5 gpurun_out/final_tfm.log; exit 1; }
grep '^{' gpurun_out/final_tfm.log | tail -1 > gpurun_out/final_tfm.json; cut -c1-200 gpurun_out/final_tfm.json
