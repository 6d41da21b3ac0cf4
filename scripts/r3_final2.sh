#!/bin/bash
# final tree after the block-output / LayerNorm-plane changes: GPU suite, smoke, driver-shaped
# headline, kernel profile, emulated 8-rank share, Transformer-base FedOBD with stage 2, GTG eval
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/final2_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/final2_gpu_tests.log; [ $rc -ne 0 ] && { grep -n "Error\|FAIL" gpurun_out/final2_gpu_tests.log | head; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2_smoke.log 2>&1 || { tail -5 gpurun_out/final2_smoke.log; exit 1; }
bash scripts/gpu.sh bench --steps 20 --warmup 5 > /dev/null || exit 1
cp gpurun_out/bench.json gpurun_out/final2_bench.json; cut -c1-200 gpurun_out/final2_bench.json
bash scripts/gpu.sh prof --steps 3 --warmup 1 > /dev/null || exit 1
cp gpurun_out/prof_kernel_stats.csv gpurun_out/final2_kernel_stats.csv
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --emulate-world 8 > gpurun_out/final2_emu8.log 2>&1 || { tail -5 gpurun_out/final2_emu8.log; exit 1; }
grep '^{' gpurun_out/final2_emu8.log | tail -1 > gpurun_out/final2_emu8.json; cut -c1-200 gpurun_out/final2_emu8.json
timeout -k 10 500 python -u bench.py --workload fedobd_transformer --steps 1 --warmup 1 > gpurun_out/final2_tfm.log 2>&1 || { tail -5 gpurun_out/final2_tfm.log; exit 1; }
grep '^{' gpurun_out/final2_tfm.log | tail -1 > gpurun_out/final2_tfm.json; cut -c1-200 gpurun_out/final2_tfm.json
timeout -k 10 300 python -u bench/eval_bench.py --M 32 --iters 3 > gpurun_out/final2_eval.log 2>&1 || { tail -5 gpurun_out/final2_eval.log; exit 1; }
grep '^{' gpurun_out/final2_eval.log | tail -1 > gpurun_out/final2_eval.json; cut -c1-200 gpurun_out/final2_eval.json
