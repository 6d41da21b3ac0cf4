#!/bin/bash
# compact shortcut dgrad: tests + headline; 8-rank share; 4-rank rehearsal on one GPU; sign-SGD planes A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_kernels_f32_gpu.py -k "compact or planes_every or halo or wgrad" tests/test_gpu_sessions.py::test_resnet18_bitwise_reproducible_and_planes tests/test_gpu_sessions.py::test_fedavg_resnet18_matches_cpu tests/test_multirank_gpu.py || exit 1
timeout -k 10 600 python -u bench/kernel_bench.py --f32 --planes --K 50 --skip-misc --iters 5 --only l1,l2,l3,l4 > gpurun_out/kbench_wh.log 2>&1 || { tail -20 gpurun_out/kbench_wh.log; exit 1; }
grep '^{' gpurun_out/kbench_wh.log | cut -c1-120
bash scripts/gpu.sh bench --steps 3 --warmup 1 || exit 1
cp gpurun_out/bench.json gpurun_out/bench_headline.json
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --emulate-world 8 > gpurun_out/emu8.log 2>&1 || { tail -5 gpurun_out/emu8.log; exit 1; }
grep '^{' gpurun_out/emu8.log | tail -1 | tee gpurun_out/emu8.json
DLS_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 4 --steps 2 --warmup 1 > gpurun_out/multirank4.log 2>&1 || { tail -20 gpurun_out/multirank4.log; exit 1; }
grep '^{' gpurun_out/multirank4.log | tail -1 | tee gpurun_out/multirank4.json
for sp in 0 1; do
  DLS_SHARED_PLANES=$sp timeout -k 10 400 python -u bench.py --workload signsgd_resnet50 --steps 1 --warmup 1 --cohort 8 > gpurun_out/signsgd_sp$sp.log 2>&1 || { tail -5 gpurun_out/signsgd_sp$sp.log; exit 1; }
  grep '^{' gpurun_out/signsgd_sp$sp.log | tail -1 | cut -c1-200
done
