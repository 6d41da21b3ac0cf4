#!/bin/bash
# round-3 GPU batch 2: sign-SGD ResNet-50 and DenseNet-40 fp32 kernel profiles (+ their bench lines)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
prof() {  # prof TAG ARGS...: rocprofv3 kernel stats of one bench run -> gpurun_out/TAG_kernel_stats.csv
  tag=$1; shift
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
    python -u bench.py "$@" > gpurun_out/prof_$tag.log 2>&1
  rc=$?
  grep '^{' gpurun_out/prof_$tag.log | tail -1 > gpurun_out/prof_$tag.json
  stats=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
  [ -n "$stats" ] && cp "$stats" gpurun_out/${tag}_kernel_stats.csv
  rm -rf gpurun_out/prof_$tag
  return $rc
}
prof signsgd --workload signsgd_resnet50 --steps 1 --warmup 1 || exit 1
prof densenet --workload fedavg_densenet40 --steps 1 --warmup 1 || exit 1
for t in signsgd densenet; do cut -d, -f1-5 gpurun_out/${t}_kernel_stats.csv | cut -c1-160 | head -14; done
timeout -k 10 600 python -u bench/kernel_bench.py --f32 --planes --K 50 --skip-misc --iters 5 > gpurun_out/kbench_f32_planes_K50.log 2>&1 || { tail -20 gpurun_out/kbench_f32_planes_K50.log; exit 1; }
bash scripts/gpu.sh pmcset --steps 1 --warmup 1 || exit 1
timeout -k 10 600 python -u bench.py --workload fedobd_transformer --steps 1 --warmup 1 > gpurun_out/fedobd_tb.log 2>&1 || { tail -20 gpurun_out/fedobd_tb.log; exit 1; }
grep '^{' gpurun_out/fedobd_tb.log | tail -1 > gpurun_out/fedobd_tb.json
