#!/bin/bash
# Kernel stats (one sub-cohort stream, so kernel times do not overlap) of the 100-client headline
# round and of rank 0's share of an 8-rank round (bench.py --emulate-world 8: 13 clients), and
# their per-kernel comparison (scripts/compare_kstats.py) -> gpurun_out/emu8_vs_full.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export DLS_STREAMS=${DLS_STREAMS:-1}
run() {  # name, bench args...
  local n=$1; shift
  rm -rf gpurun_out/p_$n
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_$n -o run -- \
    python3 -u bench.py "$@" > gpurun_out/p_$n.log 2>&1 || { tail -5 gpurun_out/p_$n.log; return 1; }
  cp "$(find gpurun_out/p_$n -name '*kernel_stats.csv' | head -1)" gpurun_out/p_${n}_kernel_stats.csv
  rm -rf gpurun_out/p_$n
  grep '^{' gpurun_out/p_$n.log | tail -1 | cut -c1-160
}
run full --steps 2 --warmup 1 && run emu8 --emulate-world 8 --steps 8 --warmup 1 &&
python3 scripts/compare_kstats.py gpurun_out/p_full_kernel_stats.csv 3 gpurun_out/p_emu8_kernel_stats.csv 9 0.13 \
  > gpurun_out/emu8_vs_full.txt && head -40 gpurun_out/emu8_vs_full.txt
