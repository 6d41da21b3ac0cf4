#!/bin/bash
# GPU-box driver for this repo (run through gpurun). Every GPU step has its own time limit and
# the script stops at the first failing step (no retries).
#
#   scripts/gpu.sh tests              pytest -m gpu (every kernel vs its oracle, GPU sessions)
#   scripts/gpu.sh bench [ARGS...]    bench.py ARGS  -> gpurun_out/bench.json
#   scripts/gpu.sh prof  [ARGS...]    rocprofv3 --kernel-trace --stats of bench.py ARGS
#   scripts/gpu.sh marker [ARGS...]  roctx phase ranges + kernel stats (DLS_ROCTX=1)
#   scripts/gpu.sh pmc   COUNTERS [ARGS...]   one rocprofv3 --pmc pass (counter limits: see guide)
#   scripts/gpu.sh pmcset [ARGS...]  MFMA/LDS/HBM counter passes -> gpurun_out/pmc_summary.csv
#   scripts/gpu.sh kbench [ARGS...]   bench/kernel_bench.py ARGS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
mode=$1
shift
case "$mode" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/gpu_tests.log 2>&1
    rc=$?
    tail -15 gpurun_out/gpu_tests.log
    exit $rc
    ;;
  bench)
    timeout -k 10 1000 python -u bench.py "$@" > gpurun_out/bench.log 2>&1
    rc=$?
    grep '^{' gpurun_out/bench.log | tail -1 | tee gpurun_out/bench.json
    [ $rc -ne 0 ] && tail -20 gpurun_out/bench.log
    exit $rc
    ;;
  prof)
    timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python -u bench.py "$@" > gpurun_out/prof_bench.log 2>&1
    rc=$?
    grep '^{' gpurun_out/prof_bench.log | tail -1 | tee gpurun_out/prof_bench.json
    # keep the summaries only: the per-dispatch trace of a long run exceeds the copy-back cap
    stats=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
    [ -n "$stats" ] && cp "$stats" gpurun_out/prof_kernel_stats.csv
    rm -rf gpurun_out/prof
    [ -f gpurun_out/prof_kernel_stats.csv ] && cut -c1-200 gpurun_out/prof_kernel_stats.csv | head -25
    exit $rc
    ;;
  marker)
    # roctx phase ranges (DLS_ROCTX=1: round / train / aggregate / eval_broadcast / step) next to
    # the kernel trace; keeps the range summary and the kernel stats only
    DLS_ROCTX=1 timeout -k 10 1000 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
      -d gpurun_out/marker -o run -- python -u bench.py "$@" > gpurun_out/marker_bench.log 2>&1
    rc=$?
    python scripts/marker_summary.py gpurun_out/marker gpurun_out/marker_ranges.csv
    stats=$(find gpurun_out/marker -name '*kernel_stats.csv' | head -1)
    [ -n "$stats" ] && cp "$stats" gpurun_out/marker_kernel_stats.csv
    rm -rf gpurun_out/marker
    head -20 gpurun_out/marker_ranges.csv
    exit $rc
    ;;
  pmc)
    counters=$1
    shift
    timeout -s KILL 300 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc -o run -- \
      python -u bench.py "$@" > gpurun_out/pmc_bench.log 2>&1
    exit $?
    ;;
  pmcset)
    # two counter passes over the same bench run (each within the per-block slot limits), folded
    # into gpurun_out/pmc_summary.csv by scripts/pmc_summary.py; the raw per-dispatch CSVs are removed
    rm -rf gpurun_out/pmcA gpurun_out/pmcB
    timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
    # (HIP-graph replay under --pmc segfaults in CUDAGraph::replay: counters are taken on eager steps)
    export DLS_GRAPHS=0
    timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcA -o run -- \
      python -u bench.py "$@" > gpurun_out/pmcA.log 2>&1 || { tail -5 gpurun_out/pmcA.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --kernel-trace \
      --output-format csv -d gpurun_out/pmcB -o run -- \
      python -u bench.py "$@" > gpurun_out/pmcB.log 2>&1 || { tail -5 gpurun_out/pmcB.log; exit 1; }
    python scripts/pmc_summary.py gpurun_out/pmc_summary.csv gpurun_out/pmcA gpurun_out/pmcB
    rc=$?
    rm -rf gpurun_out/pmcA gpurun_out/pmcB
    cut -d, -f1-8 gpurun_out/pmc_summary.csv | cut -c1-220 | head -20
    exit $rc
    ;;
  kbench)
    timeout -k 10 900 python -u bench/kernel_bench.py "$@" > gpurun_out/kbench.log 2>&1
    rc=$?
    tail -40 gpurun_out/kbench.log
    exit $rc
    ;;
  *)
    echo "usage: $0 tests|bench|prof|pmc|kbench ..." >&2
    exit 2
    ;;
esac
