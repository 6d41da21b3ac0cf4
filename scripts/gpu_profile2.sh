#!/bin/bash
# GPU-box: kernel stats of one timed FedAvg round at 100 clients and at 13 clients (the 8-GPU
# per-rank load), plus plain wall time of the 13-client bench (host-bound check).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --clients 13 --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/small.log 2>&1 || exit $?
for n in 13 100; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof$n -o run -- \
    python bench.py --clients $n --steps 1 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/prof$n.log 2>&1
  rc=$?
  rm -f gpurun_out/prof$n/run_kernel_trace.csv
  echo "rc=$rc" >> gpurun_out/prof$n.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
