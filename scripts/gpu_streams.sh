#!/bin/bash
# GPU-box: sub-cohort stream count sweep at the 8-rank per-rank load (emulated) and at 100 clients.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in 1 2 3 4; do
  DLS_STREAMS=$s timeout -k 10 300 python bench.py --emulate-world 8 --steps 4 --warmup 1 > gpurun_out/streams_emu8_s$s.log 2>&1 || exit $?
done
for s in 2 4; do
  DLS_STREAMS=$s timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/streams_c100_s$s.log 2>&1 || exit $?
done
