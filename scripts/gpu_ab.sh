#!/bin/bash
# GPU-box: A/B of the fused BN coefficient stage at the 8-rank per-rank load and at 100 clients.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 0 1; do
  DLS_BN_FUSED_COEF=$f timeout -k 10 300 python bench.py --emulate-world 8 --steps 4 --warmup 1 > gpurun_out/ab_emu8_f$f.log 2>&1 || exit $?
  DLS_BN_FUSED_COEF=$f timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/ab_c100_f$f.log 2>&1 || exit $?
done
