#!/bin/bash
# per-layer split-K reference (DLS_TN_KREF) and NT tiles at a rank's small cohort (K=7) vs K=50
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for K in 7 50; do for kref in 8 16 32; do
  DLS_TN_KREF=$kref timeout -k 10 300 python -u bench/kernel_bench.py --f32 --planes --K $K --skip-misc --iters 5 --only l1,l2,l3,l4 > gpurun_out/kb9_K${K}_kref$kref.log 2>&1 || { tail -20 gpurun_out/kb9_K${K}_kref$kref.log; exit 1; }
  grep '^{' gpurun_out/kb9_K${K}_kref$kref.log | K=$K KREF=$kref python -c '
import json,os,sys
for l in sys.stdin:
    d=json.loads(l); print("K", os.environ["K"], "kref", os.environ["KREF"], d.get("layer"), "wgrad", d["planes_wgrad"], "nt", d["planes_fwd_dgrad"])'
done; done
