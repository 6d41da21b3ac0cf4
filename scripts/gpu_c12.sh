#!/bin/bash
# downsample-BN fold: its tests, then alternating headline / eval A/Bs (DLS_BN_RES_FOLD 1 / 0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_f32_gpu.py \
  tests/test_gpu_sessions.py -k "folded_residual or downsample_bn_fold or bn_bwd_in_wgrad or pixel_major" \
  > gpurun_out/c12_tests.log 2>&1 || { tail -20 gpurun_out/c12_tests.log; exit 1; }
tail -1 gpurun_out/c12_tests.log
for r in 1 2; do
  for f in 1 0; do
    DLS_BN_RES_FOLD=$f timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > gpurun_out/c12_hl.log 2>&1 || { tail -5 gpurun_out/c12_hl.log; exit 1; }
    echo "headline fold=$f $(grep '^{' gpurun_out/c12_hl.log | tail -1 | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"],1))')"
  done
done
for f in 1 0 1 0; do
  DLS_BN_RES_FOLD=$f timeout -k 10 300 python -u bench/eval_bench.py --rounds 2 > gpurun_out/c12_ev.log 2>&1 || { tail -5 gpurun_out/c12_ev.log; exit 1; }
  echo "eval fold=$f $(grep '^{' gpurun_out/c12_ev.log | tail -1 | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_model"],2))')"
done
