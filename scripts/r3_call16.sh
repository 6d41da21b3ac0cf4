#!/bin/bash
# chunked deterministic embedding backward (tests), FedOBD Transformer-base A/B of weight planes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_kernels_f32_gpu.py -k "embedding" tests/test_kernels_gpu.py::test_embedding_gather tests/test_gpu_sessions.py::test_transformer_imdb_bitwise_reproducible_and_matches_cpu || exit 1
grep -E "passed|failed" gpurun_out/quick_tests.log | tail -1
for v in 1 0; do
  DLS_WSPLIT=$v timeout -k 10 400 python -u bench.py --workload fedobd_transformer --steps 1 --warmup 1 --no-stage2 > gpurun_out/k16_ws$v.log 2>&1 || { tail -5 gpurun_out/k16_ws$v.log; exit 1; }
  echo "wsplit=$v $(grep '^{' gpurun_out/k16_ws$v.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
