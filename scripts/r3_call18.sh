#!/bin/bash
# LayerNorm split planes feeding the Transformer's plane linears: tests, FedOBD Transformer-base A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_kernels_f32_gpu.py -k "layernorm or linear or attention" tests/test_gpu_sessions.py::test_transformer_imdb_bitwise_reproducible_and_matches_cpu tests/test_gpu_sessions.py::test_methods_match_cpu || exit 1
grep -E "passed|failed" gpurun_out/quick_tests.log | tail -1
for i in 1; do for v in 1 0; do
  DLS_LN_PLANES=$v timeout -k 10 400 python -u bench.py --workload fedobd_transformer --steps 1 --warmup 1 --no-stage2 > gpurun_out/k18_pl${v}_$i.log 2>&1 || { tail -5 gpurun_out/k18_pl${v}_$i.log; exit 1; }
  echo "DLS_LN_PLANES=$v run $i $(grep '^{' gpurun_out/k18_pl${v}_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
bash scripts/r3_final2.sh || exit 1
