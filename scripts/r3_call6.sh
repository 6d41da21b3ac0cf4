#!/bin/bash
# BN backward partials from the dgrad epilogue: kernel + session tests, then an alternating A/B
# of DLS_BN_BWD_PARTS on the headline round
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_kernels_f32_gpu.py -k "bn_bwd_parts or epilogue_bn_stats or batchnorm or halo" tests/test_gpu_sessions.py::test_resnet18_bn_bwd_partials_from_dgrad tests/test_gpu_sessions.py::test_fedavg_resnet18_matches_cpu || exit 1
bash scripts/ab_env.sh DLS_BN_BWD_PARTS "1 0" --steps 3 --warmup 1 || exit 1
