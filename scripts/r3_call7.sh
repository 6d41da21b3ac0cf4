#!/bin/bash
# session tests for the BN partials; small-cohort knobs (DLS_PL_MIN_WG, DLS_TN_KREF) on the
# emulated 8-rank share and on the full 1-GPU round
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_gpu_sessions.py::test_resnet18_bn_bwd_partials_from_dgrad tests/test_gpu_sessions.py::test_fedavg_resnet18_matches_cpu tests/test_gpu_sessions.py::test_methods_match_cpu tests/test_kernels_gpu.py -k "quant or sign or compress or stochastic or methods or resnet18" || exit 1
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python -u bench.py "$@" > "gpurun_out/k7_$name.log" 2>&1 || { tail -5 "gpurun_out/k7_$name.log"; exit 1; }
  echo "$name $(grep '^{' "gpurun_out/k7_$name.log" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for i in 1 2; do
  run emu8_base_$i X=0 -- --steps 3 --warmup 1 --emulate-world 8
  run emu8_wg_$i DLS_PL_MIN_WG=512 -- --steps 3 --warmup 1 --emulate-world 8
  run emu8_kref_$i DLS_TN_KREF=8 -- --steps 3 --warmup 1 --emulate-world 8
  run emu8_both_$i DLS_PL_MIN_WG=512 DLS_TN_KREF=8 -- --steps 3 --warmup 1 --emulate-world 8
done
run full_base X=0 -- --steps 3 --warmup 1
run full_both DLS_PL_MIN_WG=512 DLS_TN_KREF=8 -- --steps 3 --warmup 1
