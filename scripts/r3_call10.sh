#!/bin/bash
# cohort-class split-K + small-cohort NT tile defaults: tests, full round, emulated 8-rank share
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_kernels_f32_gpu.py -k "wgrad or planes_every" || exit 1
cp gpurun_out/quick_tests.log gpurun_out/quick_tests_k.log
bash scripts/r3_quick.sh tests/test_gpu_sessions.py::test_resnet18_bitwise_reproducible_and_planes tests/test_gpu_sessions.py::test_resnet18_bn_bwd_partials_from_dgrad tests/test_multirank_gpu.py || exit 1
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python -u bench.py "$@" > "gpurun_out/k10_$name.log" 2>&1 || { tail -5 "gpurun_out/k10_$name.log"; exit 1; }
  echo "$name $(grep '^{' "gpurun_out/k10_$name.log" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for i in 1 2; do
  run full_$i X=0 -- --steps 3 --warmup 1
  run full_old_$i DLS_TN_KREF=32 DLS_PL_MIN_WG=0 -- --steps 3 --warmup 1
  run emu8_$i X=0 -- --steps 3 --warmup 1 --emulate-world 8
done
run emu4 X=0 -- --steps 3 --warmup 1 --emulate-world 4
run emu2 X=0 -- --steps 3 --warmup 1 --emulate-world 2
