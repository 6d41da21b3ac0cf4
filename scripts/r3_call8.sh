#!/bin/bash
# new TN wave tiles (sweep), DenseNet BN partials (tests + A/B), small-cohort knob A/B at full size
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_kernels_f32_gpu.py -k "bn_bwd_parts or wgrad_planes_every or dense_block" || exit 1
cp gpurun_out/quick_tests.log gpurun_out/quick_tests_k.log
bash scripts/r3_quick.sh tests/test_gpu_sessions.py::test_densenet40_session_matches_cpu tests/test_gpu_sessions.py::test_resnet18_bn_bwd_partials_from_dgrad || exit 1
timeout -k 10 600 python -u bench/kernel_bench.py --f32 --planes --K 50 --skip-misc --iters 5 --only l1,l2,l3,l4 > gpurun_out/kbench_tn.log 2>&1 || { tail -20 gpurun_out/kbench_tn.log; exit 1; }
grep '^{' gpurun_out/kbench_tn.log | python -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get("layer"), "wgrad", d.get("planes_wgrad"))'
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python -u bench.py "$@" > "gpurun_out/k8_$name.log" 2>&1 || { tail -5 "gpurun_out/k8_$name.log"; exit 1; }
  echo "$name $(grep '^{' "gpurun_out/k8_$name.log" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
}
for i in 1 2; do
  run full_base_$i X=0 -- --steps 3 --warmup 1
  run full_kref_$i DLS_TN_KREF=8 -- --steps 3 --warmup 1
  run full_wg_$i DLS_PL_MIN_WG=128 -- --steps 3 --warmup 1
done
run emu8_both DLS_PL_MIN_WG=128 DLS_TN_KREF=8 -- --steps 3 --warmup 1 --emulate-world 8
run emu8_base X=0 -- --steps 3 --warmup 1 --emulate-world 8
run dense_parts X=0 -- --model densenet40 --steps 1 --warmup 1
run dense_noparts DLS_BN_BWD_PARTS=0 -- --model densenet40 --steps 1 --warmup 1
