#!/bin/bash
# epilogue operand prefetch: fp32 kernel tests + sessions, headline x2, kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r3_quick.sh tests/test_kernels_f32_gpu.py tests/test_gpu_sessions.py tests/test_multirank_gpu.py || exit 1
grep -E "passed|failed" gpurun_out/quick_tests.log | tail -2
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/k13_full_$i.log 2>&1 || { tail -5 gpurun_out/k13_full_$i.log; exit 1; }
  echo "full_$i $(grep '^{' gpurun_out/k13_full_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
bash scripts/gpu.sh prof --steps 3 --warmup 1 > /dev/null || exit 1
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_kernel_stats.csv")))
for r in rows[:12]:
    n = r["Name"].replace("(anonymous namespace)::", "")
    print(f'{float(r["Percentage"]):6.2f}% {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f}us  {n[:100]}')
PY
