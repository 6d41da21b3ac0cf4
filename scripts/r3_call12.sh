#!/bin/bash
# kernel profile of the GTG utility evaluation (32 subset models x 10k images)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/evprof -o run -- \
  python -u bench/eval_bench.py --M 32 --iters 2 > gpurun_out/evprof.log 2>&1 || { tail -10 gpurun_out/evprof.log; exit 1; }
grep '^{' gpurun_out/evprof.log | tail -1
stats=$(find gpurun_out/evprof -name '*kernel_stats.csv' | head -1)
cp "$stats" gpurun_out/eval_kernel_stats.csv
rm -rf gpurun_out/evprof
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/eval_kernel_stats.csv")))
for r in rows[:25]:
    n = r["Name"].replace("(anonymous namespace)::", "")
    print(f'{float(r["Percentage"]):6.2f}% {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f}us  {n[:120]}')
PY
