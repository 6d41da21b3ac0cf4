#!/bin/bash
# kernel profile of rank 0's share of an 8-rank round (13 clients, 2 streams)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu.sh prof --steps 3 --warmup 1 --emulate-world 8 > /dev/null || { tail -20 gpurun_out/prof_bench.log; exit 1; }
cut -c1-200 gpurun_out/prof_bench.json
cp gpurun_out/prof_kernel_stats.csv gpurun_out/emu8_kernel_stats.csv
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/emu8_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", tot / 1e6)
for r in rows[:25]:
    n = r["Name"].replace("(anonymous namespace)::", "")
    print(f'{float(r["Percentage"]):6.2f}% {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f}us  {n[:110]}')
PY
