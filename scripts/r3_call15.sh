#!/bin/bash
# FedOBD Transformer-base stage-1 round: kernel profile (round 2 -> 3 regression check)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu.sh prof --workload fedobd_transformer --steps 1 --warmup 1 --no-stage2 > /dev/null || { tail -20 gpurun_out/prof_bench.log; exit 1; }
cut -c1-300 gpurun_out/prof_bench.json
cp gpurun_out/prof_kernel_stats.csv gpurun_out/tfm_kernel_stats.csv
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/tfm_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", tot / 1e6)
for r in rows[:25]:
    n = r["Name"].replace("(anonymous namespace)::", "")
    print(f'{float(r["Percentage"]):6.2f}% {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f}us  {n[:110]}')
PY
