#!/bin/bash
# attention occupancy change: the attention / Transformer GPU tests, the attention bench, and the
# FedOBD Transformer-base bench (3 timed rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "attention or attn or transformer or imdb" \
  > gpurun_out/c13_tests.log 2>&1 || { tail -20 gpurun_out/c13_tests.log; exit 1; }
tail -1 gpurun_out/c13_tests.log
timeout -k 10 120 python -u bench/attn_bench.py > gpurun_out/c13_attn.log 2>&1 || { tail -3 gpurun_out/c13_attn.log; exit 1; }
grep '^{' gpurun_out/c13_attn.log
timeout -k 10 700 python -u bench.py --workload fedobd_transformer --steps 3 --warmup 1 > gpurun_out/c13_tfm.log 2>&1 || { tail -5 gpurun_out/c13_tfm.log; exit 1; }
grep '^{' gpurun_out/c13_tfm.log | tail -1 > gpurun_out/c13_tfm.json
python3 -c 'import json; d=json.load(open("gpurun_out/c13_tfm.json")); print(round(d["ms_per_step"],1), "ms/round", d.get("stage2", ""))'
