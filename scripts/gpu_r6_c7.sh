#!/bin/bash
# round 6: GPU idle gaps of the headline round (2 streams), A/B of the halo-wgrad small-cohort
# pixel groups on rank 0's 8-rank share (this tree vs ab_old/ = the previous commit), and the
# per-kernel 13-client vs 100-client comparison
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
DLS_STREAMS=2 bash scripts/trace_gaps_run.sh && head -8 gpurun_out/trace_gaps_s2.txt &&
bash scripts/ab_tree.sh --emulate-world 8 --steps 4 --warmup 1 &&
bash scripts/prof_emu8.sh
