cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
DLS_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/multirank2.log 2>&1 || { tail -20 gpurun_out/multirank2.log; exit 1; }
grep '^{' gpurun_out/multirank2.log | cut -c1-400
bash scripts/ab_streams.sh "1 2" "0" || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcL -o run -- python -u bench/kernel_bench.py --f32 --skip-misc --K 100 --only l1,l3 --iters 3 > gpurun_out/pmcL.log 2>&1 || { tail -5 gpurun_out/pmcL.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_kernels.csv gpurun_out/pmcL && rm -rf gpurun_out/pmcL
cut -d, -f1-14 gpurun_out/pmc_kernels.csv | cut -c1-300 | head -12
