set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_f32_gpu.py -x -q -k planes --timeout 120 --timeout-method thread > gpurun_out/t_f32.log 2>&1 || { tail -30 gpurun_out/t_f32.log; exit 1; }
timeout -k 10 300 python -u bench/kernel_bench.py --f32 --planes --skip-misc --K 50 --iters 5 --only l1,l2,l3,l4,l4a > gpurun_out/kb_planes3.jsonl 2>&1 || exit 1
