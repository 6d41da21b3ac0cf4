set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_f32_gpu.py tests/test_gpu_sessions.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sess.log 2>&1 || { tail -40 gpurun_out/t_sess.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_halo.log 2>&1 || exit 1
DLS_PLANES=0 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_noplanes.log 2>&1 || exit 1
