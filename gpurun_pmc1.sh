set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
python -c "
from distributed_learning_simulator_amd.parallel import launch; import subprocess, sys
print('visible_gpus', launch.visible_gpus(), 'kfd', launch._kfd_gpus())
print('torch count', subprocess.run([sys.executable,'-c','import torch;print(torch.cuda.device_count())'],capture_output=True,text=True).stdout.strip())" > gpurun_out/visible.log 2>&1
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_halo.log 2>&1 || exit 1
DLS_PLANES=0 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_noplanes.log 2>&1 || exit 1
