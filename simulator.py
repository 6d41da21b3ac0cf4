"""CLI: `python simulator.py --config-name fed_avg/mnist.yaml ++fed_avg.round=1 ...`

Same flags as the reference (`simulator.py:1-13`, `test.sh`). Multi-GPU: launch one rank
per GPU with torchrun, e.g.
`python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 simulator.py
--config-name large_scale/fed_avg/cifar10.yaml`.
"""

import os
import sys

sys.path.insert(0, os.path.abspath(os.path.dirname(__file__)))

from distributed_learning_simulator_amd.config import global_config, load_config  # noqa: E402
from distributed_learning_simulator_amd.training import train  # noqa: E402

if __name__ == "__main__":
    load_config()
    global_config.apply_global_config()
    train(config=global_config)
