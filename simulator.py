"""CLI: `python simulator.py --config-name fed_avg/mnist.yaml ++fed_avg.round=1 ...`

Same flags as the reference (`simulator.py:1-13`, `test.sh`). Like the reference
(`config.py:22`: `parallel_number = len(get_devices())`), a plain `python simulator.py ...` runs
one rank per visible GPU: the process spawns `parallel_number` ranks itself
(parallel/launch.py) before touching the GPU. Under torchrun (WORLD_SIZE set) it is one rank.
"""

import os
import sys

sys.path.insert(0, os.path.abspath(os.path.dirname(__file__)))

from distributed_learning_simulator_amd.config import global_config, load_config  # noqa: E402
from distributed_learning_simulator_amd.parallel import launch  # noqa: E402

if __name__ == "__main__":
    load_config()
    n = int(global_config.parallel_number or 0) or max(launch.visible_gpus(), 1)
    if n > 1 and not launch.under_launcher():
        sys.exit(launch.spawn_ranks(n))
    from distributed_learning_simulator_amd.training import train

    from distributed_learning_simulator_amd.parallel.comm import shutdown

    global_config.apply_global_config()
    try:
        train(config=global_config)
    finally:
        shutdown()  # every rank leaves the process group before exit
