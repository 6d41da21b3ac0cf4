"""bench.py with one plane-TN tile variant forced for every launch (an A/B helper, not product
code): TN_PL_VARIANT=<id> python scripts/bench_tn_variant.py [bench.py args]."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
v = int(os.environ.get("TN_PL_VARIANT", "-1"))
if v >= 0:
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip

    hip._C.conv_tn_pl_set_variant(v)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
