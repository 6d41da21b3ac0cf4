"""bench.py with one plane-TN tile variant (TN_PL_VARIANT) and / or one LDS-halo conv variant
(HALO_VARIANT) forced for every launch, or the halo shape rule (HALO_MODE: 1 = every supported
shape, the 4x4 l4 convs too) — an A/B helper, not product code:
    TN_PL_VARIANT=<id> HALO_VARIANT=<id> HALO_MODE=<m> python scripts/bench_tn_variant.py [bench.py args]."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
v = int(os.environ.get("TN_PL_VARIANT", "-1"))
hv = int(os.environ.get("HALO_VARIANT", "-1"))
hm = int(os.environ.get("HALO_MODE", "-1"))
if v >= 0 or hv >= 0 or hm >= 0:
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip

    if v >= 0:
        hip._C.conv_tn_pl_set_variant(v)
    if hv >= 0:
        hip._C.conv_halo_set_variant(hv)
    if hm >= 0:
        hip._C.conv_halo_set_mode(hm)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
