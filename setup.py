"""pip packaging (reference `setup.py:8-44`): the package, its YAML config tree and the
in-tree gfx950 extension. `python setup.py build_ext --inplace` (or `pip install -e .`)
compiles every `csrc/*.hip` with hipcc for gfx950 into
`distributed_learning_simulator_amd/_dls_hip*.so`."""

import os

import setuptools
from setuptools.command.build_ext import build_ext

ROOT = os.path.dirname(os.path.abspath(__file__))


class HipBuildExt(build_ext):
    def run(self):
        import sys

        sys.path.insert(0, ROOT)
        from distributed_learning_simulator_amd.ops import build

        print(build.build(force=False, verbose=True))


def _conf_files():
    out = []
    for d, _, files in os.walk(os.path.join(ROOT, "conf")):
        out += [os.path.relpath(os.path.join(d, f), ROOT) for f in files if f.endswith(".yaml")]
    return out


setuptools.setup(
    name="distributed_learning_simulator_amd",
    version="0.1.0",
    description="MI355X-native federated-learning simulator (cohort execution, gfx950 HIP kernels, RCCL)",
    packages=setuptools.find_packages(include=["distributed_learning_simulator_amd", "distributed_learning_simulator_amd.*"]),
    package_data={"distributed_learning_simulator_amd": ["_dls_hip*.so"]},
    data_files=[("conf", _conf_files())],
    cmdclass={"build_ext": HipBuildExt},
    python_requires=">=3.10",
    install_requires=["torch", "pyyaml", "numpy"],
)
