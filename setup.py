"""pip-installable package.  The native extension is built by csrc/build.py (hipcc --offload-arch=gfx950
for the kernels, g++ against the PyTorch-ROCm headers for the bindings) into svoc/_C.so, in-tree.

    python setup.py build_ext --inplace     # == python csrc/build.py
    pip install -e .                         # editable install (builds first)
"""
import os
import subprocess
import sys

from setuptools import Command, find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


def _build_native():
    subprocess.check_call([sys.executable, os.path.join(ROOT, "csrc", "build.py")], cwd=ROOT)


class BuildExt(Command):
    description = "build svoc/_C.so (HIP kernels for gfx950 + torch bindings)"
    user_options = [("inplace", "i", "ignored: the extension is always built in-tree")]

    def initialize_options(self):
        self.inplace = 1

    def finalize_options(self):
        pass

    def run(self):
        _build_native()


class BuildPy(build_py):
    def run(self):
        _build_native()
        super().run()


setup(
    name="svoc",
    version="0.1.0",
    description="MI355X-native stochastic vector oracle consensus (HIP/CDNA4 kernels, RCCL)",
    packages=find_packages(include=["svoc", "svoc.*"]),
    package_data={"svoc": ["_C.so"]},
    python_requires=">=3.10",
    install_requires=["torch", "numpy"],
    entry_points={"console_scripts": ["svoc=svoc.__main__:main"]},
    cmdclass={"build_ext": BuildExt, "build_py": BuildPy},
)
