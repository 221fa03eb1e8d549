#!/usr/bin/env python3
"""Packaging for shellac_amd (reference: setup.py:1-24 + vendored ez_setup.py).

`python setup.py build_ext --inplace` (or `pip install -e .`) compiles the native
core for gfx950 in-tree via shellac_amd/_build.py (hipcc + g++); console scripts
mirror the reference's `shellac = shellac.server.Server:main`.
"""
from setuptools import Command, find_packages, setup
from setuptools.command.build_ext import build_ext


class BuildNative(build_ext):
    def run(self):
        from shellac_amd import _build

        _build.build()


setup(
    name="shellac_amd",
    version="0.2.0",
    description="Shellac web accelerator, MI355X-native (HBM cache, HIP kernels, RCCL)",
    license="MIT",
    packages=find_packages(include=["shellac_amd", "shellac_amd.*"]),
    package_data={"shellac_amd": ["csrc/*.h", "csrc/*.cc", "csrc/*.hip", "_shellac_core*.so"]},
    python_requires=">=3.8",
    install_requires=["numpy"],
    extras_require={"gpu": ["torch"]},
    cmdclass={"build_ext": BuildNative},
    entry_points={
        "console_scripts": [
            "shellac = shellac_amd.server.proxy:main",
            "shellac-cached = shellac_amd.server.cached:main",
            "shellac-ab = shellac_amd.bench.ab:main",
            "shellac-prof = shellac_amd.utils.prof:main",
        ]
    },
)
