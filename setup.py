"""Packaging: ``pip install -e .`` builds both native extensions in-tree (see torchkafka_amd/_build.py)."""
from setuptools import find_packages, setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        from torchkafka_amd import _build

        _build.build_all(force=False, verbose=True)
        super().run()


setup(
    name="torchkafka-amd",
    version="1.2.0+mi355x.7",
    description="Kafka -> PyTorch streaming with per-batch commits, native on AMD Instinct MI355X (gfx950)",
    license="GPL-3.0-or-later",
    packages=find_packages(include=["torchkafka_amd", "torchkafka_amd.*", "torchkafka"]),
    package_data={"torchkafka_amd": ["csrc/core/*", "csrc/hip/*", "*.so"]},
    python_requires=">=3.8",
    install_requires=["torch>=1.6.0", "numpy", "pybind11"],
    extras_require={"kafka": ["kafka-python>=2.0.2"],
                    "dev": ["pytest", "pytest-timeout", "hypothesis", "pylint", "ruff"]},
    cmdclass={"build_py": BuildNative},
)
