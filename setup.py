"""Packaging of the drop-in: ``pip install --no-build-isolation .`` compiles the HIP library for
gfx950 and installs the package ``replicat_amd`` (with ``libreplicat_chunker.so``) and the
top-level module ``_replicat_adapters`` that replicat imports (replicat/utils/adapters.py:10).

It replaces the reference's native build -- ``CMakeExtension('_replicat_adapters')``
(/root/reference/setup.py:26-75,126-127) over /root/reference/CMakeLists.txt:3-7 (pybind11,
``-mpclmul -msse4.1``) -- with hipcc (replicat_amd/build.py: --offload-arch=gfx950, a build id
hashed over the sources).  The oracle, tests and bench are not part of the package.
"""
import glob
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution

HERE = os.path.dirname(os.path.abspath(__file__))


class build_hip(build_py):
    """Build libreplicat_chunker.so (skipped when the in-tree library's build id matches the
    sources) before the package files are collected."""

    def run(self):
        sys.path.insert(0, HERE)
        from replicat_amd import build as hip
        hip.build(verbose=True)
        super().run()


class BinaryDistribution(Distribution):
    """The wheel carries a gfx950 code object inside a host .so: platform-specific."""

    def has_ext_modules(self):
        return True


def version():
    with open(os.path.join(HERE, 'replicat_amd', '__init__.py')) as f:
        for line in f:
            if line.startswith('__version__'):
                return line.split('=')[1].strip().strip("'")
    raise RuntimeError('no __version__')


setup(
    name='replicat-amd',
    version=version(),
    description="MI355X (gfx950) drop-in for replicat's native chunker _replicat_adapters",
    packages=['replicat_amd'],
    py_modules=['_replicat_adapters'],
    package_data={'replicat_amd': ['libreplicat_chunker.so', 'csrc/*.hip', 'csrc/*.cpp',
                                   'csrc/*.h']},
    data_files=[('include/replicat_amd', sorted(glob.glob('include/*.h')))],
    install_requires=['numpy'],
    python_requires='>=3.8',
    cmdclass={'build_py': build_hip},
    distclass=BinaryDistribution,
    zip_safe=False,
)
