"""The packaged boundary (setup.py): an offline ``pip install --no-build-isolation`` of this tree
into a fresh target directory makes ``import _replicat_adapters`` -- replicat's import,
replicat/utils/adapters.py:10 -- resolve to the installed drop-in, whose HIP library loads and
is the same build as the tree's.  Replaces the reference's CMakeExtension build
(/root/reference/setup.py:126-127, CMakeLists.txt:3-7)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r'''
import json, sys
import _replicat_adapters, replicat_amd
from replicat_amd import _lib
from replicat_amd.chunker import build_id
out = {'mod': _replicat_adapters.__file__, 'pkg': replicat_amd.__file__,
       'cls': _replicat_adapters._gclmulchunker.__module__, 'build': build_id(),
       'lib': _lib.LIB_PATH}
try:
    _replicat_adapters._gclmulchunker(4, 8, b'\xff' * 16)
    out['create'] = 'ok'
except _lib.ChunkerUnavailable:
    out['create'] = 'unavailable'
print(json.dumps(out))
'''


@pytest.mark.skipif(subprocess.run([sys.executable, '-m', 'pip', '--version'],
                                   capture_output=True).returncode != 0, reason='no pip')
def test_pip_install_provides_replicat_module(tmp_path):
    target = tmp_path / 'site'
    r = subprocess.run([sys.executable, '-m', 'pip', 'install', '--no-build-isolation', '--no-deps',
                        '--no-index', '--target', str(target), ROOT],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    env = dict(os.environ, PYTHONPATH=str(target))
    r = subprocess.run([sys.executable, '-c', PROBE], capture_output=True, text=True,
                       cwd=str(tmp_path), env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out['mod'].startswith(str(target)) and out['pkg'].startswith(str(target))
    assert out['lib'].startswith(str(target))
    assert out['cls'] == '_replicat_adapters'
    from replicat_amd import build
    assert out['build'] == build.source_id()          # the tree's sources, compiled
    import torch
    if not torch.cuda.is_available():
        assert out['create'] == 'unavailable'         # no CPU fallback in the package either
