"""Build libreplicat_chunker.so in-tree: hipcc, gfx950 only, no torch extension machinery.

    python -m replicat_amd.build            (also run by __graft_entry__.build() and setup.py)
    python -m replicat_amd.build --force
    python -m replicat_amd.build --variant STAMPS -DRC_DIAG_STAMPS   (diag/lib_STAMPS.so)
    python -m replicat_amd.build --diag     (+ the GCM watchdog harness under diag/)

Staleness is decided by content, not mtime: the library embeds a build id -- a hash over every
source and header and the compile command -- and a library whose id differs from the tree's is
rebuilt (``rc_build_id()`` returns it at run time; profiles record it).
"""
import hashlib
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
LIB = os.path.join(HERE, 'libreplicat_chunker.so')
SOURCES = [os.path.join(CSRC, n) for n in ('kernels.hip', 'capi.cpp', 'blake2b.hip', 'capi_digest.cpp', 'gcm.hip',
                                             'capi_cipher.cpp')]
HEADERS = [os.path.join(CSRC, n) for n in ('gclmul.h', 'digest_kernels.h', 'capi_internal.h', 'cipher_kernels.h',
                                             'knobs.h', 'diag.h')] + [
    os.path.join(ROOT, 'include', n) for n in ('replicat_chunker.h', 'replicat_digest.h', 'replicat_cipher.h')]
ARCH = 'gfx950'
# -amdgpu-atomic-optimizer-strategy=None: the tile kernel's one-lane grab of its next work unit
# must stay a plain global_atomic_add whose result is read a unit later; the optimizer rewrites a
# uniform-address atomic into a wave reduction + readfirstlane, i.e. an immediate vmcnt(0) that
# drains the wave's whole HBM ring (kernels.hip TileUnits)
FLAGS = [f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-fPIC', '-shared', '-Wall',
         '-mllvm', '-amdgpu-atomic-optimizer-strategy=None']
_ID_RE = re.compile(rb'RC_BUILD_ID:([0-9a-f]{16})')


def hipcc():
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', shutil.which('hipcc')):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError('hipcc not found (ROCm 7.x required)')


_COMPILER = {}


def compiler_id():
    """The resolved hipcc and its version banner (a ROCm upgrade changes the code object)."""
    if 'id' not in _COMPILER:
        cc = hipcc()
        try:
            banner = subprocess.run([cc, '--version'], capture_output=True, text=True,
                                    timeout=120).stdout
        except (OSError, subprocess.SubprocessError):
            banner = ''
        _COMPILER['id'] = os.path.realpath(cc) + '\n' + banner.strip()
    return _COMPILER['id']


def source_id(extra=()):
    """Hash of every source/header (path relative to the package), the compile flags and the
    compiler (path + version)."""
    h = hashlib.sha256()
    for p in SOURCES + HEADERS:
        h.update(os.path.relpath(p, ROOT).encode() + b'\0')
        with open(p, 'rb') as f:
            h.update(f.read())
    h.update(' '.join(FLAGS + list(extra)).encode())
    h.update(b'\0' + compiler_id().encode())
    return h.hexdigest()[:16]


def embedded_id(path=LIB):
    """The build id compiled into a library file, or None."""
    try:
        with open(path, 'rb') as f:
            m = _ID_RE.search(f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def stale(path=LIB, extra=()):
    return embedded_id(path) != source_id(extra)


def _compile(out, extra=(), verbose=False):
    bid = source_id(extra)
    cmd = [hipcc(), *FLAGS, *extra, f'-DRC_BUILD_ID="{bid}"', '-I', os.path.join(ROOT, 'include'),
           *SOURCES, '-o', out + '.tmp']
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + '.tmp', out)
    return out


def build(force=False, verbose=False):
    if not force and not stale():
        return LIB
    return _compile(LIB, verbose=verbose)


def build_variant(name, defines, verbose=False):
    """A diagnostic build (e.g. -DRC_DIAG_STAMPS) as diag/lib_<name>.so, loaded through
    RC_LIB_PATH by the diagnostics scripts only."""
    out_dir = os.path.join(ROOT, 'diag')
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f'lib_{name}.so')
    if stale(out, defines):
        _compile(out, defines, verbose)
    return out


def build_diag(verbose=False):
    """The AES-GCM watchdog harness (scripts/gcm_diag.cpp) as two executables under diag/: on the
    production kernel, and with -DRC_GCM_TRACE (a progress word the host polls while the kernel
    runs).  Diagnostics only; nothing in the product loads them."""
    out_dir = os.path.join(ROOT, 'diag')
    os.makedirs(out_dir, exist_ok=True)
    srcs = SOURCES + [os.path.join(ROOT, 'scripts', 'gcm_diag.cpp')]
    for name, extra in (('gcm_diag_notrace', []), ('gcm_diag', ['-DRC_GCM_TRACE'])):
        cmd = [hipcc(), f'--offload-arch={ARCH}', '-O3', '-std=c++17', *extra,
               '-I', os.path.join(ROOT, 'include'), *srcs, '-o', os.path.join(out_dir, name)]
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.run(cmd, check=True)


if __name__ == '__main__':
    if '--variant' in sys.argv:
        i = sys.argv.index('--variant')
        build_variant(sys.argv[i + 1], [a for a in sys.argv[i + 2:] if a.startswith('-D')], True)
    else:
        build(force='--force' in sys.argv, verbose=True)
    if '--diag' in sys.argv:
        build_diag(verbose=True)
