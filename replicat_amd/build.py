"""Build libreplicat_chunker.so in-tree: hipcc, gfx950 only, no torch extension machinery.

    python -m replicat_amd.build        (also run by __graft_entry__.build())
    python -m replicat_amd.build --diag (+ the GCM watchdog harness under diag/)
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
LIB = os.path.join(HERE, 'libreplicat_chunker.so')
SOURCES = [os.path.join(CSRC, n) for n in ('kernels.hip', 'capi.cpp', 'blake2b.hip', 'capi_digest.cpp', 'gcm.hip',
                                             'capi_cipher.cpp')]
HEADERS = [os.path.join(CSRC, n) for n in ('gclmul.h', 'digest_kernels.h', 'capi_internal.h', 'cipher_kernels.h')] + [
    os.path.join(ROOT, 'include', n) for n in ('replicat_chunker.h', 'replicat_digest.h', 'replicat_cipher.h')]
ARCH = 'gfx950'


def hipcc():
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', shutil.which('hipcc')):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError('hipcc not found (ROCm 7.x required)')


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS)


def build(force=False, verbose=False):
    if not force and not stale():
        return LIB
    cmd = [hipcc(), f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-fPIC', '-shared', '-Wall',
           '-I', os.path.join(ROOT, 'include'), *SOURCES, '-o', LIB + '.tmp']
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + '.tmp', LIB)
    return LIB


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
    build(force='--force' in sys.argv, verbose=True)
    if '--diag' in sys.argv:
        build_diag(verbose=True)
