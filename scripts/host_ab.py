"""Per-call host cost of rc_chunk_device for several library builds on ONE allocation: the wall
time of the enqueue alone (the host's staging of the descriptors) and of K back-to-back calls to
completion, calls in sequence on one stream, timing events off.  Config 3 (i) (65,536 x 1 MiB at
the defaults: no key is hashed, the step is host staging plus one small chain kernel) shows the
host path; 3 (iii) and config 2 for scale.

    python scripts/host_ab.py [3i|3iii|2] [rounds] LIB [LIB ...]
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import _lib, synth  # noqa: E402
from replicat_amd.chunker import fill_splitmix_streams  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else '3i'
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
paths = sys.argv[3:] or [_lib.LIB_PATH]
n, size, mn, mx = {'3i': (65536, 1 << 20, 128_000, 5_120_000),
                   '3iii': (65536, 1 << 20, 2_000, 80_000),
                   '2': (1024, 64 << 20, 128_000, 5_120_000)}[cfg]
torch.cuda.set_stream(torch.cuda.Stream())
hs = torch.cuda.current_stream().cuda_stream
pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
ptrs = np.ascontiguousarray(np.arange(n, dtype=np.uint64) * size + pool.data_ptr())
lens = np.ascontiguousarray([size] * n, dtype=np.uint64)
last = np.zeros(n, dtype=np.uint64)


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return L


libs = []
for p in paths:
    L = load(p)
    h = ctypes.c_void_p()
    assert L.rc_chunker_create(mn, mx, b'\xff' * 16, 16, torch.cuda.current_device(), ctypes.byref(h)) == 0
    caps = np.zeros(n, dtype=np.uint64)
    total = L.rc_cut_capacity(h, n, lens.ctypes.data, caps.ctypes.data)
    libs.append((p, L, h, total))
cuts = torch.zeros(max(x[3] for x in libs), dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
K = 20
res = {p: {'enqueue_ms': [], 'step_ms': []} for p in paths}
for r in range(rounds):
    for p, L, h, _ in (libs if r % 2 == 0 else libs[::-1]):
        def call():
            assert L.rc_chunk_device(h, n, ptrs.ctypes.data, lens.ctypes.data, last.ctypes.data, 0,
                                     cuts.data_ptr(), counts.data_ptr(), hs) == 0, L.rc_last_error()
        call()
        torch.cuda.synchronize()
        enq = 0.0
        t0 = time.perf_counter()
        for _ in range(K):
            t = time.perf_counter()
            call()
            enq += time.perf_counter() - t
        torch.cuda.synchronize()
        res[p]['step_ms'].append((time.perf_counter() - t0) * 1e3 / K)
        res[p]['enqueue_ms'].append(enq * 1e3 / K)
out = {'config': cfg, 'rounds': rounds, 'calls': K}
for p, v in res.items():
    out[os.path.basename(p)] = {k: round(float(np.median(x)), 4) for k, x in v.items()}
print(json.dumps(out), flush=True)
