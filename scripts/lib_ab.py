"""A/B of several builds of the chunker library in ONE process on ONE allocation: each library
is loaded with ctypes (its own code object; the C ABI of include/replicat_chunker.h), gets its
own chunker, and the builds take turns chunking the same device arena, round after round
(ABBA order).  Removes the per-process allocation spread (profiles/r02/placement) from the
comparison.  Every build must produce the same cut lists (except the RC_DIAG_NO_TAIL
diagnostic build, diag/lib_NOTAIL.so, which stores no records and is timed only).

    python scripts/lib_ab.py [config] [rounds] LIB [LIB ...]      config: 2 | 3ii | 3iii | 4 | harness

LIB_AB_FLAGS (environment): the rc_chunk_device flags of every call (2 = RC_PIPELINED; with
RC_PIPE_ALL=1 small-window batches overlap too).  Timing-only builds whose cut lists differ by
design carry NOTAIL, NOEXACT or NOWORDS in their file name.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import _lib, synth  # noqa: E402
from replicat_amd.chunker import fill_splitmix_streams  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else '2'
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
paths = sys.argv[3:] or [_lib.LIB_PATH]
FLAGS = int(os.environ.get('LIB_AB_FLAGS', '0'))


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return L


hs = torch.cuda.current_stream().cuda_stream
if cfg == 'harness':
    pieces = list(synth.harness_buffers())
    total_len = sum(len(p) for p in pieces)
    pool = torch.empty(total_len + 64, dtype=torch.uint8, device='cuda')
    off = 0
    for p in pieces:
        pool[off:off + len(p)].copy_(torch.frombuffer(p, dtype=torch.uint8))
        off += len(p)
    ptrs, lens, last = [pool.data_ptr()], [total_len], [total_len - len(pieces[-1])]
    mn, mx = 128_000, 5_120_000
else:
    n, size, mn, mx = {'2': (1024, 64 << 20, 128_000, 5_120_000),
                       '3iii': (65536, 1 << 20, 2_000, 80_000),
                       '3ii': (1, 64 << 30, 128_000, 5_120_000),
                       '4': (16, 8 << 30, 128_000, 5_120_000)}[cfg]
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
    ptrs = np.arange(n, dtype=np.uint64) * size + pool.data_ptr()
    lens, last = [size] * n, None
ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
lens = np.ascontiguousarray(lens, dtype=np.uint64)
last = np.ascontiguousarray(last if last is not None else np.zeros(len(lens)), dtype=np.uint64)
libs = []
for p in paths:
    L = load(p)
    h = ctypes.c_void_p()
    key = b'\xff' * 16
    assert L.rc_chunker_create(mn, mx, key, 16, torch.cuda.current_device(), ctypes.byref(h)) == 0
    caps = np.zeros(len(lens), dtype=np.uint64)
    total = L.rc_cut_capacity(h, len(lens), lens.ctypes.data, caps.ctypes.data)
    libs.append((p, L, h, total))
total = max(x[3] for x in libs)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(len(lens), dtype=torch.int64, device='cuda')
ref = None
res = {p: [] for p in paths}
for r in range(rounds):
    order = libs if r % 2 == 0 else libs[::-1]
    for p, L, h, _ in order:
        def call():
            rc = L.rc_chunk_device(h, len(lens), ptrs.ctypes.data, lens.ctypes.data,
                                   last.ctypes.data, FLAGS, cuts.data_ptr(), counts.data_ptr(), hs)
            assert rc == 0, L.rc_last_error()
        cuts.zero_()  # a diagnostic build's longer lists must not leave entries behind
        for _ in range(2):
            call()
        torch.cuda.synchronize()
        L.rc_timing_enable(h, 1)
        for _ in range(8):
            call()
        torch.cuda.synchronize()
        L.rc_timing_enable(h, 0)
        t, e, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        k = ctypes.c_uint64()
        L.rc_timing_read_kernels(h, ctypes.byref(t), ctypes.byref(e), ctypes.byref(c), ctypes.byref(k))
        res[p].append((t.value / k.value, e.value / k.value, c.value / k.value))
        sig = (int(counts.sum().item()), int(cuts.sum().item()))
        if not any(t in p for t in ('NOTAIL', 'NOEXACT', 'NOWORDS')):  # timing-only builds
            ref = ref or sig
            assert sig == ref, (p, sig, ref)
out = {'config': cfg, 'rounds': rounds}
for p, v in res.items():
    a = np.array(v)
    out[os.path.basename(p)] = {'tile_ms': round(float(np.median(a[:, 0])), 4),
                                'edge_ms': round(float(np.median(a[:, 1])), 4),
                                'chain_ms': round(float(np.median(a[:, 2])), 4)}
print(json.dumps(out), flush=True)
