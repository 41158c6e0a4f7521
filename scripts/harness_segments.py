"""Diagnostic: the harness stream (one 5.12 GB stream, P = L - 512 MB) chunked with different
chain segmentations (RC_SEGMENT_BYTES / RC_SEGMENT_EXT), kernel times per phase and parity."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_util as G  # noqa: E402
from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker  # noqa: E402

bufs = list(synth.harness_buffers())
L = sum(len(b) for b in bufs)
P = L - len(bufs[-1])
pool = torch.empty(L + 64, dtype=torch.uint8, device='cuda')
off = 0
for b in bufs:
    pool[off:off + len(b)].copy_(torch.frombuffer(b, dtype=torch.uint8))
    off += len(b)
del bufs
gold = G.load('harness.json')
hs = torch.cuda.current_stream().cuda_stream
for seg, ext in [(None, None), (None, '4'), (str(32 << 20), None), (str(64 << 20), None),
                 (str(16 << 20), '4')]:
    for k, v in (('RC_SEGMENT_BYTES', seg), ('RC_SEGMENT_EXT', ext)):
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    ch = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
    total, caps = ch.capacity([L])
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(1, dtype=torch.int64, device='cuda')
    for _ in range(2):
        ch.chunk_device([pool.data_ptr()], [L], [P], cuts.data_ptr(), counts.data_ptr(), hs)
    torch.cuda.synchronize()
    ch.timing(True)
    t0 = time.perf_counter()
    for _ in range(5):
        ch.chunk_device([pool.data_ptr()], [L], [P], cuts.data_ptr(), counts.data_ptr(), hs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    ch.timing(False)
    t, e, c, n = ch.read_kernel_timing()
    cnt = int(counts.cpu()[0])
    ends = cuts[:cnt].cpu().numpy().view(np.uint64)
    print(json.dumps({'seg': seg, 'ext': ext, 'ms': round(dt * 1e3, 3), 'tile': round(t / n, 3),
                      'edge': round(e / n, 3), 'chain': round(c / n, 3), 'chunks': cnt,
                      'parity': G.cutlist_digest([ends]) == gold['sha256']}), flush=True)
    ch.close()
