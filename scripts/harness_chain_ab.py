"""Diagnostic: the harness stream's chain phase (speculative segments + join) under different
segment lengths / extensions, on ONE allocation in one process (chunkers created with
RC_SEGMENT_BYTES / RC_SEGMENT_EXT set; settings alternate round after round).  Every setting
must give the reference's cut list (tests/golden/harness.json).

    python scripts/harness_chain_ab.py [rounds] [SEG:EXT ...]     (SEG 0 = the default choice)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_util as G  # noqa: E402
from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
settings = sys.argv[2:] or ['0:4', '0:3', '10240000:3', '5120000:3', '5120000:2', '7680000:2']
g = G.load('harness.json')
pieces = list(synth.harness_buffers())
L = sum(len(p) for p in pieces)
pool = torch.empty(L + 64, dtype=torch.uint8, device='cuda')
off = 0
for p in pieces:
    pool[off:off + len(p)].copy_(torch.frombuffer(p, dtype=torch.uint8))
    off += len(p)
hs = torch.cuda.current_stream().cuda_stream
chs = {}
for s in settings:
    seg, ext = s.split(':')
    os.environ.pop('RC_SEGMENT_BYTES', None)
    if seg != '0':
        os.environ['RC_SEGMENT_BYTES'] = seg
    os.environ['RC_SEGMENT_EXT'] = ext
    chs[s] = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
os.environ.pop('RC_SEGMENT_BYTES', None)
os.environ.pop('RC_SEGMENT_EXT', None)
total, caps = chs[settings[0]].capacity([L])
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(1, dtype=torch.int64, device='cuda')
res = {s: [] for s in settings}
for r in range(rounds):
    for s in (settings if r % 2 == 0 else settings[::-1]):
        ch = chs[s]
        for _ in range(2):
            ch.chunk_device([pool.data_ptr()], [L], [L - len(pieces[-1])], cuts.data_ptr(),
                            counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(True)
        for _ in range(8):
            ch.chunk_device([pool.data_ptr()], [L], [L - len(pieces[-1])], cuts.data_ptr(),
                            counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(False)
        t, e, c, k = ch.read_kernel_timing()
        n = int(counts.item())
        ok = G.cutlist_digest([cuts[:n].cpu().numpy().view(np.uint64)]) == g['sha256']
        assert ok, s
        res[s].append((t / k, c / k))
out = {'rounds': rounds}
for s, v in res.items():
    out[s] = {'tile_ms': round(float(np.median([x[0] for x in v])), 4),
              'chain_ms': round(float(np.median([x[1] for x in v])), 4)}
print(json.dumps(out), flush=True)
