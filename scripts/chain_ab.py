"""Diagnostic: the chain phase (speculative segments + merge / join) of config 2, 3 (ii) or 4
under different segment lengths / extensions, on ONE allocation in one process (chunkers created
with RC_SEGMENT_BYTES / RC_SEGMENT_EXT set; settings alternate round after round).  Every
setting must give the same cut lists (config 2: the reference's digest, tests/golden).

    python scripts/chain_ab.py CONFIG [rounds] [SEG:EXT[:norepair] ...]  (SEG 0 = the default,
                                                                     fK = floor of K max_lengths)

CONFIG harness: the reference harness's one 5.12 GB stream (its cut lists against
tests/golden/harness.json).  ':norepair' runs that setting with RC_REPAIR=0 (a boundary whose
lists miss sends the stream to the sequential join).
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
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else '2'
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
settings = sys.argv[3:] or ['0:4', '0:3', '0:2']
hs = torch.cuda.current_stream().cuda_stream
last = None
if cfg == 'harness':
    pieces = list(synth.harness_buffers())
    n, size = 1, sum(len(p) for p in pieces)
    pool = torch.empty(size + 64, dtype=torch.uint8, device='cuda')
    off = 0
    for p in pieces:
        pool[off:off + len(p)].copy_(torch.frombuffer(p, dtype=torch.uint8))
        off += len(p)
    last = [size - len(pieces[-1])]
else:
    n, mib = {'2': (1024, 64), '3ii': (1, 64 << 10), '4': (16, 8 << 10)}[cfg]
    size = mib << 20
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
ptrs = [pool.data_ptr() + i * size for i in range(n)]
chs = {}
for s in settings:
    seg, ext = s.split(':')[:2]
    os.environ.pop('RC_SEGMENT_BYTES', None)
    os.environ.pop('RC_SEGMENT_FLOOR', None)
    if seg.startswith('f'):  # fK: the default choice with a floor of K max_lengths
        os.environ['RC_SEGMENT_FLOOR'] = seg[1:]
    elif seg != '0':
        os.environ['RC_SEGMENT_BYTES'] = seg
    os.environ['RC_SEGMENT_EXT'] = ext
    os.environ['RC_REPAIR'] = '0' if s.endswith(':norepair') else '1'
    chs[s] = GpuChunker(128_000, 5_120_000, b'\xff' * 16)  # knobs read at creation (knobs.h)
os.environ.pop('RC_SEGMENT_BYTES', None)
os.environ.pop('RC_SEGMENT_EXT', None)
os.environ.pop('RC_SEGMENT_FLOOR', None)
os.environ.pop('RC_REPAIR', None)
total, caps = chs[settings[0]].capacity([size] * n)
base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
gold = {d['name']: d for d in G.load('digests.json')}
want = (gold['config2_ff']['sha256'] if cfg == '2' else
        G.load('harness.json')['sha256'] if cfg == 'harness' else None)
res = {s: [] for s in settings}
for r in range(rounds):
    for s in (settings if r % 2 == 0 else settings[::-1]):
        ch = chs[s]
        ch.chunk_device(ptrs, [size] * n, last, cuts.data_ptr(), counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(True)
        for _ in range(5):
            ch.chunk_device(ptrs, [size] * n, last, cuts.data_ptr(), counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(False)
        t, e, c, k = ch.read_kernel_timing()
        ch_h = cuts.cpu().numpy().view(np.uint64)
        k_h = counts.cpu().numpy()
        dig = G.cutlist_digest([ch_h[b:b + m] for b, m in zip(base, k_h)])
        want = want or dig
        assert dig == want, s
        res[s].append((t / k, c / k))
out = {'config': cfg, 'rounds': rounds}
for s, v in res.items():
    out[s] = {'tile_ms': round(float(np.median([x[0] for x in v])), 4),
              'chain_ms': round(float(np.median([x[1] for x in v])), 4),
              'chain_ms_min': round(float(np.min([x[1] for x in v])), 4)}
print(json.dumps(out), flush=True)
