"""A/B of the tile kernel's work-unit schedule on ONE allocation (the per-allocation read-rate
spread of profiles/r02/placement is larger than the effect, so settings are compared inside one
process on one arena).  Each setting is a chunker created with RC_TILE_STATIC (per mille of the
tiles handed out statically; 1000 = fully static, the round-2 schedule) and RC_TILE_CHUNK (tiles
per dynamic unit) in the environment -- the library reads its knobs when a chunker is created
(replicat_amd/csrc/knobs.h); settings alternate round after round and the median tile-kernel
time per setting is printed.

    python scripts/tile_sched_ab.py [config] [rounds] [setting ...]  setting = STATIC:CHUNK[:g]
    python scripts/tile_sched_ab.py 2 6 1000:32 750:32 500:16 500:64

A trailing ":g" runs that setting on a chunker created with RC_TILE_GROUPS=1 (group records
and edge-range trimming for large windows too).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else '2'
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
settings = sys.argv[3:] or ['1000:32', '750:32', '500:16', '500:64']
hs = torch.cuda.current_stream().cuda_stream
if cfg == 'harness':
    pieces = list(synth.harness_buffers())
    L = sum(len(p) for p in pieces)
    pool = torch.empty(L + 64, dtype=torch.uint8, device='cuda')
    off = 0
    for p in pieces:
        pool[off:off + len(p)].copy_(torch.frombuffer(p, dtype=torch.uint8))
        off += len(p)
    ptrs, lens, last = [pool.data_ptr()], [L], [L - len(pieces[-1])]
    mn, mx = 128_000, 5_120_000
else:
    n, size, mn, mx = {'2': (1024, 64 << 20, 128_000, 5_120_000),
                       '3iii': (65536, 1 << 20, 2_000, 80_000),
                       '4': (16, 8 << 30, 128_000, 5_120_000)}[cfg]
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
    ptrs = np.arange(n, dtype=np.uint64) * size + pool.data_ptr()
    lens, last = [size] * n, None



def chunker_with(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return GpuChunker(mn, mx, b'\xff' * 16)  # knobs are read here
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


chunkers = {}
for s in settings:
    st, ck = s.split(':')[:2]
    env = {'RC_TILE_STATIC': st, 'RC_TILE_CHUNK': ck}
    if ':g' in s[len(st) + len(ck) + 1:]:
        env['RC_TILE_GROUPS'] = '1'
    chunkers[s] = chunker_with(env)
total, caps = chunkers[settings[0]].capacity(lens)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(len(lens), dtype=torch.int64, device='cuda')
ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
lens = np.ascontiguousarray(lens, dtype=np.uint64)
last = np.ascontiguousarray(last if last is not None else np.zeros(len(lens)), dtype=np.uint64)
ref = None
res = {s: [] for s in settings}
for r in range(rounds):
    order = settings if r % 2 == 0 else settings[::-1]
    for s in order:
        ch = chunkers[s]
        for _ in range(2):
            ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(True)
        for _ in range(8):
            ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(False)
        t, e, c, k = ch.read_kernel_timing()
        res[s].append((t / k, c / k))
        # every schedule must give the same cut lists
        sig = (int(counts.sum().item()), int(cuts.sum().item()))
        if ref is None:
            ref = sig
        assert sig == ref, (s, sig, ref)
out = {'config': cfg, 'rounds': rounds}
for s, v in res.items():
    tm = np.array([x[0] for x in v])
    out[s] = {'tile_ms_median': round(float(np.median(tm)), 4), 'tile_ms_min': round(float(tm.min()), 4),
              'chain_ms_median': round(float(np.median([x[1] for x in v])), 4)}
print(json.dumps(out), flush=True)
