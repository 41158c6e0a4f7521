"""Config 3 (iii) against config 2 on ONE allocation ("within 3 % of config 2 on one
allocation"): one 64 GiB arena of splitmix bytes, chunked alternately as config 2 (1024 x 64
MiB, replicat's defaults, pipelined steps as bench.py runs them) and as config 3 (iii) (65,536 x
1 MiB of the same bytes, min 2,000 / max 80,000: the library runs small-window requests in
sequence), K back-to-back steps each, rounds in ABBA order; median wall ms per step, the tile
kernel's HIP-event time and the bytes each reads.

    python scripts/c2_vs_3iii.py [rounds] [steps] [--piped]

--piped (round 6): also config 3 (iii) on a chunker created with RC_PIPE_ALL=1, so that its
steps overlap as config 2's do -- the three setups on the same allocation.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams, keys_needed  # noqa: E402

argv = [a for a in sys.argv[1:] if not a.startswith('--')]
rounds = int(argv[0]) if len(argv) > 0 else 4
K = int(argv[1]) if len(argv) > 1 else 10
PIPED = '--piped' in sys.argv
torch.cuda.set_stream(torch.cuda.Stream())
hs = torch.cuda.current_stream().cuda_stream
GIB = 1 << 30
pool = torch.empty((64 << 30) + 64, dtype=torch.uint8, device='cuda')
fill_splitmix_streams(pool.data_ptr(), 1024, 64 << 20, 64 << 20, synth.DEFAULT_SEED, 0, 1, hs)
setups = {}
cases = [('config2', 1024, 64 << 20, 128_000, 5_120_000),
         ('config3iii', 65536, 1 << 20, 2_000, 80_000)]
if PIPED:
    cases.append(('config3iii_piped', 65536, 1 << 20, 2_000, 80_000))
for name, n, size, mn, mx in cases:
    if name.endswith('_piped'):  # knobs are read when the chunker is created
        os.environ['RC_PIPE_ALL'] = '1'
    ch = GpuChunker(mn, mx, b'\xff' * 16)
    os.environ.pop('RC_PIPE_ALL', None)
    total, caps = ch.capacity([size] * n)
    j = keys_needed(mx, size, 0)
    setups[name] = dict(
        ch=ch, n=n, size=size,
        ptrs=np.arange(n, dtype=np.uint64) * size + pool.data_ptr(),
        lens=np.full(n, size, dtype=np.uint64), last=np.zeros(n, dtype=np.uint64),
        cuts=torch.zeros(total, dtype=torch.int64, device='cuda'),
        counts=torch.zeros(n, dtype=torch.int64, device='cuda'),
        read=n * min(size, 4 * j + 4))
res = {k: [] for k in setups}
for r in range(rounds):
    for name in (list(setups) if r % 2 == 0 else list(setups)[::-1]):
        S = setups[name]
        ch = S['ch']

        def step(end=False):
            ch.chunk_device(S['ptrs'], S['lens'], S['last'], S['cuts'].data_ptr(),
                            S['counts'].data_ptr(), hs, pipelined=True, end=end)
        for i in range(2):
            step(end=i == 1)
        ch.wait(hs)
        torch.cuda.synchronize()
        ch.timing(True)
        t0 = time.perf_counter()
        for i in range(K):
            step(end=i == K - 1)
        ch.wait(hs)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3 / K
        ch.timing(False)
        t, e, c, k = ch.read_kernel_timing()
        res[name].append((el, t / max(k, 1), ch.pipelined_calls()))
out = {'rounds': rounds, 'steps': K, 'arena_bytes': 64 << 30}
for name, v in res.items():
    a = np.array(v, dtype=float)
    med = np.median(a[:, :2], axis=0)
    out[name] = {'ms_per_step': round(float(med[0]), 4), 'tile_ms': round(float(med[1]), 4),
                 'GiBps': round((64 << 30) / (med[0] * 1e-3) / GIB, 1),
                 'bytes_read': setups[name]['read'], 'pipelined_calls': int(a[-1, 2])}
out['3iii_over_config2'] = round(out['config3iii']['ms_per_step'] / out['config2']['ms_per_step'], 4)
if PIPED:
    out['3iii_piped_over_config2'] = round(out['config3iii_piped']['ms_per_step'] /
                                           out['config2']['ms_per_step'], 4)
print(json.dumps(out), flush=True)
