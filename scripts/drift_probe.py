"""Tile-kernel time over a long run of config-2 steps in ONE process (does a slow process stay
slow -- placement -- or speed up -- transient contention such as the driver clearing freed
VRAM?).  Prints the average step and tile-kernel time per block of steps.

    python scripts/drift_probe.py [blocks] [steps_per_block]
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams  # noqa: E402

blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 12
per = int(sys.argv[2]) if len(sys.argv) > 2 else 25
n, size = 1024, 64 << 20
torch.cuda.set_device(0)
t0 = time.perf_counter()
pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
hs = torch.cuda.current_stream().cuda_stream
fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
torch.cuda.synchronize()
ch = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
total, caps = ch.capacity([size] * n)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
ptrs = np.ascontiguousarray([pool.data_ptr() + i * size for i in range(n)], dtype=np.uint64)
lens = np.full(n, size, dtype=np.uint64)
last = np.zeros(n, dtype=np.uint64)
print(json.dumps({'alloc_fill_s': round(time.perf_counter() - t0, 3)}), flush=True)
for b in range(blocks):
    ch.timing(True)
    t = time.perf_counter()
    for _ in range(per):
        ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / per
    ch.timing(False)
    tile, edge, chain, calls = ch.read_kernel_timing()
    print(json.dumps({'block': b, 't_s': round(time.perf_counter() - t0, 2),
                      'step_ms': round(dt * 1e3, 3), 'tile_ms': round(tile / calls, 3)}), flush=True)
