"""Time the BLAKE2b chunk digests on config 2 (1024 x 64 MiB, default params): chunk once,
then digest the chunks N times (HIP events around the digest kernels)."""
import json
import sys
import time

import torch

sys.path.insert(0, '.')
from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix  # noqa: E402
from replicat_amd.hashing import SLOT, GpuBlake2b  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
mib = int(sys.argv[2]) if len(sys.argv) > 2 else 64
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 128_000
mx = int(sys.argv[4]) if len(sys.argv) > 4 else 5_120_000
size = mib << 20
torch.cuda.set_device(0)
hs = torch.cuda.current_stream().cuda_stream
pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
ptrs = [pool.data_ptr() + i * size for i in range(n)]
for i, p in enumerate(ptrs):
    fill_splitmix(p, size, synth.DEFAULT_SEED, i, hs)
ch = GpuChunker(mn, mx, b'\xff' * 16)
h = GpuBlake2b(length=64)
lens = [size] * n
total, caps = ch.capacity(lens)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
dig = torch.zeros((total, SLOT), dtype=torch.uint8, device='cuda')
ch.chunk_device(ptrs, lens, None, cuts.data_ptr(), counts.data_ptr(), hs)
torch.cuda.synchronize()
nchunks = int(counts.sum().item())
h.digest_chunks(ch, ptrs, lens, cuts.data_ptr(), counts.data_ptr(), dig.data_ptr(), hs)
torch.cuda.synchronize()
h.timing(True)
t0 = time.perf_counter()
reps = 3
for _ in range(reps):
    h.digest_chunks(ch, ptrs, lens, cuts.data_ptr(), counts.data_ptr(), dig.data_ptr(), hs)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / reps
ms, calls = h.read_timing()
ms /= max(calls, 1)
print(json.dumps({'streams': n, 'stream_mib': mib, 'min': mn, 'max': mx, 'chunks': nchunks,
                  'digest_ms': round(ms, 3), 'wall_ms': round(wall * 1e3, 3),
                  'gib_s': round(n * size / (ms * 1e-3) / 2**30, 1)}), flush=True)
