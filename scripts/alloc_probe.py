"""Diagnostic: does the arena's allocation history change the tile kernel's rate?  In one
process: allocate the config-2 arena, time the chunker (and the read probe); free it, allocate
again, time again; repeat."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams, read_probe  # noqa: E402

n, size = 1024, 64 << 20
slot = size
hs = torch.cuda.current_stream().cuda_stream
ch = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
total, caps = ch.capacity([size] * n)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
out = torch.zeros(4, dtype=torch.int32, device='cuda')
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    t0 = time.perf_counter()
    pool = torch.empty(n * slot + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, slot, synth.DEFAULT_SEED, 0, 1, hs)
    torch.cuda.synchronize()
    t_alloc = time.perf_counter() - t0
    ptrs = [pool.data_ptr() + i * slot for i in range(n)]
    for _ in range(2):
        ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs)
    torch.cuda.synchronize()
    ch.timing(True)
    for _ in range(10):
        ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs)
    torch.cuda.synchronize()
    ch.timing(False)
    t, e, c, k = ch.read_kernel_timing()
    probes = {}
    for block in ('0', '1', '4', '16'):
        os.environ['RC_PROBE_BLOCK'] = block
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        read_probe(pool.data_ptr(), n * size, out.data_ptr(), hs)
        ev0.record()
        for _ in range(5):
            read_probe(pool.data_ptr(), n * size, out.data_ptr(), hs)
        ev1.record()
        torch.cuda.synchronize()
        probes[block] = round(5 * n * size / (ev0.elapsed_time(ev1) * 1e-3) / 1e9, 1)
    os.environ.pop('RC_PROBE_BLOCK', None)
    print(json.dumps({'rep': rep, 'alloc_fill_s': round(t_alloc, 3), 'tile_ms': round(t / k, 3),
                      'chain_ms': round(c / k, 3), 'probe_gbs_by_block': probes}), flush=True)
    del pool
    torch.cuda.empty_cache()
