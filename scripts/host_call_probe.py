"""Host time per chunk_device call (descriptor staging, upload, launches, and the wait for the
workspace the call reuses) against the GPU step, for a batch of many streams: config 3 (iii)
(65,536 x 1 MiB) and config 2 (1024 x 64 MiB), in sequence and pipelined.  A call whose host
time approaches the step makes the host the bound.

    python scripts/host_call_probe.py [steps]
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
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
torch.cuda.set_stream(torch.cuda.Stream())
hs = torch.cuda.current_stream().cuda_stream
pool = torch.empty((64 << 30) + 64, dtype=torch.uint8, device='cuda')
fill_splitmix_streams(pool.data_ptr(), 1024, 64 << 20, 64 << 20, synth.DEFAULT_SEED, 0, 1, hs)
out = {}
for name, n, size, mn, mx in (('config3iii', 65536, 1 << 20, 2_000, 80_000),
                              ('config2', 1024, 64 << 20, 128_000, 5_120_000)):
    ch = GpuChunker(mn, mx, b'\xff' * 16)
    ptrs = np.arange(n, dtype=np.uint64) * size + pool.data_ptr()
    lens = np.full(n, size, dtype=np.uint64)
    last = np.zeros(n, dtype=np.uint64)
    total, caps = ch.capacity(lens)
    cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    for mode in ('seq', 'pipelined'):
        pip = mode == 'pipelined'
        for i in range(3):
            ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs,
                            pipelined=pip, end=pip and i == 2)
        ch.wait(hs)
        torch.cuda.synchronize()
        host, marks = [], []
        t0 = time.perf_counter()
        for i in range(K):
            a = time.perf_counter()
            ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs,
                            pipelined=pip, end=pip and i == K - 1)
            b = time.perf_counter()
            host.append((b - a) * 1e3)
            marks.append((round((a - t0) * 1e3, 3), round((b - t0) * 1e3, 3)))
        ch.wait(hs)
        torch.cuda.synchronize()
        step = (time.perf_counter() - t0) * 1e3 / K
        # the host's own share: calls timed with the GPU idle (each after a synchronize)
        idle = []
        for i in range(5):
            torch.cuda.synchronize()
            a = time.perf_counter()
            ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs,
                            pipelined=pip, end=pip)
            idle.append((time.perf_counter() - a) * 1e3)
            ch.wait(hs)
        torch.cuda.synchronize()
        out[f'{name}_{mode}'] = {'ms_per_step': round(step, 4),
                                 'host_ms_median': round(float(np.median(host)), 4),
                                 'host_ms_max': round(float(np.max(host)), 4),
                                 'host_ms_gpu_idle': round(float(np.median(idle)), 4),
                                 'pipelined_calls': ch.pipelined_calls(),
                                 'call_marks_ms': marks}
        print(json.dumps({f'{name}_{mode}': out[f'{name}_{mode}']}), flush=True)
print(json.dumps(out), flush=True)
