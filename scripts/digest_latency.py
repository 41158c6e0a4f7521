"""Digest-kernel latency vs occupancy: n messages of `size` bytes each (distinct offsets of one
buffer), one rc_blake2b_device launch, HIP-event timed.  Per-compression time of one quad =
t / (size / 128) when n is small."""
import json
import sys

import torch

sys.path.insert(0, '.')
from replicat_amd.hashing import SLOT, GpuBlake2b  # noqa: E402

torch.cuda.set_device(0)
size = int(sys.argv[1]) if len(sys.argv) > 1 else 5_120_000
h = GpuBlake2b(length=64)
stream = torch.cuda.current_stream()
buf = torch.randint(0, 255, (8 << 30,), dtype=torch.uint8, device='cuda')
out = torch.zeros((65536, SLOT), dtype=torch.uint8, device='cuda')
import os
NS = [int(x) for x in os.environ.get('N_LIST', '1,4,16,64,256,1024,4096,16384,32768,65536').split(',')]
for n in NS:
    stride = min(size, (8 << 30) // n) // 16 * 16
    ptrs = [buf.data_ptr() + (i * stride) % ((8 << 30) - size) for i in range(n)]
    lens = [size] * n
    h.digest_device(ptrs, lens, out.data_ptr(), stream.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    h.digest_device(ptrs, lens, out.data_ptr(), stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    blocks = (size + 127) // 128
    print(json.dumps({'n': n, 'size': size, 'ms': round(ms, 3),
                      'us_per_block': round(ms * 1e3 / blocks, 4),
                      'GBps': round(n * size / ms / 1e6, 1)}), flush=True)
