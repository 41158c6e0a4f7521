"""Diagnostic: why the same build reads one 64 GiB allocation ±5-10 % faster
than another (profiles/r02/placement/).

Per repetition, one fresh allocation of the config-2 arena (1024 x 64 MiB) of each kind:

* ``torch``      -- torch's caching allocator after empty_cache(): a fresh hipMalloc;
* ``contiguous`` -- hipExtMallocWithFlags(hipDeviceMallocContiguous): one physically contiguous
                    range (when the driver can find one; "failed" otherwise);

filled with the config-2 streams, then timed with HIP events: the streaming read probe over the
whole arena, the read probe over each 4 GiB block of it (is a slow allocation slow everywhere or
in a few blocks?), and the config-2 tile kernel.  Run it again under
``rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum`` to see whether the slow
allocations are the ones whose reads miss the L1 TLB more (small physical fragments).

    python scripts/placement_probe.py [reps] [kinds]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams, read_probe  # noqa: E402

n, size = 1024, 64 << 20
NBYTES = n * size
BLOCK = 4 << 30
hs = torch.cuda.current_stream().cuda_stream
ch = GpuChunker(128_000, 5_120_000, b'\xff' * 16)
total, caps = ch.capacity([size] * n)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
out = torch.zeros(4, dtype=torch.int32, device='cuda')
hip = ctypes.CDLL('libamdhip64.so')
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]


def probe_gbs(ptr, nbytes, reps=5):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    read_probe(ptr, nbytes, out.data_ptr(), hs)
    ev0.record()
    for _ in range(reps):
        read_probe(ptr, nbytes, out.data_ptr(), hs)
    ev1.record()
    torch.cuda.synchronize()
    return round(reps * nbytes / (ev0.elapsed_time(ev1) * 1e-3) / 1e9, 1)


def measure(base):
    fill_splitmix_streams(base, n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
    ptrs = [base + i * size for i in range(n)]
    for _ in range(2):
        ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs)
    torch.cuda.synchronize()
    ch.timing(True)
    for _ in range(10):
        ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs)
    torch.cuda.synchronize()
    ch.timing(False)
    t, _, _, k = ch.read_kernel_timing()
    whole = probe_gbs(base, NBYTES)
    blocks = [probe_gbs(base + b, BLOCK) for b in range(0, NBYTES, BLOCK)]
    return {'tile_ms': round(t / k, 3), 'probe_gbs': whole,
            'probe_gbs_per_4gib': blocks,
            'block_spread': round(max(blocks) / min(blocks), 3)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    kinds = (sys.argv[2] if len(sys.argv) > 2 else 'torch,contiguous').split(',')
    for rep in range(reps):
        for kind in kinds:
            row = {'rep': rep, 'kind': kind}
            if kind == 'torch':
                pool = torch.empty(NBYTES + 64, dtype=torch.uint8, device='cuda')
                row.update(measure(pool.data_ptr()))
                row['va'] = hex(pool.data_ptr())
                del pool
                torch.cuda.empty_cache()
            else:
                flag = {'contiguous': 0x4, 'default': 0x0}[kind]
                p = ctypes.c_void_p()
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), NBYTES + 64, flag)
                if rc != 0:
                    row['failed'] = rc
                else:
                    row.update(measure(p.value))
                    row['va'] = hex(p.value)
                    torch.cuda.synchronize()
                    hip.hipFree(p)
            print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
