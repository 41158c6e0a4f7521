"""Diagnostic, step 2 of the placement study (scripts/placement_probe.py found every 4 GiB block
of a slow allocation read at the fast rate when each block is its own launch).  Per fresh 64 GiB
allocation, the streaming read probe over the whole arena in several shapes:

* one launch, tile orders: contiguous 16 MiB per wave (block 0, the tile kernel's order),
  interleaved runs of 1 / 64 / 256 tiles per wave (the concurrent window is then
  nw x run x 16 KiB: 64 MiB / 4 GiB / 16 GiB);
* k launches of 64/k GiB each (k = 2, 4, 16), contiguous order inside each.

If the slow allocations are slow only when one launch spans the whole arena, whatever the order,
the cause is not the access pattern.

    python scripts/placement_probe2.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from replicat_amd import synth  # noqa: E402
from replicat_amd.chunker import fill_splitmix_streams, read_probe  # noqa: E402

n, size = 1024, 64 << 20
NBYTES = n * size
hs = torch.cuda.current_stream().cuda_stream
out = torch.zeros(4, dtype=torch.int32, device='cuda')


def timed(fn, reps=5):
    fn()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return round(reps * NBYTES / (ev0.elapsed_time(ev1) * 1e-3) / 1e9, 1)


def whole(block):
    def f():
        os.environ['RC_PROBE_BLOCK'] = str(block)
        read_probe(base, NBYTES, out.data_ptr(), hs)
    return f


def split(k):
    part = NBYTES // k

    def f():
        os.environ['RC_PROBE_BLOCK'] = '0'
        for i in range(k):
            read_probe(base + i * part, part, out.data_ptr(), hs)
    return f


for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    pool = torch.empty(NBYTES + 64, dtype=torch.uint8, device='cuda')
    base = pool.data_ptr()
    fill_splitmix_streams(base, n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
    torch.cuda.synchronize()
    row = {'rep': rep}
    for b in (0, 1, 64, 256):
        row[f'one_launch_run{b}'] = timed(whole(b))
    for k in (2, 4, 16):
        row[f'{k}_launches'] = timed(split(k))
    row['one_launch_run0_again'] = timed(whole(0))
    os.environ.pop('RC_PROBE_BLOCK', None)
    print(json.dumps(row), flush=True)
    del pool
    torch.cuda.empty_cache()
