"""Diagnostic: when each wave of the tile kernel starts and ends (diag/lib_TSTAMPS.so, built with
-DRC_DIAG_TILE_STAMPS).  The kernel gives every wave the same number of tiles; how far apart the
waves finish is the time a dynamic tile hand-out could recover at the end of the launch.

    python -m replicat_amd.build --variant TSTAMPS -DRC_DIAG_TILE_STAMPS
    python scripts/tile_stamps.py [n_streams] [stream_mib] [min] [max]     (default: config 2)
    python scripts/tile_stamps.py harness                                  (the reference harness)
    STAMPS_PIPE=32 python scripts/tile_stamps.py harness     (pipelined calls: the tile kernel on
                                                              the CU-masked stream, 32 CUs reserved)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ['RC_LIB_PATH'] = os.path.join(ROOT, 'diag', 'lib_TSTAMPS.so')
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import _lib, synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams  # noqa: E402

hs = torch.cuda.current_stream().cuda_stream
last = None
if len(sys.argv) > 1 and sys.argv[1] == 'harness':  # the reference harness's one 5.12 GB stream
    pieces = list(synth.harness_buffers())
    size = sum(len(p) for p in pieces)
    pool = torch.empty(size + 64, dtype=torch.uint8, device='cuda')
    off = 0
    for p in pieces:
        pool[off:off + len(p)].copy_(torch.frombuffer(p, dtype=torch.uint8))
        off += len(p)
    n, mn, mx, ptrs, last = 1, 128_000, 5_120_000, [pool.data_ptr()], [size - len(pieces[-1])]
else:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    size = (int(sys.argv[2]) if len(sys.argv) > 2 else 64) << 20
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 128_000
    mx = int(sys.argv[4]) if len(sys.argv) > 4 else 5_120_000
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    ptrs = [pool.data_ptr() + i * size for i in range(n)]
    fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
ch = GpuChunker(mn, mx, b'\xff' * 16)
PIPE = int(os.environ.get('STAMPS_PIPE', '0') or 0)
if PIPE:
    ch.overlap(PIPE)
total, caps = ch.capacity([size] * n)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(n, dtype=torch.int64, device='cuda')
L = _lib.lib()
L.rc_diag_tile_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
waves = torch.cuda.get_device_properties(0).multi_processor_count * 16
for rep in range(4):
    ch.timing(True)
    ch.chunk_device(ptrs, [size] * n, last, cuts.data_ptr(), counts.data_ptr(), hs,
                    pipelined=bool(PIPE))
    ch.wait(hs)
    torch.cuda.synchronize()
    ch.timing(False)
    tile_ms = ch.read_kernel_timing()[0]
    buf = np.zeros(3 * waves, np.uint64)
    assert L.rc_diag_tile_read(buf.ctypes.data, waves) == 0
    s, e, k = buf[0::3].astype(np.int64), buf[1::3].astype(np.int64), buf[2::3]
    ok = e > 0
    s, e, k = s[ok], e[ok], k[ok]
    t0 = s.min()
    ends = (e - t0) / 100.0  # us (100 MHz)
    starts = (s - t0) / 100.0
    dur = ends - starts
    wg = np.nonzero(ok)[0] // 16
    xcd = wg % 8
    per_xcd = {int(x): round(float(np.median(ends[xcd == x])), 1) for x in range(8)}
    q = np.percentile(ends, [0, 1, 10, 50, 90, 99, 100])
    print(json.dumps({'rep': rep, 'tile_kernel_ms': round(tile_ms, 3), 'waves': int(ok.sum()),
                      'tiles_per_wave': [int(k.min()), int(k.max())],
                      'pipelined_reserve': PIPE,
                      'start_us_percentiles_50_90_99_100': [round(float(x), 1) for x in
                                                            np.percentile(starts, [50, 90, 99, 100])],
                      'end_us_percentiles_0_1_10_50_90_99_100': [round(float(x), 1) for x in q],
                      'tail_us_after_median_end': round(float(q[-1] - q[3]), 1),
                      'tail_frac_of_last_end': round(float((q[-1] - q[3]) / q[-1]), 4),
                      'duration_us_min_med_max': [round(float(x), 1) for x in
                                                  (dur.min(), np.median(dur), dur.max())],
                      'median_end_by_xcd_us': per_xcd}), flush=True)
