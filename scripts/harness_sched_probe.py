"""Where a short tile launch (the reference harness: one 5.12 GB stream, ~87 tiles per wave)
loses its rate.  In ONE process on ONE allocation, per tile schedule: the
tile kernel's HIP-event time over sequential calls, the streaming read probe under the same
schedule over the same bytes (rc_chunker_read_probe: its ceiling), and -- when the library is the
TSTAMPS diagnostic build (RC_LIB_PATH=diag/lib_TSTAMPS.so) -- every wave's start and end
(s_memrealtime) and tile count.  Settings alternate round after round (ABBA).

    python scripts/harness_sched_probe.py [harness|2|3ii|3iii|4] [rounds] SETTING ...
        SETTING = STATIC:CHUNK:DYN_MIN:GROUP   (RC_TILE_STATIC / CHUNK / DYN_MIN / GROUP)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from replicat_amd import _lib, synth  # noqa: E402
from replicat_amd.chunker import GpuChunker, fill_splitmix_streams  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'harness'
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
settings = sys.argv[3:] or ['1000:12:128:0', '100:12:0:0', '100:3:0:32']
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
    MN, MX = 128_000, 5_120_000
else:
    n, size, MN, MX = {'2': (1024, 64 << 20, 128_000, 5_120_000),
                       '3ii': (1, 64 << 30, 128_000, 5_120_000),
                       '3iii': (65536, 1 << 20, 2_000, 80_000),
                       '4': (16, 8 << 30, 128_000, 5_120_000)}[cfg]
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
    ptrs, lens = list(np.arange(n, dtype=np.uint64) * size + pool.data_ptr()), [size] * n
    last = [size - (1 << 20)] if cfg == '3ii' else None
nbytes = int(sum(lens))
L_ = _lib.lib()
stamped = hasattr(L_, 'rc_diag_tile_read')
if stamped:
    L_.rc_diag_tile_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
waves_max = torch.cuda.get_device_properties(0).multi_processor_count * 16


def chunker_with(s):
    st, ck, dm, gp = s.split(':')
    env = {'RC_TILE_STATIC': st, 'RC_TILE_CHUNK': ck, 'RC_TILE_DYN_MIN': dm, 'RC_TILE_GROUP': gp}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return GpuChunker(MN, MX, b'\xff' * 16)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


chunkers = {s: chunker_with(s) for s in settings}
total, caps = chunkers[settings[0]].capacity(lens)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(len(lens), dtype=torch.int64, device='cuda')
out = torch.zeros(4, dtype=torch.int32, device='cuda')
P = np.ascontiguousarray(ptrs, dtype=np.uint64)
N = np.ascontiguousarray(lens, dtype=np.uint64)
Z = np.ascontiguousarray(last if last is not None else np.zeros(len(lens)), dtype=np.uint64)
res = {s: {'tile_ms': [], 'probe_ms': [], 'stamps': []} for s in settings}
ref = None
for r in range(rounds):
    for s in (settings if r % 2 == 0 else settings[::-1]):
        ch = chunkers[s]
        ch.chunk_device(P, N, Z, cuts.data_ptr(), counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(True)
        for _ in range(6):
            ch.chunk_device(P, N, Z, cuts.data_ptr(), counts.data_ptr(), hs)
        torch.cuda.synchronize()
        ch.timing(False)
        ch.check()
        t, e, c, k = ch.read_kernel_timing()
        res[s]['tile_ms'].append(t / k)
        sig = (int(counts.sum().item()), int(cuts.sum().item()))
        ref = ref or sig
        assert sig == ref, (s, sig, ref)
        if stamped:  # the last call's waves
            buf = np.zeros(3 * waves_max, np.uint64)
            assert L_.rc_diag_tile_read(buf.ctypes.data, waves_max) == 0
            st, en, kk = buf[0::3].astype(np.int64), buf[1::3].astype(np.int64), buf[2::3]
            ok = en > 0
            t0 = st[ok].min()
            ends = (en[ok] - t0) / 100.0
            q = np.percentile(ends, [0, 10, 50, 90, 100])
            starts = (st[ok] - t0) / 100.0
            # round 6: per workgroup (16 waves), when its first and last wave ended
            wg = np.arange(len(en))[ok] // 16
            wg_first = np.array([ends[wg == g].min() for g in np.unique(wg)])
            wg_last = np.array([ends[wg == g].max() for g in np.unique(wg)])
            res[s]['stamps'].append({'end_us_0_10_50_90_100': [round(float(x), 1) for x in q],
                                     'mean_end_us': round(float(ends.mean()), 1),
                                     'start_us_0_50_100': [round(float(x), 1) for x in
                                                           np.percentile(starts, [0, 50, 100])],
                                     'wg_last_end_us_0_50_100': [round(float(x), 1) for x in
                                                                 np.percentile(wg_last, [0, 50, 100])],
                                     'wg_spread_us_median': round(float(np.median(wg_last - wg_first)), 1),
                                     'tiles_min_max': [int(kk[ok].min()), int(kk[ok].max())]})
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ch.read_probe(pool.data_ptr(), nbytes, out.data_ptr(), hs)
        ev0.record()
        for _ in range(6):
            ch.read_probe(pool.data_ptr(), nbytes, out.data_ptr(), hs)
        ev1.record()
        torch.cuda.synchronize()
        res[s]['probe_ms'].append(ev0.elapsed_time(ev1) / 6)
summary = {'config': cfg, 'bytes': nbytes, 'rounds': rounds, 'stamped': stamped}
for s, v in res.items():
    tm, pm = np.median(v['tile_ms']), np.median(v['probe_ms'])
    summary[s] = {'tile_ms': round(float(tm), 4), 'tile_GBps': round(nbytes / tm / 1e6, 1),
                  'probe_ms': round(float(pm), 4), 'probe_GBps': round(nbytes / pm / 1e6, 1),
                  'tile_over_probe': round(float(pm / tm), 4)}
    if v['stamps']:
        summary[s]['stamps_last_round'] = v['stamps'][-1]
print(json.dumps(summary), flush=True)
