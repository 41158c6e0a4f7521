"""The drop-in path's own rate: replicat's adapter loop
(adapters.py:287-303, restated in oracle/adapter_loop.py) over

* the HIP ``_gclmulchunker`` (replicat_amd._replicat_adapters: one rc_next_cut per chunk), and
* the reference's own ``_gclmulchunker`` (oracle/_ref, compiled from src/adapters.cpp),

on config 1's stream (256 MiB in 16 MiB pieces, as Repository.snapshot reads a file) and on the
reference harness stream (10 x 512,000,000 B pieces).  Reports, per chunker: GiB/s of the whole
loop, the time inside next_cut, calls per second, and bytes uploaded per byte chunked (the HIP
path copies min(size, 4 * window + 4) bytes per argmax call).  The cut lists must agree.

    python scripts/dropin_probe.py [--workload config1|harness|both] [--repeat R]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle.adapter_loop import adapter_chunks  # noqa: E402
from replicat_amd import synth  # noqa: E402

GIB = 1 << 30
MIN_LEN, MAX_LEN = 128_000, 5_120_000


class Timed:
    """A next_cut wrapper that counts calls, argmax calls and time inside the native call."""

    def __init__(self, native):
        self.native, self.t, self.calls, self.uploaded = native, 0.0, 0, 0
        self.window = (MAX_LEN - 1) // 4

    def next_cut(self, buf, final):
        n = len(buf)
        if not (final and n < 2 * MAX_LEN) and not (not final and n < MAX_LEN):
            self.uploaded += min(n, 4 * self.window + 4)
        t0 = time.perf_counter()
        r = self.native.next_cut(buf, final)
        self.t += time.perf_counter() - t0
        self.calls += 1
        return r


def run(native, pieces, repeat):
    best = None
    for _ in range(repeat):
        tn = Timed(native)
        t0 = time.perf_counter()
        lens = [len(c) for c in adapter_chunks(tn, pieces)]
        dt = time.perf_counter() - t0
        if best is None or dt < best[0]:
            best = (dt, tn, lens)
    dt, tn, lens = best
    total = sum(lens)
    return {'loop_gibs': round(total / dt / GIB, 3), 'loop_s': round(dt, 4),
            'next_cut_s': round(tn.t, 4), 'next_cut_gibs': round(total / tn.t / GIB, 3),
            'calls': tn.calls, 'calls_per_s': round(tn.calls / tn.t, 1),
            'chunks': len(lens), 'uploaded_per_byte': round(tn.uploaded / total, 3)}, lens


def ref_native():
    sys.path.insert(0, ROOT)
    import bench
    return bench._ref_chunker(MIN_LEN, MAX_LEN, b'\xff' * 16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='both', choices=['config1', 'harness', 'both'])
    ap.add_argument('--repeat', type=int, default=3)
    args = ap.parse_args()
    from replicat_amd._replicat_adapters import _gclmulchunker
    hip = _gclmulchunker(MIN_LEN, MAX_LEN, b'\xff' * 16)
    ref = ref_native()
    loads = []
    if args.workload in ('config1', 'both'):
        data = synth.stream_bytes(256 << 20, synth.DEFAULT_SEED, 0)
        loads.append(('config1: 256 MiB in 16 MiB pieces',
                      [data[k:k + (16 << 20)].tobytes() for k in range(0, len(data), 16 << 20)]))
    if args.workload in ('harness', 'both'):
        loads.append(('harness: 10 x 512,000,000 B Random(0)', list(synth.harness_buffers())))
    for name, pieces in loads:
        # warm the device path (first call builds workspaces)
        list(adapter_chunks(hip, [pieces[0][:2 * MAX_LEN + 8]]))
        out = {'workload': name, 'bytes': sum(len(p) for p in pieces)}
        rh, lh = run(hip, pieces, args.repeat)
        out['hip_dropin'] = rh
        if ref is not None:
            rr, lr = run(ref, pieces, args.repeat)
            out['reference_so'] = rr
            out['identical'] = lh == lr
            out['speedup_loop'] = round(rr['loop_s'] / rh['loop_s'], 3)
            out['speedup_next_cut'] = round(rr['next_cut_s'] / rh['next_cut_s'], 3)
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
