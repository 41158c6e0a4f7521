"""A/B of pipelined steps (RC_PIPELINED: the chain on reserved CUs beside the next step's tile
kernel) against sequential steps, on ONE allocation (the per-allocation read-rate spread,
DESIGN §4, is larger than the effect).  Settings alternate round after round; per setting the
median wall time per step over K back-to-back steps, the tile kernel's HIP-event time and the
edge + chain time are printed.  Every setting must give the same cut lists.

    python scripts/overlap_ab.py [config] [rounds] [setting ...]   setting = seq | pR (R CUs)
                                          | mR (pipelined on R CUs, each step waits for its chain)
                                          [+full | +plain] (RC_TILE_MASK: the tile stream's mask)
                                          | pRx2 (R CUs, RC_TILE_STREAMS=2: two tile streams)
                                          [@STATIC:CHUNK[:DYN_MIN[:GROUP]]] (tile schedule: a
                                          chunker created with RC_TILE_STATIC / RC_TILE_CHUNK /
                                          RC_TILE_DYN_MIN / RC_TILE_GROUP, knobs.h)
    python scripts/overlap_ab.py 2 4 seq p8 p16 p32
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

cfg = sys.argv[1] if len(sys.argv) > 1 else '2'
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
settings = sys.argv[3:] or ['seq', 'p8', 'p16', 'p32']
K = int(os.environ.get('AB_STEPS', '10'))
TIMING = os.environ.get('AB_TIMING', '1') == '1'  # 0: wall clock only (no HIP events per call)
torch.cuda.set_stream(torch.cuda.Stream())  # not the NULL stream (it syncs with the masked streams)
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
    mn, mx = 128_000, 5_120_000
else:
    n, size, mn, mx = {'2': (1024, 64 << 20, 128_000, 5_120_000),
                       '3ii': (1, 64 << 30, 128_000, 5_120_000),
                       '3iii': (65536, 1 << 20, 2_000, 80_000),
                       '4': (16, 8 << 30, 128_000, 5_120_000)}[cfg]
    pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
    fill_splitmix_streams(pool.data_ptr(), n, size, size, synth.DEFAULT_SEED, 0, 1, hs)
    ptrs = np.arange(n, dtype=np.uint64) * size + pool.data_ptr()
    lens, last = [size] * n, ([size - (1 << 20)] if cfg == '3ii' else None)


def chunker_with(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return GpuChunker(mn, mx, b'\xff' * 16)  # knobs are read here
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


def chunker_key(s):
    base, _, sched = s.partition('@')
    base, _, mask = base.partition('+')  # p32+full / p32+plain: RC_TILE_MASK
    return sched + ('x2' if base.endswith('x2') else '') + ('+' + mask if mask else '')


chunkers = {}
for s in settings:
    key = chunker_key(s)
    if key not in chunkers:
        sched = s.partition('@')[2]
        env = {}
        if sched:  # STATIC:CHUNK[:DYN_MIN]
            parts = sched.split(':')
            env.update({'RC_TILE_STATIC': parts[0], 'RC_TILE_CHUNK': parts[1]})
            if len(parts) > 2:
                env['RC_TILE_DYN_MIN'] = parts[2]
            if len(parts) > 3:
                env['RC_TILE_GROUP'] = parts[3]
        if 'x2' in key:
            env['RC_TILE_STREAMS'] = '2'
        if '+' in key:
            env['RC_TILE_MASK'] = key.partition('+')[2]
        chunkers[key] = chunker_with(env)
ch = next(iter(chunkers.values()))
total, caps = ch.capacity(lens)
cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
counts = torch.zeros(len(lens), dtype=torch.int64, device='cuda')
ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
lens = np.ascontiguousarray(lens, dtype=np.uint64)
last = np.ascontiguousarray(last if last is not None else np.zeros(len(lens)), dtype=np.uint64)
w = torch.arange(total, dtype=torch.int64, device='cuda') % 1000003
ref = None
res = {s: [] for s in settings}
for r in range(rounds):
    order = settings if r % 2 == 0 else settings[::-1]
    for s in order:
        base, _, sched = s.partition('@')  # ...@STATIC:CHUNK -- the tile schedule's chunker
        base = base.partition('+')[0]
        ch = chunkers[chunker_key(s)]
        pipe = base != 'seq'
        # mR: pipelined on R reserved CUs, but each step waits for its own chain before the next
        # (isolates the masked tile launch from a chain running beside it)
        isolated = base.startswith('m')
        if pipe:
            ch.overlap(int(base[1:].split(':')[0].removesuffix('x2')))

        def step():
            ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs,
                            pipelined=pipe)
            if isolated:
                ch.wait(hs)
                torch.cuda.current_stream().synchronize()
        cuts.zero_()
        for _ in range(2):
            step()
        ch.wait(hs)
        torch.cuda.synchronize()
        ch.timing(TIMING)
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        ch.wait(hs)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3 / K
        ch.timing(False)
        t, e, c, k = ch.read_kernel_timing()
        k = max(k, 1)
        res[s].append((el, t / k, (e + c) / k))
        ch.check()  # no fail-safe stop of a group grab
        sig = (int(counts.sum().item()), int(cuts.sum().item()), int((cuts * w).sum().item()))
        if ref is None:
            ref = sig
        assert sig == ref, (s, sig, ref)
out = {'config': cfg, 'rounds': rounds, 'steps': K, 'cuts': ref[0],
       'bytes': int(np.sum(lens))}
for s, v in res.items():
    a = np.array(v)
    med = np.median(a, axis=0)
    out[s] = {'ms_per_step': round(float(med[0]), 4), 'ms_per_step_min': round(float(a[:, 0].min()), 4),
              'tile_ms': round(float(med[1]), 4), 'edge_chain_ms': round(float(med[2]), 4),
              'GiBps': round(float(np.sum(lens)) / (med[0] * 1e-3) / 2**30, 1)}
print(json.dumps(out), flush=True)
torch.cuda.synchronize()
for c in chunkers.values():
    c.close()  # the CU-masked streams go while the runtime is up (the library would at exit)
