"""The tile kernel's fail-safe stop is loud on every product surface.

With workgroup grabs (kernels.hip UnitGrab) a wave whose group slot is never published stops
after ~1 s -- or at once when its slot was overwritten -- instead of hanging the GPU, and the
launch's records are then incomplete.  The edge kernel turns the flag into the call's fault
stamp, the chain kernels write RC_COUNT_FAULT for every stream and walk nothing, and each
surface raises ChunkerFault instead of returning cuts: the blocking C entry points return
RC_ERR_DEVICE_FAULT, and readers of device counts go through check_counts.

The stop has never been seen on the product library, so it is forced: diag/lib_GRABFAULT.so
(-DRC_DIAG_GRAB_FAULT, built by __graft_entry__.build()) stops wave 1 of workgroup 0 at its
first grab -- the unit it took is never run -- in every launch.  One child process (the library
is chosen at import through RC_LIB_PATH) drives every surface once and reports what each did;
each test below checks one surface.  The last tests run the PRODUCT library the same way and
check that nothing faults (the flag, stamp and count words stay clear call after call)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAULT_LIB = os.path.join(ROOT, 'diag', 'lib_GRABFAULT.so')

CHILD = textwrap.dedent("""
    import json, os, sys, tempfile, traceback
    sys.path.insert(0, {root!r})
    import numpy as np
    import torch
    from replicat_amd import _lib, synth
    from replicat_amd.chunker import (ChunkerFault, GpuChunker, check_counts, counts_host,
                                      fill_splitmix_streams)
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    hs = torch.cuda.current_stream().cuda_stream
    out = {{'lib': _lib.LIB_PATH}}

    def run(name, fn):
        try:
            out[name] = {{'ok': True, 'value': fn()}}
        except ChunkerFault as e:
            out[name] = {{'ok': False, 'fault': True, 'msg': str(e)[:300]}}
        except Exception as e:
            out[name] = {{'ok': False, 'fault': False, 'msg': repr(e)[:300],
                          'tb': traceback.format_exc()[-1500:]}}

    def arena(n, size, seed=0x5EED):
        pool = torch.empty(n * size + 64, dtype=torch.uint8, device='cuda')
        fill_splitmix_streams(pool.data_ptr(), n, size, size, seed, 0, 1, hs)
        return pool, [pool.data_ptr() + i * size for i in range(n)]

    def device_call(mn, mx, n, size, pipelined=False, seg=None):
        if seg:
            os.environ['RC_SEGMENT_BYTES'] = str(seg)
        ch = GpuChunker(mn, mx, b'\\xff' * 16)
        os.environ.pop('RC_SEGMENT_BYTES', None)
        pool, ptrs = arena(n, size)
        total, caps = ch.capacity([size] * n)
        cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
        counts = torch.full((n,), 12345, dtype=torch.int64, device='cuda')
        for _ in range(2):  # two calls: both workspaces
            ch.chunk_device(ptrs, [size] * n, None, cuts.data_ptr(), counts.data_ptr(), hs,
                            pipelined=pipelined, end=True)
        ch.wait(hs)
        torch.cuda.synchronize()
        raw = counts.cpu().numpy()
        out[name_of(mn, n, pipelined, seg) + '_raw'] = sorted(set(int(c) for c in raw))
        counts_host(counts)  # raises on RC_COUNT_FAULT
        return int(raw.sum())

    def name_of(mn, n, pipelined, seg):
        return 'device_%d_%d_%s_%s' % (mn, n, 'piped' if pipelined else 'seq', seg or 0)

    # rc_chunk_device: the wave-per-stream chain, pipelined, segmented (spec / merge / scan /
    # copy / join), and the quad chain of many small-window streams
    run('chunk_device', lambda: device_call(128_000, 5_120_000, 16, 16 << 20))
    run('chunk_device_pipelined', lambda: device_call(128_000, 5_120_000, 16, 16 << 20, True))
    run('chunk_device_segments', lambda: device_call(2_000, 80_000, 4, 16 << 20, seg=1 << 20))
    run('chunk_device_quads', lambda: device_call(2_000, 80_000, 1024, 1 << 20))

    def check_twice():
        ch = GpuChunker(2_000, 80_000, b'\\xff' * 16)
        pool, ptrs = arena(4, 4 << 20)
        total, _ = ch.capacity([4 << 20] * 4)
        cuts = torch.zeros(total, dtype=torch.int64, device='cuda')
        counts = torch.zeros(4, dtype=torch.int64, device='cuda')
        for _ in range(3):
            ch.chunk_device(ptrs, [4 << 20] * 4, None, cuts.data_ptr(), counts.data_ptr(), hs)
        first = None
        try:
            ch.check()
        except ChunkerFault as e:
            first = str(e)
        ch.check()  # nothing since the last check: the count restarted
        return first
    run('check', check_twice)

    data = np.frombuffer(synth.stream_bytes(12 << 20, synth.DEFAULT_SEED, 3), dtype=np.uint8)
    run('next_cut', lambda: GpuChunker(128_000, 5_120_000, b'\\xff' * 16).next_cut(data, False))
    import _replicat_adapters as RA
    run('dropin_next_cut', lambda: RA._gclmulchunker(128_000, 5_120_000, b'\\xff' * 16)
        .next_cut(data.tobytes(), True))
    run('chunk_host', lambda: len(GpuChunker(128_000, 5_120_000, b'\\xff' * 16)
                                  .chunk_host([data], [len(data) - 1000])[0]))
    from replicat_amd.hashing import GpuBlake2b, chunk_digest_host
    run('chunk_digest_host', lambda: len(chunk_digest_host(
        GpuChunker(128_000, 5_120_000, b'\\xff' * 16), GpuBlake2b(), [data])[0][0]))
    from replicat_amd.adapters import gclmulchunker
    pieces = [data[i:i + (4 << 20)].tobytes() for i in range(0, len(data), 4 << 20)]
    run('adapter_call', lambda: sum(len(c) for c in gclmulchunker(batch_bytes=1 << 20)(
        iter(pieces), params=b'')))
    run('tile_records', lambda: len(GpuChunker(2_000, 80_000, b'\\xff' * 16).tile_records(
        [arena(1, 4 << 20)[1][0]], [4 << 20])[0]))

    from replicat_amd.pipeline import DeviceSnapshotProducer
    tmp = tempfile.mkdtemp()
    paths = []
    for i in range(3):
        p = os.path.join(tmp, 'f%d' % i)
        with open(p, 'wb') as f:
            f.write(synth.stream_bytes((3 + i) << 20, synth.DEFAULT_SEED, 50 + i))
        paths.append(p)
    run('producer_run', lambda: len(DeviceSnapshotProducer(
        min_length=128_000, max_length=1_000_000, batch_bytes=4 << 20).run(paths).chunks))

    def stream_all():
        prod = DeviceSnapshotProducer(min_length=128_000, max_length=1_000_000, batch_bytes=4 << 20)
        n = 0
        with prod.stream(paths) as s:
            for rec in s:
                rec.release()
                n += 1
        return n
    run('producer_stream', stream_all)
    print('RESULT ' + json.dumps(out), flush=True)
""")


def _child(lib):
    env = dict(os.environ)
    if lib:
        env['RC_LIB_PATH'] = lib
    else:
        env.pop('RC_LIB_PATH', None)
    p = subprocess.run([sys.executable, '-u', '-c', CHILD.format(root=ROOT)], capture_output=True,
                       text=True, timeout=240, env=env, cwd=ROOT)
    line = [x for x in p.stdout.splitlines() if x.startswith('RESULT ')]
    assert p.returncode == 0 and line, (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    return json.loads(line[0][7:])


@pytest.fixture(scope='module')
def faulted():
    if not os.path.exists(FAULT_LIB):
        pytest.fail(f'{FAULT_LIB} missing: __graft_entry__.build() builds it')
    return _child(FAULT_LIB)


@pytest.fixture(scope='module')
def product():
    return _child(None)


SURFACES = ['chunk_device', 'chunk_device_pipelined', 'chunk_device_segments',
            'chunk_device_quads', 'next_cut', 'dropin_next_cut', 'chunk_host',
            'chunk_digest_host', 'adapter_call', 'tile_records', 'producer_run',
            'producer_stream']


@pytest.mark.parametrize('surface', SURFACES)
def test_fault_raises(faulted, surface):
    """The forced stop reaches the caller as ChunkerFault -- never as cuts."""
    r = faulted[surface]
    assert faulted['lib'].endswith('lib_GRABFAULT.so')
    assert not r['ok'], f'{surface} returned {r.get("value")!r} from a faulted launch'
    assert r['fault'], r


def test_fault_counts_are_the_sentinel(faulted):
    """rc_chunk_device writes RC_COUNT_FAULT (-3) for EVERY stream of a faulted call, whatever
    chain kernel ran (wave per stream, segments + scan, quads; pipelined or not)."""
    raws = {k: v for k, v in faulted.items() if k.endswith('_raw')}
    assert len(raws) == 4, raws
    for k, v in raws.items():
        assert v == [-3], (k, v)


def test_check_reports_once_then_clears(faulted):
    r = faulted['check']
    assert r['ok'] and r['value'] and '3 call(s)' in r['value'], r


def test_product_library_never_faults(product):
    """The same calls on the product library: results, no fault; rc_chunker_check stays clear."""
    assert product['lib'].endswith('libreplicat_chunker.so')
    for s in SURFACES + ['check']:
        assert product[s]['ok'], (s, product[s])
    assert product['check']['value'] is None
    for k, v in product.items():
        if k.endswith('_raw'):
            assert min(v) >= 0, (k, v)


def test_bench_exits_nonzero_on_fault():
    """bench.py checks every call (rc_chunker_check after the timed region, the counts before
    the parity digest): on the faulting library it prints no line and exits non-zero."""
    if not os.path.exists(FAULT_LIB):
        pytest.fail(f'{FAULT_LIB} missing')
    env = dict(os.environ, RC_LIB_PATH=FAULT_LIB)
    p = subprocess.run([sys.executable, '-u', 'bench.py', '--streams', '8', '--stream-mib', '64',
                        '--steps', '2', '--warmup', '1', '--cpu-streams', '0'],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode != 0, p.stdout[-2000:]
    assert '"metric"' not in p.stdout
    assert 'ChunkerFault' in p.stderr, p.stderr[-2000:]
