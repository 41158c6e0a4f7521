"""Time the device snapshot producer end to end (SURVEY §8 d config 1 and a larger file set).

    python scripts/producer_probe.py [total_mib] [files]

Writes `files` files of random bytes (total `total_mib` MiB; default one 256 MiB file = config 1)
under $TMPDIR, then times DeviceSnapshotProducer.run over them (page-cache reads, as a repeated
snapshot sees them): unencrypted and encrypted, contents kept as replicat's upload queue needs
them.  The CPU leg of the same work (the oracle's chunker over the framed stream + hashlib
BLAKE2b per chunk and per file, one core) is timed beside it as the baseline; it is the checker,
not the measured path.  One JSON line per variant.
"""
import hashlib
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, '.')
import torch  # noqa: E402

from oracle import oracle as o  # noqa: E402
from replicat_amd import snapshot  # noqa: E402
import importlib  # noqa: E402

# RC_PRODUCER_MODULE: time another producer module (an A/B of two versions on one box)
_mod = importlib.import_module(os.environ.get('RC_PRODUCER_MODULE', 'replicat_amd.pipeline'))
ChunkEncryption, DeviceSnapshotProducer = _mod.ChunkEncryption, _mod.DeviceSnapshotProducer

total_mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
nfiles = int(sys.argv[2]) if len(sys.argv) > 2 else 1
MIN, MAX = 128_000, 5_120_000
GIB = float(1 << 30)

torch.cuda.set_device(0)
tmp = tempfile.mkdtemp(prefix='rc_probe_')
paths, sizes = [], []
rng = __import__('random').Random(1)
per = (total_mib << 20) // nfiles
for i in range(nfiles):
    n = per + (rng.randrange(0, 4096) if nfiles > 1 else 0)
    p = os.path.join(tmp, 'f%04d' % i)
    with open(p, 'wb') as f:
        f.write(os.urandom(n))
    paths.append(p)
    sizes.append(n)
total = sum(sizes)
print(json.dumps({'progress': 'files written', 'bytes': total, 'files': nfiles}), flush=True)


def phases(prod):
    return {k: round(v, 4) for k, v in prod.profile.items() if k not in ('t0', 'timeline')}


def timeline_of(prod):
    """The last run's per-batch device phases (timeline=True producers), summarised."""
    tl = prod.profile.get('timeline')
    if not tl:
        return {}
    keys = ('upload_ms', 'chunk_ms', 'file_digest_ms', 'digest_ms', 'device_ms',
            'enqueue_to_done_ms')
    return {'timeline_median': {k: round(sorted(b[k] for b in tl)[len(tl) // 2], 3) for k in keys},
            'timeline': tl}


def timed(fn, reps=3):
    fn()  # warm (page cache, allocations)
    best = None
    for _ in range(reps):
        t = time.perf_counter()
        out = fn()
        dt = time.perf_counter() - t
        best = dt if best is None or dt < best else best
    return best, out


enc = ChunkEncryption(shared_key=os.urandom(32), shared_kdf_params=os.urandom(16))
variants = [('plain', {}), ('encrypted', {'encryption': enc})]
if 'parallel_reads' in DeviceSnapshotProducer.__init__.__code__.co_varnames:
    variants.insert(1, ('plain_reads_in_line', {'parallel_reads': False}))
HAS_RT = 'read_threads' in DeviceSnapshotProducer.__init__.__code__.co_varnames
if HAS_RT:  # one positional read per piece (the default reads each piece as 4 parallel parts)
    variants.insert(1, ('plain_1_reader', {'read_threads': 1}))
plain = None
if os.environ.get('PROBE_VARIANTS'):
    variants = [v for v in variants if v[0] in os.environ['PROBE_VARIANTS'].split(',')]
for name, kw in variants:
    prod = DeviceSnapshotProducer(min_length=MIN, max_length=MAX, **kw)
    dt, res = timed(lambda: prod.run(paths))
    print(json.dumps({'variant': name, 'bytes': total, 'files': nfiles, 'chunks': len(res.chunks),
                      's': round(dt, 4), 'gib_s': round(total / dt / GIB, 3),
                      'phases_s': phases(prod)}), flush=True)
    if name == 'plain':
        plain = res


# stream(): zero-copy records (views into the pinned batches), consumed as replicat's upload
# workers take _SnapshotChunks (repository.py:1355,1492,1507-1554): 'release' hands each record
# back at once (the producer's own rate); 'workers' puts them on a queue of concurrent * 10 = 50
# for 5 threads that touch every byte (a checksum pass standing in for the upload) and release
def consume(prod, workers):
    import queue
    import threading
    import zlib
    q = queue.Queue(maxsize=50)
    n = [0]

    def work():
        while (r := q.get()) is not None:
            zlib.adler32(r.contents)
            r.release()

    ts = [threading.Thread(target=work) for _ in range(workers)]
    for t in ts:
        t.start()
    with prod.stream(paths) as st:
        for r in st:
            n[0] += 1
            if workers:
                q.put(r)
            else:
                r.release()
            del r
        snap = st.snapshot()
    for _ in ts:
        q.put(None)
    for t in ts:
        t.join()
    return snap


if hasattr(DeviceSnapshotProducer, 'stream'):
    svars = [('stream_release', 0, {}), ('stream_5_workers', 5, {}),
             ('stream_release_encrypted', 0, {'encryption': enc})]
    if HAS_RT:
        svars.insert(1, ('stream_release_1_reader', 0, {'read_threads': 1}))
        svars.insert(2, ('stream_release_3_slots', 0, {'slots': 3}))
        svars.insert(3, ('stream_release_2gib_batches', 0, {'batch_bytes': 2 << 30}))
    if 'timeline' in DeviceSnapshotProducer.__init__.__code__.co_varnames:
        svars.insert(1, ('stream_release_timeline', 0, {'timeline': True}))
        svars.insert(2, ('stream_release_3_slots_timeline', 0, {'timeline': True, 'slots': 3}))
    if os.environ.get('PROBE_VARIANTS'):  # a comma list: only those stream() variants
        keep = os.environ['PROBE_VARIANTS'].split(',')
        svars = [v for v in svars if v[0] in keep]
    for name, workers, kw in svars:
        prod = DeviceSnapshotProducer(min_length=MIN, max_length=MAX, **kw)
        dt, snap = timed(lambda: consume(prod, workers))
        if plain is not None and (not kw or kw.get('read_threads') or kw.get('slots')
                                  or kw.get('batch_bytes') or kw.get('timeline')):
            assert [c.stream_end for c in snap.chunks] == [c.stream_end for c in plain.chunks]
            assert [c.digest for c in snap.chunks] == [c.digest for c in plain.chunks]
        print(json.dumps({'variant': name, 'bytes': total, 'files': nfiles,
                          'chunks': len(snap.chunks), 's': round(dt, 4),
                          'gib_s': round(total / dt / GIB, 3),
                          'phases_s': phases(prod), **timeline_of(prod)}),
              flush=True)

# CPU baseline: the oracle's chunker + hashlib over the same framed stream (one core)
def cpu_leg():
    pieces = list(snapshot.stream_pieces(snapshot.sort_files(paths)))
    stream = b''.join(pieces)
    P = len(stream) - len(pieces[-1]) if pieces else 0
    ends = o.chunk_stream(stream, MIN, MAX, None, P)
    prev, digs = 0, []
    for e in ends:
        digs.append(hashlib.blake2b(stream[prev:e]).digest())
        prev = e
    fd = [hashlib.blake2b(open(p, 'rb').read()).digest() for p in paths]
    return ends, digs, fd


dt, (ends, digs, fd) = timed(cpu_leg, reps=1)


# the bound of the producer on few large files: each file digest is one sequential BLAKE2b
# chain (repository.py:1437-1446), hashed here alone on one core from the page cache
def file_digests_alone():
    for p in paths:
        with open(p, 'rb') as f:
            h = hashlib.blake2b()
            while piece := f.read(16 << 20):
                h.update(piece)


fdt, _ = timed(file_digests_alone)
print(json.dumps({'variant': 'hashlib_file_digests_only', 'bytes': total, 's': round(fdt, 4),
                  'gib_s': round(total / fdt / GIB, 3),
                  'largest_file_s': round(fdt * max(sizes) / total, 4)}), flush=True)


# the same per-file BLAKE2b chains on the producer's host pool size (min(16, cpu_count) threads,
# one file per task, 16 MiB pieces): the host's ceiling for a producer whose large files'
# digests run on host threads (pipeline.py HOST_DIGEST_MIN)
def file_digests_pool():
    from concurrent.futures import ThreadPoolExecutor

    def one(p):
        with open(p, 'rb') as f:
            h = hashlib.blake2b()
            while piece := f.read(16 << 20):
                h.update(piece)
        return h.digest()
    with ThreadPoolExecutor(max_workers=max(1, min(16, os.cpu_count() or 1))) as ex:
        return list(ex.map(one, paths))


if nfiles > 1:
    pdt, _ = timed(file_digests_pool)
    print(json.dumps({'variant': 'hashlib_file_digests_pool', 'threads': max(1, min(16, os.cpu_count() or 1)),
                      'bytes': total, 's': round(pdt, 4), 'gib_s': round(total / pdt / GIB, 3)}),
          flush=True)
assert [c.stream_end for c in plain.chunks] == ends, 'cut mismatch'
assert [c.digest for c in plain.chunks] == digs, 'digest mismatch'
assert sorted(f.digest for f in plain.files) == sorted(fd), 'file digest mismatch'
print(json.dumps({'variant': 'cpu_oracle_1core', 'bytes': total, 's': round(dt, 4),
                  'gib_s': round(total / dt / GIB, 3), 'matches_gpu': True}), flush=True)
for p in paths:
    os.unlink(p)
os.rmdir(tmp)
