"""CPU tests of the device producer's host side (replicat_amd/pipeline.py): the batches
fill_batch places from the files (through snapshot.PieceReader) hold exactly the reference's
stream (repository.py:1413-1447), whole pieces per batch, with the closed-file counts and file
ranges the producer's digests rely on.  No GPU: fill_batch runs on a numpy buffer."""
import os
import random

import numpy as np
import pytest

from replicat_amd import pipeline, snapshot


def _fill_all(paths, batch, threads=1):
    files = []
    reader = snapshot.PieceReader(paths, files, None, record=pipeline.FileRecord,
                                  on_open=pipeline._fstat_size, threads=threads)
    head = 64
    buf = np.zeros(head + batch + snapshot.PIECE + 64, dtype=np.uint8)
    look_buf = bytearray(snapshot.PIECE)
    look = reader.read_into(look_buf)
    batches, pieces = [], []
    try:
        while True:
            look, n, last = pipeline.fill_batch(
                reader, look_buf, look, buf, head, batch,
                lambda fi, at, ln: pieces.append((fi, at - head, ln)))
            batches.append((buf[head:head + n].tobytes(), last,
                            len(files) if look is None else look[1]))
            if look is None:
                break
    finally:
        reader.close()
    return batches, pieces, [(f.path, f.stream_start, f.stream_end, f.size) for f in files]


def _files(tmp_path, seed, n=24):
    rnd = random.Random(seed)
    paths = []
    for i in range(n):
        size = rnd.choice([0, 1, 3, 4099, rnd.randrange(0, 3 << 20), rnd.randrange(0, 20 << 20)])
        p = tmp_path / ('f%02d' % i)
        p.write_bytes(os.urandom(size))
        paths.append(p)
    return snapshot.sort_files(paths)


@pytest.mark.parametrize('threads', [1, 4])
@pytest.mark.parametrize('batch', [1 << 20, 5 << 20, 64 << 20])
def test_fill_batch_is_the_reference_stream(tmp_path, batch, threads):
    """Batches of whole pieces: concatenated, the reference's stream; every batch but the last
    holds at least `batch` bytes and ends at a piece boundary; the closed-file count of a batch
    is the number of files whose bytes all lie in it or before; the last piece's offset is where
    the stream's final piece starts (P of the final batch).  threads=4: pieces of regular files
    read as parallel positional parts (the producer's default)."""
    paths = _files(tmp_path, batch)
    batches, pieces, files = _fill_all(paths, batch, threads)
    pieces_ref = list(snapshot.stream_pieces(paths))
    assert b''.join(b for b, _, _ in batches) == b''.join(pieces_ref)
    assert [ln for _, _, ln in pieces] == [len(p) for p in pieces_ref]
    pos = 0
    for k, (data, last, closed) in enumerate(batches):
        end = pos + len(data)
        if k + 1 < len(batches):
            assert len(data) >= batch
        for fi, (_, a, b, _) in enumerate(files):
            if fi < closed:  # complete: every byte in this batch or before
                assert b <= end
            else:  # still open: starts after this batch or runs past it
                assert a >= end or b > end
        pos = end
    data, last, _ = batches[-1]
    assert len(data) - last == len(pieces_ref[-1])


def test_host_file_digests_in_order_across_threads():
    """_HostHash: pieces of many files pushed from one thread are hashed by a pool with one
    drain job per file at a time -- each file's pieces in order, files in parallel -- and a
    slot's _Pending waits for exactly its pieces (repository.py:1437-1446's per-file digests)."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    rnd = random.Random(9)
    datas = [rnd.randbytes(rnd.randrange(0, 3 << 20)) for _ in range(12)]
    hs = [pipeline._HostHash(hashlib.blake2b()) for _ in datas]
    slots = [pipeline._Pending() for _ in range(3)]
    with ThreadPoolExecutor(4) as pool:
        offs = [0] * len(datas)
        k = 0
        while any(o < len(d) for o, d in zip(offs, datas)):
            for i, d in enumerate(datas):
                if offs[i] < len(d):
                    n = rnd.randrange(1, 200_000)
                    hs[i].push(memoryview(d)[offs[i]:offs[i] + n], slots[k % 3], pool)
                    offs[i] += n
                    k += 1
        for sl in slots:
            sl.wait()
            assert sl.n == 0
    assert [h.h.digest() for h in hs] == [hashlib.blake2b(d).digest() for d in datas]


def test_pending_reports_a_failed_piece():
    from concurrent.futures import ThreadPoolExecutor

    class Bad:
        def update(self, view):
            raise ValueError('boom')

    sl = pipeline._Pending()
    with ThreadPoolExecutor(2) as pool:
        pipeline._HostHash(Bad()).push(memoryview(b'x'), sl, pool)
        with pytest.raises(ValueError, match='boom'):
            sl.wait()


@pytest.mark.parametrize('slots', [0, 1])
def test_producer_needs_two_slots(slots):
    """One batch is filled while another is on the device: fewer than two slots is refused
    before anything touches a device."""
    with pytest.raises(ValueError, match='slots'):
        pipeline.DeviceSnapshotProducer(slots=slots, device=0)


def test_producer_queue_modes():
    """queues='own' (the default: batch streams with hardware queues of their own) or 'shared'
    (torch streams); anything else is refused before any device work."""
    import inspect
    sig = inspect.signature(pipeline.DeviceSnapshotProducer.__init__)
    assert sig.parameters['queues'].default == 'own'
    assert sig.parameters['slots'].default == 3  # round 5: host-bound, 3 reach 90 % of it
    with pytest.raises(ValueError, match='queues'):
        pipeline.DeviceSnapshotProducer(queues='many', device=0)


def test_record_release_is_idempotent():
    """stream() records hold a lease on their batch until release() (or garbage collection)."""
    lease = pipeline._Lease()
    recs = [pipeline.ChunkRecord(k + 1, k, k + 1, b'd', 0, memoryview(b'x'), lease)
            for k in range(3)]
    lease.take(3)
    recs[0].release()
    recs[0].release()
    assert lease.n == 2 and recs[0].contents is None
    del recs[1]
    assert lease.n == 1
    import threading
    recs[-1].release()
    assert lease.wait(threading.Event()) is True


@pytest.mark.parametrize('threads', [2, 3, 4, 8])
def test_parallel_piece_reads_are_read_piece(tmp_path, threads):
    """PieceReader(threads > 1) against one read(PIECE) per piece (stream_pieces, threads=1) at
    the sizes where parts meet pieces: a piece of exactly PIECE, one byte either side, a part
    boundary (READ_SPLIT multiples), empty and tiny files, files opened by a `read` hook that
    are not regular buffered files (BytesIO: read as before)."""
    import io
    P, S = snapshot.PIECE, snapshot.READ_SPLIT
    sizes = [0, 1, S - 1, S, S + 1, 3 * S + 5, P - 1, P, P + 1, 2 * P + S - 3]
    paths = []
    for i, n in enumerate(sizes):
        p = tmp_path / ('g%02d' % i)
        p.write_bytes(os.urandom(n))
        paths.append(p)
    paths = snapshot.sort_files(paths)
    ref_files, got_files = [], []
    ref = list(snapshot.stream_pieces(paths, ref_files))
    got = list(snapshot.stream_pieces(paths, got_files, threads=threads))
    assert [len(x) for x in got] == [len(x) for x in ref]
    assert got == ref
    assert got_files == ref_files
    hooked = list(snapshot.stream_pieces(
        paths, read=lambda p: io.BytesIO(open(p, 'rb').read()), threads=threads))
    assert hooked == ref


def test_close_releases_records_still_queued():
    """A consumer that stops early: the records the producer thread had already queued (a whole
    batch or more, with 3 slots) are released by close() -- not when the stream object is
    garbage-collected -- so the next run on the producer finds its slots free (round 5: the GPU
    test of an abandoned encrypted stream waited 60 s for such a batch's lease)."""
    leases = [pipeline._Lease() for _ in range(3)]

    def batch(lease):
        recs = [pipeline.ChunkRecord(i + 1, i, i + 1, b'd', 0, memoryview(b'x'), lease)
                for i in range(5)]
        lease.take(len(recs))
        return recs

    class FakeProd:
        def _produce(self, paths, read, files, zero_copy, sink, abort, stall_timeout=None):
            sink(batch(leases[0]))
            abort.wait(10)
            # batches a collector thread hands over while the producer is already stopping: the
            # thread is gone by the time the consumer's drain loop looks again
            sink(batch(leases[1]))
            sink(batch(leases[2]))
            raise pipeline._Aborted()

    with pipeline.ChunkStream(FakeProd(), []) as st:
        for rec in st:
            rec.release()
            break
        kept = st  # the stream object stays referenced, as in a `with` block
    assert [lease.n for lease in leases] == [0, 0, 0]
    assert kept._done
