"""GPU parity of the device snapshot producer (replicat_amd/pipeline.py): replicat's
_stream_files + _chunk_producer + _chunk_done (repository.py:1374-1505) with chunks, chunk
digests and per-file digests computed on the device from one upload per batch.

Expected values: chunk lengths from the reference adapter over the reference framing
(tests/golden/snapshots.json), the oracle's closed form for other sets, and hashlib.blake2b
(replicat's hash_digest / incremental_hasher, adapters.py:106-114,224-228) for every digest.
Runs on an MI355X only (-m gpu)."""
import hashlib
import os
import random

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip('needs an MI355X', allow_module_level=True)

import golden_util as G  # noqa: E402
from test_snapshot import file_sets, write  # noqa: E402

from replicat_amd import snapshot, synth  # noqa: E402
from replicat_amd.pipeline import DeviceSnapshotProducer  # noqa: E402

SNAPS = {s['name']: s for s in G.load('snapshots.json')}


def check_stream(res, files_data, lengths=None):
    # chunks tile the stream; contents, digests, counters, dedup indices
    pos, table = 0, {}
    for k, c in enumerate(res.chunks):
        assert c.counter == k + 1 and c.stream_start == pos
        pos = c.stream_end
        assert c.digest == hashlib.blake2b(c.contents).digest()
        assert c.table_index == table.setdefault(c.digest, len(table))
    if lengths is not None:
        assert [c.stream_end - c.stream_start for c in res.chunks] == lengths
    # per-file digests and reassembly from the snapshot_files ranges (repository.py:1374-1411)
    sf = res.snapshot_files()
    for f in res.files:
        data = files_data[os.path.basename(f.path)]
        assert f.digest == hashlib.blake2b(data).digest(), f.path
        if data:
            parts = sf[f.path]['chunks']
            got = b''.join(res.chunks[p['counter'] - 1].contents[p['range'][0]:p['range'][1]]
                           for p in parts)
            assert got == data
            assert sf[f.path]['digest'] == f.digest


@pytest.mark.parametrize('name', sorted(SNAPS))
def test_reference_snapshots(tmp_path, name):
    s = SNAPS[name]
    files_data = file_sets()[name]
    paths = write(tmp_path, files_data)
    params = None if s['params'] is None else bytes.fromhex(s['params'])
    res = DeviceSnapshotProducer(min_length=s['min'], max_length=s['max'], params=params,
                                 batch_bytes=1 << 20).run(paths)
    check_stream(res, files_data, s['lengths'])
    assert len(res.files) == len(files_data)


@pytest.mark.parametrize('batch,engine', [(1, 'auto'), (3 << 20, 'auto'), (64 << 20, 'auto'),
                                          (3 << 20, 'device'), (1, 'host')])
def test_many_files_many_batches(oracle, tmp_path, batch, engine):
    """Small params and small batches: files straddle batches, the carried tail, empty files
    between batches; cuts against the oracle over the whole framed stream."""
    rnd = random.Random(batch)
    files_data = {}
    for i in range(120):
        n = rnd.choice([0, 1, 2, 3, 5, 127, 128, 129, rnd.randrange(0, 5000),
                        rnd.randrange(0, 300_000), rnd.randrange(0, 2_000_000)])
        files_data['f%03d' % i] = rnd.randbytes(n)
    paths = write(tmp_path, files_data)
    mn, mx = 2_000, 80_000
    key = synth.seeded_key(7)
    res = DeviceSnapshotProducer(min_length=mn, max_length=mx, params=key,
                                 batch_bytes=batch, file_digests=engine).run(paths)
    pieces = list(snapshot.stream_pieces(snapshot.sort_files(paths)))
    stream = b''.join(pieces)
    P = len(stream) - len(pieces[-1]) if pieces else 0
    ends = oracle.chunk_stream(stream, mn, mx, key, P)
    lengths = [b - a for a, b in zip([0] + ends[:-1], ends)]
    check_stream(res, files_data, lengths)


@pytest.mark.parametrize('engine', ['auto', 'device'])
def test_big_files_default_params(tmp_path, engine):
    """Files across the 16 MiB piece size with default params (reference fixture); file digests
    on host threads ('auto': these files are large) and all on the device."""
    files_data = file_sets()['big_files']
    paths = write(tmp_path, files_data)
    s = SNAPS['big_files']
    res = DeviceSnapshotProducer(min_length=s['min'], max_length=s['max'],
                                 batch_bytes=20 << 20, file_digests=engine).run(paths)
    check_stream(res, files_data, s['lengths'])


def test_empty_snapshot(tmp_path):
    paths = write(tmp_path, {'a': b'', 'b': b''})
    res = DeviceSnapshotProducer(min_length=256, max_length=512).run(paths)
    assert res.chunks == []
    assert [f.digest for f in res.files] == [hashlib.blake2b(b'').digest()] * 2


@pytest.mark.parametrize('key_bits,nonce_bits,batch', [(256, 96, 1 << 20), (128, 96, 3 << 20),
                                                       (256, 128, 64 << 20)])
def test_encrypted_snapshot(oracle, tmp_path, key_bits, nonce_bits, batch):
    """An encrypted repository's chunk loop (repository.py:1470-1473): every uploaded blob is
    nonce || AESGCM(derive_shared_subkey(digest)).encrypt(nonce, chunk) with the subkey
    blake2b(digest, key=shared_key, salt=shared_kdf_params, digest_size=key_bits // 8)
    (repository.py:132-137; adapters.py:205-213), checked by the oracle's GCM decrypt against the
    framed stream; nonces are fresh per chunk."""
    from replicat_amd.pipeline import ChunkEncryption
    rnd = random.Random(key_bits + nonce_bits + batch)
    files_data = {'f%02d' % i: rnd.randbytes(rnd.choice([0, 1, 7, 4096, rnd.randrange(0, 900_000)]))
                  for i in range(24)}
    paths = write(tmp_path, files_data)
    enc = ChunkEncryption(shared_key=rnd.randbytes(32), shared_kdf_params=rnd.randbytes(16),
                          key_bits=key_bits, nonce_bits=nonce_bits)
    mn, mx = 2_000, 80_000
    res = DeviceSnapshotProducer(min_length=mn, max_length=mx, params=synth.seeded_key(5),
                                 batch_bytes=batch, encryption=enc).run(paths)
    stream = b''.join(snapshot.stream_pieces(snapshot.sort_files(paths)))
    assert res.chunks and res.chunks[-1].stream_end == len(stream)
    nb, nonces = nonce_bits // 8, set()
    for c in res.chunks:
        plain = stream[c.stream_start:c.stream_end]
        assert c.digest == hashlib.blake2b(plain).digest()
        subkey = hashlib.blake2b(c.digest, salt=enc.shared_kdf_params, key=enc.shared_key,
                                 digest_size=key_bits // 8).digest()
        blob = c.contents
        assert len(blob) == nb + len(plain) + 16
        assert oracle.gcm_decrypt(subkey, blob[:nb], blob[nb:]) == plain
        nonces.add(blob[:nb])
    assert len(nonces) == len(res.chunks)
    for f in res.files:
        assert f.digest == hashlib.blake2b(files_data[os.path.basename(f.path)]).digest()


@pytest.mark.parametrize('encrypted', [False, True])
def test_deduplicated_references(oracle, tmp_path, encrypted):
    """replicat's own dedup cases (test_repository.py:691-736): min = max = 256 over one file
    of b'A' * 8192 gives 32 chunk references in the file's entry and ONE unique chunk, whose
    digest is hash_digest of the first chunk -- unencrypted, and encrypted with a random chunker
    key (a min = max chunker cuts every 256 bytes whatever the key)."""
    from replicat_amd.pipeline import ChunkEncryption
    contents = b'A' * 8_192
    paths = write(tmp_path, {'file': contents})
    rnd = random.Random(736)
    enc = ChunkEncryption(shared_key=rnd.randbytes(32), shared_kdf_params=rnd.randbytes(16)) \
        if encrypted else None
    params = rnd.randbytes(16) if encrypted else None  # key.params['chunker_params'] (:177)
    res = DeviceSnapshotProducer(min_length=256, max_length=256, params=params,
                                 encryption=enc).run(paths)
    sf = res.snapshot_files()
    assert len(sf) == 1
    refs = sf[str(paths[0])]['chunks']
    assert len(refs) == 32
    assert len(res.chunks_table) == 1
    digest = hashlib.blake2b(contents[:256]).digest()
    assert list(res.chunks_table) == [digest]
    assert all(c.digest == digest and c.table_index == 0 for c in res.chunks)
    assert [r['range'] for r in refs] == [[0, 256]] * 32
    assert res.files[0].digest == hashlib.blake2b(contents).digest()
    if encrypted:
        subkey = hashlib.blake2b(digest, salt=enc.shared_kdf_params, key=enc.shared_key,
                                 digest_size=32).digest()
        for c in res.chunks:
            assert oracle.gcm_decrypt(subkey, c.contents[:12], c.contents[12:]) == contents[:256]


def test_read_hook_without_fileno(tmp_path):
    """A read hook whose objects have no file descriptor: each file's digest engine is decided
    once, from the bytes read when the file is first seen, and every digest still equals
    hashlib's across batches (large files straddle them)."""
    import io
    rnd = random.Random(42)
    files_data = {'f%02d' % i: rnd.randbytes(n) for i, n in
                  enumerate([0, 100, 5000, (1 << 20) + 3, (3 << 20) + 1, 700_000])}
    paths = write(tmp_path, files_data)
    prod = DeviceSnapshotProducer(min_length=2_000, max_length=80_000, batch_bytes=1 << 20)
    res = prod.run(paths, read=lambda p: io.BytesIO(files_data[os.path.basename(str(p))]))
    check_stream(res, files_data)
    assert all(f.size is None for f in res.files)


def test_close_and_context_manager(tmp_path):
    """close() (or leaving a with block) releases the batches, device handles and threads; a
    closed producer refuses to run."""
    files_data = {'a': random.Random(3).randbytes(300_000)}
    paths = write(tmp_path, files_data)
    with DeviceSnapshotProducer(min_length=2_000, max_length=80_000, batch_bytes=1 << 20) as prod:
        check_stream(prod.run(paths), files_data)
    with pytest.raises(RuntimeError, match='closed'):
        prod.run(paths)


# ------------------------------------------------------------- stream(): zero-copy records

def _streamed(prod, paths, queue_size=0, workers=0):
    """Consume prod.stream(paths) the way replicat's snapshot loop does (repository.py:1355,
    1492, 1507-1554): workers=0 -- each record 'uploaded' (its contents checked against its
    digest) and released at once; otherwise the records go through a bounded queue of
    queue_size to `workers` upload threads that release them after their upload, out of order
    and later than the producer moves on."""
    import queue as Q
    import threading
    out, bad, lock = {}, [], threading.Lock()
    plain = prod.encryption is None  # encrypted contents are nonce || C || T

    def upload(rec):
        data = bytes(rec.contents)
        if plain and hashlib.blake2b(data).digest() != rec.digest:
            bad.append(rec.counter)
        rec.release()
        with lock:
            out[rec.counter] = data

    q = Q.Queue(maxsize=queue_size) if workers else None

    def worker():
        while True:
            rec = q.get()
            if rec is None:
                return
            upload(rec)

    threads = [threading.Thread(target=worker) for _ in range(workers)]
    for t in threads:
        t.start()
    try:
        with prod.stream(paths, stall_timeout=60) as st:
            for rec in st:
                assert isinstance(rec.contents, memoryview) and rec.contents.readonly
                if q is None:
                    upload(rec)
                else:
                    q.put(rec)
                del rec
            res = st.snapshot()
    finally:
        for _ in threads:
            q.put(None)
        for t in threads:
            t.join()
    assert not bad, bad[:5]
    for c in res.chunks:  # the run's records carry no contents: give them the uploaded bytes
        assert c.contents is None
        c.contents = out[c.counter]
    return res


@pytest.mark.parametrize('name', sorted(SNAPS))
@pytest.mark.parametrize('queue_size,workers', [(0, 0), (50, 5), (3, 2)])
def test_stream_reference_snapshots(tmp_path, name, queue_size, workers):
    """stream() gives the reference's chunks, digests and file ranges with views into the
    pinned batches; records released late and out of order by upload workers (replicat's
    queue of concurrent * 10 and 5 workers) never see a refilled buffer."""
    s = SNAPS[name]
    files_data = file_sets()[name]
    paths = write(tmp_path, files_data)
    params = None if s['params'] is None else bytes.fromhex(s['params'])
    prod = DeviceSnapshotProducer(min_length=s['min'], max_length=s['max'], params=params,
                                  batch_bytes=1 << 20)
    res = _streamed(prod, paths, queue_size, workers)
    check_stream(res, files_data, s['lengths'])
    # the same producer again, now through run(): the same stream
    again = prod.run(paths)
    assert [(c.stream_end, c.digest) for c in again.chunks] == \
        [(c.stream_end, c.digest) for c in res.chunks]


def test_stream_encrypted_and_abandoned(oracle, tmp_path):
    """Encrypted records view the pinned ciphertexts (nonce || C || T, decrypted by the oracle
    under the chunk's subkey); a consumer that stops early (close()) leaves the producer
    usable for the next stream."""
    from replicat_amd.pipeline import ChunkEncryption
    rnd = random.Random(1470)
    files_data = {'f%02d' % i: rnd.randbytes(rnd.choice([7, 4096, rnd.randrange(0, 3_000_000)]))
                  for i in range(16)}
    paths = write(tmp_path, files_data)
    enc = ChunkEncryption(shared_key=rnd.randbytes(32), shared_kdf_params=rnd.randbytes(16))
    mn, mx = 2_000, 80_000
    prod = DeviceSnapshotProducer(min_length=mn, max_length=mx, batch_bytes=1 << 20,
                                  encryption=enc)
    stream = b''.join(snapshot.stream_pieces(snapshot.sort_files(paths)))
    n = 0
    with prod.stream(paths) as st:
        for rec in st:
            plain = stream[rec.stream_start:rec.stream_end]
            subkey = hashlib.blake2b(rec.digest, salt=enc.shared_kdf_params, key=enc.shared_key,
                                     digest_size=32).digest()
            blob = bytes(rec.contents)
            assert oracle.gcm_decrypt(subkey, blob[:12], blob[12:]) == plain
            rec.release()
            n += 1
            if n == 40:
                break  # abandoned: the producer thread stops at its next batch
    assert n == 40
    res = _streamed(prod, paths, queue_size=10, workers=3)
    assert res.chunks[-1].stream_end == len(stream)
    for c in res.chunks:
        blob = c.contents
        subkey = hashlib.blake2b(c.digest, salt=enc.shared_kdf_params, key=enc.shared_key,
                                 digest_size=32).digest()
        assert oracle.gcm_decrypt(subkey, blob[:12], blob[12:]) == \
            stream[c.stream_start:c.stream_end]


def test_stream_abandoned_by_a_bare_loop(tmp_path):
    """a plain ``for rec in prod.stream(p): ... break`` with no close() must
    stop the producer thread (the iterator's finally), so that the next run() on the same
    producer neither hangs on the old run's slots nor runs beside it; and a second run while a
    stream is still producing fails fast instead of sharing the slots."""
    import gc
    import threading
    rnd = random.Random(1505)
    files_data = {'f%02d' % i: rnd.randbytes(rnd.randrange(200_000, 900_000)) for i in range(24)}
    paths = write(tmp_path, files_data)
    prod = DeviceSnapshotProducer(min_length=2_000, max_length=80_000, batch_bytes=1 << 20)
    n = 0
    for rec in prod.stream(paths):
        rec.release()
        n += 1
        if n == 5:
            break
    del rec
    gc.collect()
    deadline = 50
    while any(t.name == 'rc-chunk-producer' for t in threading.enumerate()) and deadline:
        threading.Event().wait(0.1)
        deadline -= 1
    assert not any(t.name == 'rc-chunk-producer' for t in threading.enumerate())
    res = prod.run(paths)
    stream = b''.join(snapshot.stream_pieces(snapshot.sort_files(paths)))
    assert res.chunks[-1].stream_end == len(stream)
    assert b''.join(c.contents for c in res.chunks) == stream
    # a stream still producing: a concurrent run() fails fast
    st = prod.stream(paths)
    it = iter(st)
    first = next(it)
    with pytest.raises(RuntimeError, match='still producing'):
        prod.run(paths)
    first.release()
    st.close()
    prod.close()
