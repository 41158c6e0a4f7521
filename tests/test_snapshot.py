"""Snapshot framing (repository.py:1340-1452): one stream per snapshot, files sorted by
(size, path), 16 MiB pieces, zero padding to 4 bytes between files.  The chunk lengths come
from the reference adapter over the reference framing (tests/golden/snapshots.json)."""
import os
import random

import pytest

import golden_util as G
from replicat_amd import snapshot, synth

SNAPS = {s['name']: s for s in G.load('snapshots.json')}


def file_sets():
    rnd = random.Random(0)
    sizes = [('a', 4099), ('b', 32), ('c', 1023), ('d', 517), ('e', 2), ('f', 128), ('g', 64),
             ('h', 2048), ('i', 19), ('j', 8), ('k', 4), ('l', 256), ('m', 1), ('n', 0),
             ('o', 0), ('p', 19)]
    test_set = {name: (rnd.randbytes(n) if n else b'') for name, n in sizes}
    big = {}
    for i, n in enumerate([0, 3, (16 << 20) - 1, (16 << 20) + 5, 7_000_001, (33 << 20) + 2]):
        big['f%02d' % i] = synth.stream_bytes(n, synth.DEFAULT_SEED, 900 + i).tobytes() if n else b''
    return {'reference_test_set': test_set, 'reference_test_set_seeded': test_set,
            'big_files': big}


def write(tmp_path, files):
    paths = []
    for name, data in files.items():
        p = tmp_path / name
        p.write_bytes(data)
        paths.append(p)
    return paths


@pytest.mark.parametrize('name', sorted(SNAPS))
def test_framing_with_oracle(oracle, tmp_path, name):
    """CPU: the restated framing + the oracle's closed form give the reference's chunks."""
    s = SNAPS[name]
    paths = write(tmp_path, file_sets()[name])
    pieces = list(snapshot.stream_pieces(snapshot.sort_files(paths)))
    params = None if s['params'] is None else bytes.fromhex(s['params'])
    assert oracle.chunk_pieces(pieces, s['min'], s['max'], params) == s['lengths']


def test_sort_and_padding(tmp_path):
    paths = write(tmp_path, {'z': b'12345', 'y': b'', 'x': b'abcde', 'w': b'1'})
    order = [os.path.basename(p) for p in snapshot.sort_files(paths)]
    assert order == ['y', 'w', 'x', 'z']
    files = []
    pieces = list(snapshot.stream_pieces(snapshot.sort_files(paths), files))
    assert pieces == [b'1', bytes(3), b'abcde', bytes(3), b'12345']
    assert [(f.stream_start, f.stream_end) for f in files] == [(0, 0), (0, 1), (4, 9), (12, 17)]


@pytest.mark.gpu
@pytest.mark.parametrize('name', sorted(SNAPS))
def test_chunk_snapshot_on_device(tmp_path, name):
    torch = pytest.importorskip('torch')
    if not torch.cuda.is_available():
        pytest.skip('needs an MI355X')
    s = SNAPS[name]
    files_data = file_sets()[name]
    paths = write(tmp_path, files_data)
    params = None if s['params'] is None else bytes.fromhex(s['params'])
    files, chunks = snapshot.chunk_snapshot(paths, min_length=s['min'], max_length=s['max'],
                                            params=params)
    assert [c.stream_end - c.stream_start for c in chunks] == s['lengths']
    # every file is reassembled from its chunk ranges (repository.py:1374-1411)
    ranges = snapshot.file_ranges(files, chunks)
    for f in files:
        data = b''.join(chunks[ci].data[a:b] for ci, (a, b) in ranges[f.path])
        assert data == files_data[os.path.basename(f.path)]


def _pieces_restated(paths, read):
    """repository.py:1413-1447 as written there: read(PIECE) until EOF, a zero piece of
    (-len) % 4 bytes before every file but the first (after the previous one), with tags."""
    out, pos, prev, nfiles = [], 0, None, 0
    for path in paths:
        if prev is not None and -prev % 4:
            out.append((bytes(-prev % 4), nfiles, None))
            pos += -prev % 4
        nfiles += 1
        prev = 0
        with read(path) as src:
            while piece := src.read(snapshot.PIECE):
                out.append((piece, nfiles - 1, nfiles - 1))
                prev += len(piece)
    return out


class _NoReadinto:
    """A read hook's object with read() only (no readinto, no fileno)."""

    def __init__(self, data, step):
        self.data, self.pos, self.step = data, 0, step

    def read(self, n):  # short reads: at most `step` bytes per call
        piece = self.data[self.pos:self.pos + min(n, self.step)]
        self.pos += len(piece)
        return piece

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


@pytest.mark.parametrize('hook', ['file', 'bytesio', 'short_reads'])
def test_piece_reader_matches_reference_framing(tmp_path, hook):
    """snapshot.PieceReader (the framing of stream_pieces and the device producer) places the
    reference's pieces -- same bytes, boundaries, tags and file ranges -- whether the file
    object is read with readinto (buffered files, BytesIO) or read() (any other read hook)."""
    import io
    rnd = random.Random(11)
    files = {'f%02d' % i: rnd.randbytes(rnd.choice([0, 1, 2, 3, 5, 4096, rnd.randrange(0, 70_000)]))
             for i in range(40)}
    files['big'] = rnd.randbytes((16 << 20) + 7)
    paths = snapshot.sort_files(write(tmp_path, files))
    opener = {'file': lambda p: open(p, 'rb'),
              'bytesio': lambda p: io.BytesIO(files[os.path.basename(p)]),
              'short_reads': lambda p: _NoReadinto(files[os.path.basename(p)], 30_001)}[hook]
    expected = _pieces_restated(paths, opener)
    recs = []
    reader = snapshot.PieceReader(paths, recs, opener)
    buf = bytearray(snapshot.PIECE)
    got = []
    while (r := reader.read_into(buf)) is not None:
        got.append((bytes(buf[:r[0]]), r[1], r[2]))
    assert got == expected
    assert reader.pos == sum(len(p) for p, _, _ in expected)
    # file records: start / end of each file's bytes in the stream
    pos, ranges = 0, {}
    for p, tag, fi in expected:
        if fi is not None:
            ranges.setdefault(fi, [pos, pos])[1] = pos + len(p)
        pos += len(p)
    assert len(recs) == len(files)
    for fi, f in enumerate(recs):
        assert [f.stream_start, f.stream_end] == ranges.get(fi, [f.stream_start] * 2)
        assert f.path == str(paths[fi])


def test_file_parts_order():
    """file_parts: the chunk -> file pieces in _chunk_done's order (repository.py:1374-1411),
    the files a chunk touches from its last one backwards; file_ranges groups them per file."""
    F = snapshot.SnapshotFile
    files = [F('a', 0, 0), F('b', 0, 5), F('c', 8, 20), F('d', 20, 21)]
    chunks = [snapshot.SnapshotChunk(0, 12, b''), snapshot.SnapshotChunk(12, 21, b'')]
    parts = list(snapshot.file_parts(files, chunks))
    assert parts == [(0, 2, [8, 12]), (0, 1, [0, 5]), (0, 0, [0, 0]),
                     (1, 3, [8, 9]), (1, 2, [0, 8])]
    assert snapshot.file_ranges(files, chunks) == {
        'a': [(0, [0, 0])], 'b': [(0, [0, 5])], 'c': [(0, [8, 12]), (1, [0, 8])],
        'd': [(1, [8, 9])]}
