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
