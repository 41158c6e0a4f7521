"""Pin the CPU restatement (oracle/) against the reference's outputs (tests/golden/).

The fixtures were produced by replicat's own adapter over its own extension
(tests/golden/make_golden.py); these tests make the oracle a trustworthy checker for the
GPU parity tests.  CPU only.
"""
import random

import numpy as np
import pytest

import golden_util as G
from replicat_amd import synth

SMALL = G.load('small_cases.json')
KNOWN = G.load('known_answers.json')
STREAMS = G.load('streams.json')
DIGESTS = G.load('digests.json')


@pytest.mark.parametrize('idx', range(len(SMALL)))
def test_small_cases(oracle, idx):
    case = SMALL[idx]
    got = oracle.chunk_pieces(G.case_pieces(case), case['min'], case['max'], G.params_of(case))
    assert got == case['expected']


@pytest.mark.parametrize('idx', range(len(KNOWN['alignment'])))
def test_known_alignment(oracle, idx):
    c = KNOWN['alignment'][idx]
    pieces = [bytes([c['byte']]) * n for n in c['pieces']]
    assert oracle.chunk_pieces(pieces, c['min'], c['max']) == c['expected']


@pytest.mark.parametrize('idx', range(len(KNOWN['seeded'])))
def test_known_seeded(oracle, idx):
    c = KNOWN['seeded'][idx]
    pieces = G.seeded_inputs(c)
    params = bytes.fromhex(c['params'])
    assert oracle.chunk_pieces(pieces, 500, 10_000, params) == c['expected']
    if 'expected_after_flip0' in c:
        data = bytearray(pieces[0])
        data[0] = (data[0] - 1) % 255
        assert oracle.chunk_pieces([bytes(data)], 500, 10_000, params) == c['expected_after_flip0']


@pytest.mark.parametrize('idx', range(len(STREAMS)))
def test_streams(oracle, idx):
    e = STREAMS[idx]
    data = G.stream_of(e)
    P = G.last_piece_start(e['size'], e['piece'])
    params = None if e['params'] is None else bytes.fromhex(e['params'])
    assert oracle.chunk_stream(data, e['min'], e['max'], params, P) == e['ends']


def test_key_soft_matches_pclmul(oracle):
    rnd = random.Random(5)
    for _ in range(2000):
        k0, k1, d = (rnd.getrandbits(64) for _ in range(3))
        assert oracle.key(k0, k1, d) == oracle.key_soft(k0, k1, d)


def test_splitmix_c_matches_numpy(oracle):
    for n, s in [(0, 0), (5, 1), (64, 2), (4099, 1023)]:
        assert np.array_equal(oracle.fill_splitmix(n, synth.DEFAULT_SEED, s),
                              synth.stream_bytes(n, synth.DEFAULT_SEED, s))


def test_param_errors(oracle):
    with pytest.raises(ValueError, match='exactly 16'):
        oracle.parse_key(1, 2, b'x' * 15)
    with pytest.raises(ValueError, match='greater than the maximum'):
        oracle.parse_key(3, 2, b'\xff' * 16)
    with pytest.raises(ValueError, match='Bad key'):
        oracle.parse_key(1, 2, bytes(8) + b'\xff' * 8)


def _digest_set(oracle, d, limit=None):
    n = d['streams'] if limit is None else min(limit, d['streams'])
    params = None if d['params'] is None else bytes.fromhex(d['params'])
    ends = []
    for i in range(0, n, 16):
        bufs = [np.concatenate([synth.stream_bytes(d['size'], d['seed'], s),
                                np.zeros(16, np.uint8)]) for s in range(i, min(n, i + 16))]
        ends += oracle.chunk_streams_mt(bufs, [d['size']] * len(bufs), [0] * len(bufs),
                                        d['min'], d['max'], params, threads=8)
    return ends


@pytest.mark.slow
@pytest.mark.parametrize('name', [d['name'] for d in DIGESTS])
def test_digest_sets(oracle, name):
    d = next(x for x in DIGESTS if x['name'] == name)
    ends = _digest_set(oracle, d)
    assert sum(map(len, ends)) == d['chunks']
    assert G.cutlist_digest(ends) == d['sha256']
