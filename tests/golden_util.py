"""Helpers that rebuild golden-fixture inputs from their JSON descriptions (no reference needed)."""
import hashlib
import json
import os
import random
import struct

import numpy as np

from replicat_amd import synth

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    with open(os.path.join(GOLDEN_DIR, name)) as f:
        return json.load(f)


def small_data(spec, n):
    kind = spec[0]
    if kind == 'mt':
        return random.Random(spec[1]).randbytes(n)
    if kind == 'zero':
        return bytes(n)
    if kind == 'const':
        return bytes([spec[1]]) * n
    if kind == 'repeat':
        unit = random.Random(spec[1]).randbytes(spec[2])
        return (unit * (n // len(unit) + 1))[:n]
    raise ValueError(spec)


def case_pieces(case):
    data = small_data(case['data'], case['size'])
    out, pos = [], 0
    for n in case['pieces']:
        out.append(data[pos:pos + n])
        pos += n
    assert pos == len(data)
    return out


def params_of(case):
    return None if case['params'] is None else bytes.fromhex(case['params'])


def stream_of(entry):
    kind = entry['data'][0]
    if kind == 'splitmix':
        return synth.stream_bytes(entry['size'], entry['data'][1], entry['data'][2])
    if kind == 'fill':
        return np.full(entry['size'], entry['data'][1], dtype=np.uint8)
    raise ValueError(kind)


def last_piece_start(size, piece):
    """P for a stream read in `piece`-byte pieces (0 for a single piece)."""
    if not piece or size <= piece:
        return 0
    return ((size - 1) // piece) * piece


def seeded_inputs(entry):
    rnd = random.Random(entry['seed'])
    if entry['name'].startswith('personalization'):
        return [rnd.randbytes(entry['size'])]
    if entry['name'] == 'stabilizes':
        return [rnd.randbytes(entry['size'])]
    if entry['name'] == 'repetition':
        return [rnd.randbytes(entry['size'])] * entry['repeat']
    raise ValueError(entry['name'])


def cutlist_digest(all_ends):
    h = hashlib.sha256()
    for ends in all_ends:
        ends = [int(x) for x in ends]
        h.update(struct.pack('<Q', len(ends)))
        h.update(struct.pack('<%dQ' % len(ends), *ends))
    return h.hexdigest()
