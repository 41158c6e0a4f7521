"""Generate tests/golden/*.json from the REFERENCE chunker (build container only).

Runs replicat's own adapter (``replicat.utils.adapters.gclmulchunker``, imported from
/root/reference) over its own ``_replicat_adapters`` extension, compiled from
/root/reference/src/adapters.cpp by ``make -C oracle ref`` into oracle/_ref/.  Neither travels
to the GPU box: only the JSON this script writes does.

    make -C oracle ref
    PYTHONPATH=oracle/_ref:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/make_golden.py

Inputs are reproducible without the reference: CPython ``random.Random(seed).randbytes`` for
small cases (what the reference's own tests use, replicat/utils/compat.py:5-12) and the
splitmix64 counter streams of ``replicat_amd.synth`` for large ones.
"""
import hashlib
import json
import multiprocessing as mp
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

def _load_reference_extension():
    """Bind `_replicat_adapters` to the reference's own extension (oracle/_ref) before replicat
    imports it: the repository root also holds a module of that name (the drop-in), which
    must never stand in for the reference here."""
    import glob
    import importlib.machinery
    import importlib.util
    so = glob.glob(os.path.join(os.path.dirname(os.path.dirname(HERE)), 'oracle', '_ref',
                                '_replicat_adapters*.so'))
    if not so:
        raise SystemExit('build the reference extension first: make -C oracle ref')
    loader = importlib.machinery.ExtensionFileLoader('_replicat_adapters', so[0])
    spec = importlib.util.spec_from_loader('_replicat_adapters', loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules['_replicat_adapters'] = mod
    return mod


REF_EXT = _load_reference_extension()
from replicat.utils import adapters  # noqa: E402  (reference)
assert adapters._replicat_adapters is REF_EXT, 'reference adapter must use the reference extension'

from replicat_amd import synth  # noqa: E402

MIN_DEF, MAX_DEF = 128_000, 5_120_000


def ref_lengths(min_length, max_length, pieces, params):
    chunker = adapters.gclmulchunker(min_length=min_length, max_length=max_length)
    return [len(c) for c in chunker(pieces, params=params)]


# ---------------------------------------------------------------- small cases


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


def split_pieces(data, cuts):
    out, prev = [], 0
    for c in cuts + [len(data)]:
        out.append(data[prev:c])
        prev = c
    return out


def make_small_cases(count=320, seed=20261015):
    rnd = random.Random(seed)
    cases = []
    for n in range(count):
        aligned = n % 4 != 3  # 3 in 4 cases inside the multi-piece parity domain
        max_length = rnd.choice([4, 8, 12, 64, 100, 256, 1000, 4096, 10_000, 20_000])
        if aligned:
            max_length = max(4, max_length - max_length % 4)
        else:
            max_length += rnd.randrange(1, 4)
        min_length = rnd.randrange(1, max_length + 1)
        if rnd.random() < 0.15:
            min_length = max_length
        total = rnd.choice([0, 1, 3, 7, max_length - 1, max_length, 2 * max_length - 1,
                            2 * max_length, rnd.randrange(0, 64 * max_length + 1)])
        total = max(0, min(total, 200_000))
        dkind = rnd.random()
        if dkind < 0.75:
            spec = ['mt', rnd.randrange(1 << 30)]
        elif dkind < 0.83:
            spec = ['zero']
        elif dkind < 0.90:
            spec = ['const', rnd.randrange(256)]
        else:
            spec = ['repeat', rnd.randrange(1 << 30), rnd.randrange(1, 5000)]
        data = small_data(spec, total)
        if aligned and total and rnd.random() < 0.6:
            k = rnd.randrange(1, 12)
            cuts = sorted(rnd.randrange(0, total + 1) for _ in range(k))
        elif aligned and 0 < total <= 64 and rnd.random() < 0.5:
            cuts = list(range(1, total))  # one byte per piece (cf. test_adapters.py:287-289)
        else:
            cuts = []
        pieces = split_pieces(data, cuts)
        pk = rnd.random()
        if pk < 0.3:
            params = None
        elif pk < 0.85:
            params = rnd.randbytes(16)
            if params[:8] == bytes(8):
                params = b'\x01' + params[1:]
        else:
            params = rnd.randbytes(rnd.randrange(1, 16))
            if params[0] == 0:
                params = b'\x02' + params[1:]
        cases.append({
            'min': min_length, 'max': max_length, 'data': spec, 'size': total,
            'pieces': [len(p) for p in pieces],
            'params': None if params is None else params.hex(),
            'expected': ref_lengths(min_length, max_length, pieces, params),
        })
    return cases


def make_known_answers():
    """The reference's own test inputs (replicat/tests/test_adapters.py:273-364), as data."""
    out = {'alignment': [], 'seeded': []}
    for (mn, mx, piece, npieces, total) in [
        (5, 10, 0, 0, 0), (5, 10, 5, 1, 5), (5, 10, 6, 1, 6), (5, 10, 10, 1, 10),
        (5, 10, 11, 1, 11), (5, 10, 12, 1, 12), (5, 10, 13, 1, 13), (5, 10, 14, 1, 14),
        (5, 10, 15, 1, 15), (5, 10, 16, 1, 16), (5, 10, 17, 1, 17), (5, 10, 18, 1, 18),
        (5, 10, 19, 1, 19), (4, 4, 1, 20, 20), (4, 4, 20, 1, 20), (10, 12, 1, 11, 11),
    ]:
        pieces = [b'\xaa' * piece] * npieces
        out['alignment'].append({'min': mn, 'max': mx, 'byte': 0xAA, 'pieces': [piece] * npieces,
                                 'expected': ref_lengths(mn, mx, pieces, None)})
    # personalization (:301-313), sequence_stabilizes (:315-336), repetition (:338-364)
    rnd = random.Random(0)
    data = rnd.randbytes(1_000_000)
    person = bytearray(rnd.randbytes(16))
    out['seeded'].append({'name': 'personalization', 'seed': 0, 'size': 1_000_000, 'repeat': 1,
                          'params': bytes(person).hex(),
                          'expected': ref_lengths(500, 10_000, [data], bytes(person))})
    person[0] = (person[0] - 1) % 255
    out['seeded'].append({'name': 'personalization_flipped', 'seed': 0, 'size': 1_000_000,
                          'repeat': 1, 'params': bytes(person).hex(),
                          'expected': ref_lengths(500, 10_000, [data], bytes(person))})
    for seed in (507, 11219, 25750, 31286):
        rnd = random.Random(seed)
        data = bytearray(rnd.randbytes(1_000_000))
        person = rnd.randbytes(16)
        before = ref_lengths(500, 10_000, [bytes(data)], person)
        data[0] = (data[0] - 1) % 255
        after = ref_lengths(500, 10_000, [bytes(data)], person)
        out['seeded'].append({'name': 'stabilizes', 'seed': seed, 'size': 1_000_000,
                              'repeat': 1, 'params': person.hex(), 'expected': before,
                              'expected_after_flip0': after})
    for seed, size in [(0, 1_001), (1, 2_000), (2, 497), (2, 4_023), (3, 5_001)]:
        rnd = random.Random(seed)
        unit = rnd.randbytes(size)
        person = rnd.randbytes(16)
        for reps in (50, 100):
            out['seeded'].append({'name': 'repetition', 'seed': seed, 'size': size,
                                  'repeat': reps, 'params': person.hex(),
                                  'expected': ref_lengths(500, 10_000, [unit] * reps, person)})
    return out


# ------------------------------------------------------------- large streams


def _stream_job(job):
    kind, args = job
    if kind == 'splitmix':
        seed, idx, nbytes, piece, mn, mx, key = args
        data = synth.stream_bytes(nbytes, seed, idx).tobytes()
    elif kind == 'fill':
        value, nbytes, piece, mn, mx, key = args
        data = bytes([value]) * nbytes
    else:
        raise ValueError(kind)
    if piece:
        pieces = [data[i:i + piece] for i in range(0, len(data), piece)]
    else:
        pieces = [data]
    lens = ref_lengths(mn, mx, pieces, None if key is None else bytes.fromhex(key))
    ends, acc = [], 0
    for x in lens:
        acc += x
        ends.append(acc)
    return ends


def cutlist_digest(all_ends):
    h = hashlib.sha256()
    for ends in all_ends:
        h.update(struct.pack('<Q', len(ends)))
        h.update(struct.pack('<%dQ' % len(ends), *ends))
    return h.hexdigest()


def make_streams(pool):
    seeded = synth.seeded_key(1).hex()
    specs = []
    for key in (None, seeded):
        for i in range(4):
            specs.append(('splitmix', (synth.DEFAULT_SEED, i, 64 << 20, 0, MIN_DEF, MAX_DEF, key)))
    specs.append(('splitmix', (synth.DEFAULT_SEED, 7, 256 << 20, 16 << 20, MIN_DEF, MAX_DEF, None)))
    specs.append(('splitmix', (synth.DEFAULT_SEED, 8, (48 << 20) + 12345, 0, MIN_DEF, MAX_DEF, seeded)))
    specs.append(('fill', (0, 16 << 20, 0, MIN_DEF, MAX_DEF, None)))
    specs.append(('fill', (0xAA, 16 << 20, 0, MIN_DEF, MAX_DEF, seeded)))
    for i in range(4):
        specs.append(('splitmix', (synth.DEFAULT_SEED, i, 1 << 20, 0, MIN_DEF, MAX_DEF, None)))
        specs.append(('splitmix', (synth.DEFAULT_SEED, i, 1 << 20, 0, 2_000, 80_000, None)))
    results = pool.map(_stream_job, specs)
    out = []
    for (kind, args), ends in zip(specs, results):
        if kind == 'splitmix':
            seed, idx, nbytes, piece, mn, mx, key = args
            d = {'data': ['splitmix', seed, idx], 'size': nbytes}
        else:
            value, nbytes, piece, mn, mx, key = args
            d = {'data': ['fill', value], 'size': nbytes}
        d.update({'piece': piece, 'min': mn, 'max': mx, 'params': key, 'ends': ends})
        out.append(d)
    return out


def make_digests(pool, quick=False):
    seeded = synth.seeded_key(1).hex()
    sets = [
        # config 2: 1024 x 64 MiB, default params, unencrypted key (0xff * 16)
        ('config2_ff', 1024, 64 << 20, MIN_DEF, MAX_DEF, None),
        # config 2 subset with a generic key
        ('config2_seeded_first128', 128, 64 << 20, MIN_DEF, MAX_DEF, seeded),
        # config 3 (iii): non-default params on 1 MiB streams (first 4096 of 65536)
        ('config3iii_first4096', 4096, 1 << 20, 2_000, 80_000, None),
    ]
    out = []
    for name, n, size, mn, mx, key in sets:
        if quick:
            n = min(n, 16)
        jobs = [('splitmix', (synth.DEFAULT_SEED, i, size, 0, mn, mx, key)) for i in range(n)]
        ends = pool.map(_stream_job, jobs, chunksize=4)
        out.append({'name': name, 'streams': n, 'size': size, 'seed': synth.DEFAULT_SEED,
                    'min': mn, 'max': mx, 'params': key, 'chunks': sum(map(len, ends)),
                    'sha256': cutlist_digest(ends)})
        print(name, out[-1]['chunks'], out[-1]['sha256'], flush=True)
    return out


# ------------------------------------------------- large configs (3 ii, 5): large.json

def _ref_ends(mn, mx, pieces, params=None):
    ends, acc = [], 0
    for n in ref_lengths(mn, mx, pieces, params):
        acc += n
        ends.append(acc)
    return ends


def make_config3ii(stream_id=0, size=64 << 30, tail=1 << 20, piece=16 << 20):
    """Config 3 (ii): ONE 64 GiB stream under the reference's snapshot framing -- 16 MiB pieces
    (repository.py:1413-1452) whose last piece is the final 1 MiB (P = L - 1 MiB).  The bytes
    are generated piece by piece, so the reference adapter never needs the whole stream."""
    base = synth.stream_base(synth.DEFAULT_SEED, stream_id)

    def piece_bytes(off, n):
        w0, w1 = off // 8, (off + n + 7) // 8
        words = synth.splitmix_words(base, w0, w1 - w0)
        return words.view('<u1')[off - 8 * w0:off - 8 * w0 + n].tobytes()

    def pieces():
        P = size - tail
        off = 0
        while off < P:
            n = min(piece, P - off)
            yield piece_bytes(off, n)
            off += n
        yield piece_bytes(P, tail)

    ends = _ref_ends(MIN_DEF, MAX_DEF, pieces())
    return {'name': 'config3ii', 'stream': stream_id, 'seed': synth.DEFAULT_SEED, 'size': size,
            'last_piece': size - tail, 'min': MIN_DEF, 'max': MAX_DEF, 'params': None,
            'chunks': len(ends), 'sha256': cutlist_digest([ends]), 'first_ends': ends[:64],
            'last_ends': ends[-16:]}


def _config5_job(job):
    sid, edit, size = job
    import hashlib as _h
    data = synth.stream_bytes(size, synth.DEFAULT_SEED, sid)
    if edit is not None:
        data = synth.apply_edit(data, edit[0], edit[1], bytes.fromhex(edit[2]))
    raw = data.tobytes()
    ends = _ref_ends(MIN_DEF, MAX_DEF, [raw])
    digests, start = [], 0
    for e in ends:
        digests.append(_h.blake2b(raw[start:e]).digest())
        start = e
    return sid, ends, digests


def make_config5(pool, n_streams=1024, n_edit=512, size=64 << 20):
    """Config 5: re-chunk of the edited copies of config 2 (synth.edit_plan) and the dedup
    ratio = bytes of edited-set chunks whose content (BLAKE2b-512, as replicat digests chunks,
    repository.py:1462) occurs among the original set's chunks / edited-set bytes."""
    plan = synth.edit_plan(n_streams, n_edit, size)
    orig = pool.map(_config5_job, [(i, None, size) for i in range(n_streams)], chunksize=4)
    orig_ends = [e for _, e, _ in sorted(orig, key=lambda r: r[0])]
    known = {d for _, _, ds in orig for d in ds}
    jobs = [(sid, (kind, off, payload.hex()), size) for sid, kind, off, payload in plan]
    edited = sorted(pool.map(_config5_job, jobs, chunksize=4), key=lambda r: r[0])
    dup = total = 0
    per_kind = {}
    for (sid, kind, off, payload), (sid2, ends, digests) in zip(plan, edited):
        assert sid == sid2
        start = 0
        d_bytes = 0
        for e, dg in zip(ends, digests):
            if dg in known:
                d_bytes += e - start
            start = e
        dup += d_bytes
        total += ends[-1]
        k = per_kind.setdefault(kind, [0, 0])
        k[0] += d_bytes
        k[1] += ends[-1]
    unedited = (n_streams - n_edit) * size
    return {'name': 'config5', 'streams': n_streams, 'edited': n_edit, 'size': size,
            'seed': synth.DEFAULT_SEED, 'plan_seed': 5, 'min': MIN_DEF, 'max': MAX_DEF,
            'params': None,
            'original_sha256': cutlist_digest(orig_ends),
            'edited_sha256': cutlist_digest([e for _, e, _ in edited]),
            'edited_chunks': sum(len(e) for _, e, _ in edited),
            'edited_first_ends': [e for _, e, _ in edited[:6]],
            'dup_bytes_edited': dup, 'total_bytes_edited': total,
            'dup_bytes_by_kind': per_kind,
            'dedup_ratio_edited': dup / total,
            'dedup_ratio_set': (dup + unedited) / (total + unedited)}


# ----------------------------------------------------- config 4: 128 x 8 GiB (config4.json)

C4_STREAMS, C4_SIZE, C4_GPUS = 128, 8 << 30, 8


def _config4_job(sid):
    """One 8 GiB stream of config 4, one piece (P = 0), cut by the REFERENCE's native
    ``next_cut`` exactly as its adapter cuts a single piece (adapters.py:290-305: every call is
    final, the buffer is the uncut rest) -- on a zero-copy view instead of the adapter's
    bytearray, whose copy of an 8 GiB piece would double the memory.  The bytes come from the
    oracle's C splitmix filler (the same bytes as synth.stream_bytes and rc_fill_splitmix)."""
    import numpy as np
    from oracle import oracle as o
    data = np.empty(C4_SIZE, dtype=np.uint8)
    o.lib().oc_fill_splitmix(data.ctypes.data, C4_SIZE, synth.DEFAULT_SEED, sid)
    ch = REF_EXT._gclmulchunker(MIN_DEF, MAX_DEF, b'\xff' * 16)
    mv = memoryview(data)
    pos, ends = 0, []
    while pos < C4_SIZE:
        c = ch.next_cut(mv[pos:], True)
        if not c:
            break
        pos += c
        ends.append(pos)
    del mv, data
    return sid, ends


def _config4_adapter_check(sid=0, piece=16 << 20):
    """Stream ``sid`` through replicat's adapter itself, fed 16 MiB pieces: P = L - 16 MiB,
    which for L - P >= max cuts exactly like the single piece."""
    base = synth.stream_base(synth.DEFAULT_SEED, sid)

    def pieces():
        for off in range(0, C4_SIZE, piece):
            yield synth.splitmix_words(base, off // 8, piece // 8).view('<u1').tobytes()
    return _ref_ends(MIN_DEF, MAX_DEF, pieces())


def make_config4(procs=4):
    """Config 4 (SURVEY §8 d): 128 streams x 8 GiB, stream i on GPU i mod 8, one piece each.
    Per-stream cut-list SHA-256 (+ first/last ends) and, per GPU, the digest over its 16
    streams in shard order (bench.shard_ids('4', g, 16) = g, g + 8, ...)."""
    with mp.get_context('fork').Pool(procs) as pool:
        chk = pool.apply_async(_config4_adapter_check)
        res = dict(pool.imap_unordered(_config4_job, range(C4_STREAMS)))
        adapter_ends = chk.get()
    assert adapter_ends == res[0], 'adapter over 16 MiB pieces disagrees with one piece'
    streams = [{'id': i, 'chunks': len(res[i]), 'sha256': cutlist_digest([res[i]]),
                'first_ends': res[i][:8], 'last_ends': res[i][-8:]} for i in range(C4_STREAMS)]
    per_gpu = []
    for g in range(C4_GPUS):
        ids = [g + C4_GPUS * k for k in range(C4_STREAMS // C4_GPUS)]
        per_gpu.append({'gpu': g, 'ids': ids, 'chunks': sum(len(res[i]) for i in ids),
                        'sha256': cutlist_digest([res[i] for i in ids])})
    return {'name': 'config4', 'streams': C4_STREAMS, 'size': C4_SIZE, 'gpus': C4_GPUS,
            'seed': synth.DEFAULT_SEED, 'min': MIN_DEF, 'max': MAX_DEF, 'params': None,
            'last_piece': 0, 'adapter_checked_stream': 0, 'per_stream': streams,
            'per_gpu': per_gpu}


# ------------------------------ every rank's own shard of a multi-GPU line (ranks.json)

RANKS, RANK_STREAMS, RANK_SIZE = 8, 1024, 64 << 20
RANK_SEEDED = 128                     # the seeded key's streams per shard (encrypted leg)
RANK_3III, RANK_3III_SIZE = 65536, 1 << 20


def _ref_cut(data, mn, mx, key):
    """The REFERENCE's ``next_cut`` over one single-piece stream exactly as its adapter calls it
    (adapters.py:290-305: every call final, the buffer the uncut rest), on a zero-copy view."""
    ch = REF_EXT._gclmulchunker(mn, mx, key)
    mv, size = memoryview(data), len(data)
    pos, ends = 0, []
    while pos < size:
        c = ch.next_cut(mv[pos:], True)
        if not c:
            break
        pos += c
        ends.append(pos)
    return ends


def _rank_stream(sid, size):
    import numpy as np
    from oracle import oracle as o
    data = np.empty(size, dtype=np.uint8)
    o.lib().oc_fill_splitmix(data.ctypes.data, size, synth.DEFAULT_SEED, sid)
    return data


def _rank_job(job):
    """One config-2-shaped stream of a rank's shard: its cut list under the unencrypted key and
    its chunks' BLAKE2b-512 digests (config 5's content identity, repository.py:1462); with
    ``edit`` the edited copy instead; with ``key`` the cut list under that key only."""
    import hashlib as _h
    kind, sid, size, mn, mx, key, edit = job
    data = _rank_stream(sid, size)
    if edit is not None:
        data = synth.apply_edit(data, edit[0], edit[1], bytes.fromhex(edit[2]))
    ends = _ref_cut(data, mn, mx, b'\xff' * 16 if key is None else bytes.fromhex(key))
    digests = []
    if kind == 'digests':
        raw, start = memoryview(data), 0
        for e in ends:
            digests.append(_h.blake2b(raw[start:e]).digest())
            start = e
    return sid, ends, digests


def rank_edit_plan(rank, n=RANK_STREAMS, size=RANK_SIZE):
    """Config 5's edits on rank ``rank``'s shard (local stream indices): rank 0's plan is the
    single-GPU one (seed 5, large.json); rank r uses seed 5 + r.  bench.Config5 uses the same."""
    return synth.edit_plan(n, n // 2, size, seed=5 + rank)


def make_ranks(procs=8):
    """Per-rank fixtures for multi-GPU lines (bench.shard_ids: rank r chunks streams
    r*n .. r*n + n - 1): config 2 under key ff (the whole shard), the seeded key (the shard's
    first 128 streams), config 5 (the shard's own edit plan and dedup against the shard) and
    config 3 (iii) (65,536 x 1 MiB per rank), all cut by the reference's ``next_cut``.  Rank 0's
    entries must equal the single-GPU fixtures (digests.json, large.json): checked here."""
    seeded = synth.seeded_key(1).hex()
    out = {'ranks': RANKS, 'seed': synth.DEFAULT_SEED, 'min': MIN_DEF, 'max': MAX_DEF,
           'config2_ff': [], 'config2_seeded': [], 'config5': [], 'config3iii': []}
    with mp.get_context('fork').Pool(procs) as pool:
        for r in range(RANKS):
            ids = [r * RANK_STREAMS + i for i in range(RANK_STREAMS)]
            res = sorted(pool.map(_rank_job, [('digests', s, RANK_SIZE, MIN_DEF, MAX_DEF, None,
                                               None) for s in ids], chunksize=4))
            ends = [e for _, e, _ in res]
            known = {d for _, _, ds in res for d in ds}
            out['config2_ff'].append({'rank': r, 'first_id': ids[0], 'streams': len(ids),
                                      'chunks': sum(map(len, ends)),
                                      'sha256': cutlist_digest(ends)})
            sd = sorted(pool.map(_rank_job, [('cuts', s, RANK_SIZE, MIN_DEF, MAX_DEF, seeded,
                                              None) for s in ids[:RANK_SEEDED]], chunksize=2))
            out['config2_seeded'].append({'rank': r, 'first_id': ids[0], 'streams': RANK_SEEDED,
                                          'params': seeded,
                                          'chunks': sum(len(e) for _, e, _ in sd),
                                          'sha256': cutlist_digest([e for _, e, _ in sd])})
            plan = rank_edit_plan(r)
            jobs = [('digests', ids[loc], RANK_SIZE, MIN_DEF, MAX_DEF, None,
                     (kind, off, payload.hex())) for loc, kind, off, payload in plan]
            ed = sorted(pool.map(_rank_job, jobs, chunksize=2))
            dup = total = 0
            for _, e_ends, e_dig in ed:
                start = 0
                for e, dg in zip(e_ends, e_dig):
                    if dg in known:
                        dup += e - start
                    start = e
                total += e_ends[-1]
            out['config5'].append({'rank': r, 'plan_seed': 5 + r, 'edited': len(plan),
                                   'original_sha256': out['config2_ff'][-1]['sha256'],
                                   'edited_sha256': cutlist_digest([e for _, e, _ in ed]),
                                   'dup_bytes_edited': dup, 'total_bytes_edited': total})
            ids3 = [r * RANK_3III + i for i in range(RANK_3III)]
            e3 = sorted(pool.map(_rank_job, [('cuts', s, RANK_3III_SIZE, 2_000, 80_000, None, None)
                                             for s in ids3], chunksize=256))
            out['config3iii'].append({'rank': r, 'first_id': ids3[0], 'streams': RANK_3III,
                                      'chunks': sum(len(e) for _, e, _ in e3),
                                      'sha256': cutlist_digest([e for _, e, _ in e3])})
            print('rank', r, out['config2_ff'][-1]['sha256'][:16],
                  out['config2_seeded'][-1]['sha256'][:16], out['config5'][-1]['dup_bytes_edited'],
                  out['config3iii'][-1]['sha256'][:16], flush=True)
    with open(os.path.join(HERE, 'digests.json')) as f:
        single = {d['name']: d for d in json.load(f)}
    with open(os.path.join(HERE, 'large.json')) as f:
        c5 = {d['name']: d for d in json.load(f)}['config5']
    assert out['config2_ff'][0]['sha256'] == single['config2_ff']['sha256']
    assert out['config2_seeded'][0]['sha256'] == single['config2_seeded_first128']['sha256']
    assert out['config3iii'][0]['sha256'] == single['config3iii']['sha256']
    assert (out['config5'][0]['edited_sha256'], out['config5'][0]['dup_bytes_edited'],
            out['config5'][0]['total_bytes_edited']) == (c5['edited_sha256'],
                                                         c5['dup_bytes_edited'],
                                                         c5['total_bytes_edited'])
    return out


def make_ranks_small(n=2, size=16 << 20):
    """A small config-2-shaped shard per rank (n streams of 16 MiB, default parameters, key ff,
    streams r*n ..): what the CPU tests' stand-in ranks chunk, so that every rank of a world-2
    line carries a flag there too."""
    per_rank = []
    for r in range(RANKS):
        ends = [_ref_cut(_rank_stream(r * n + i, size), MIN_DEF, MAX_DEF, b'\xff' * 16)
                for i in range(n)]
        per_rank.append({'rank': r, 'first_id': r * n, 'chunks': sum(map(len, ends)),
                         'sha256': cutlist_digest(ends)})
    return {'streams': n, 'size': size, 'per_rank': per_rank}


def _config3ii_world(world):
    return make_config3ii(size=world * (64 << 30))


def make_config3ii_worlds(worlds=(2, 4, 8)):
    """Config 3 (ii) as bench.py runs it on `world` ranks: ONE stream of world x 64 GiB (last
    piece the final 1 MiB) split over the ranks, the whole spliced list on every rank."""
    with mp.get_context('fork').Pool(len(worlds)) as pool:
        out = pool.map(_config3ii_world, worlds)
    for w, d in zip(worlds, out):
        d['world'] = w
    return out


# ------------------------------------- the reference's benchmark harness (harness.json)

def make_harness():
    """Cut list of ``Repository._benchmark_chunker``'s stream (repository.py:1984-2008): 10 x
    512,000,000-byte Random(0) pieces through replicat's adapter over its own extension."""
    ends = _ref_ends(MIN_DEF, MAX_DEF, synth.harness_buffers())
    n, size = synth.HARNESS_NUMBER, synth.HARNESS_SIZE
    return {'name': 'harness', 'number': n, 'size': size, 'seed': 0, 'length': n * size,
            'last_piece': (n - 1) * size, 'min': MIN_DEF, 'max': MAX_DEF, 'params': None,
            'chunks': len(ends), 'sha256': cutlist_digest([ends]), 'first_ends': ends[:16],
            'last_ends': ends[-16:]}


def make_config3iii_full(pool):
    """Config 3 (iii) in full: 65,536 x 1 MiB, min 2,000 / max 80,000 (digests.json keeps the
    first 4,096 too)."""
    jobs = [('splitmix', (synth.DEFAULT_SEED, i, 1 << 20, 0, 2_000, 80_000, None))
            for i in range(65536)]
    ends = pool.map(_stream_job, jobs, chunksize=64)
    return {'name': 'config3iii', 'streams': 65536, 'size': 1 << 20, 'seed': synth.DEFAULT_SEED,
            'min': 2_000, 'max': 80_000, 'params': None, 'chunks': sum(map(len, ends)),
            'sha256': cutlist_digest(ends)}


# ------------------------------------------------------------- module surface

from golden_surface import SURFACE_CASES, surface_call  # noqa: E402


def make_surface():
    mod = REF_EXT
    out = []
    for name, args, call in SURFACE_CASES:
        try:
            r = surface_call(mod, args, call)
            out.append({'name': name, 'args': args, 'call': call, 'result': list(r) if isinstance(r, tuple) else r,
                        'error': None})
        except Exception as e:  # noqa: BLE001 - recording the reference's behaviour
            msg = str(e) if isinstance(e, ValueError) else None
            out.append({'name': name, 'args': args, 'call': call, 'result': None,
                        'error': type(e).__name__, 'message': msg})
    return out


# ------------------------------------------------------------------ snapshots


def snapshot_sets():
    """File sets (name -> bytes) for snapshot framing fixtures, reproducible without the
    reference: the reference test's own set (test_repository.py:603-620, Random(0)) and a
    synthetic set whose files straddle the 16 MiB piece size."""
    rnd = random.Random(0)
    sizes = [('a', 4099), ('b', 32), ('c', 1023), ('d', 517), ('e', 2), ('f', 128), ('g', 64),
             ('h', 2048), ('i', 19), ('j', 8), ('k', 4), ('l', 256), ('m', 1), ('n', 0),
             ('o', 0), ('p', 19)]
    test_set = {name: (rnd.randbytes(n) if n else b'') for name, n in sizes}
    big = {}
    for i, n in enumerate([0, 3, (16 << 20) - 1, (16 << 20) + 5, 7_000_001, (33 << 20) + 2]):
        big['f%02d' % i] = synth.stream_bytes(n, synth.DEFAULT_SEED, 900 + i).tobytes() if n else b''
    return [('reference_test_set', test_set, 256, 512, None),
            ('reference_test_set_seeded', test_set, 256, 512, bytes(range(16))),
            ('big_files', big, MIN_DEF, MAX_DEF, None)]


def reference_stream_pieces(files):
    """_stream_files (repository.py:1413-1452) over in-memory files, sorted per :1352."""
    order = sorted(files.items(), key=lambda kv: (len(kv[1]), kv[0]))
    prev_len = None
    for name, data in order:
        if prev_len is not None and -prev_len % 4:
            yield bytes(-prev_len % 4)
        for i in range(0, len(data), 16_777_216):
            yield data[i:i + 16_777_216]
        prev_len = len(data)


def make_snapshots():
    out = []
    for name, files, mn, mx, params in snapshot_sets():
        lens = ref_lengths(mn, mx, list(reference_stream_pieces(files)), params)
        out.append({'name': name, 'min': mn, 'max': mx,
                    'params': None if params is None else params.hex(), 'lengths': lens})
    return out


def main():
    quick = '--quick' in sys.argv
    if '--harness' in sys.argv:
        h = make_harness()
        print('harness', h['chunks'], h['sha256'], flush=True)
        with open(os.path.join(HERE, 'harness.json'), 'w') as f:
            json.dump(h, f, separators=(',', ':'))
            f.write('\n')
        return
    if '--config3iii' in sys.argv:
        with mp.get_context('fork').Pool(8) as pool:
            d = make_config3iii_full(pool)
        print('config3iii', d['chunks'], d['sha256'], flush=True)
        path = os.path.join(HERE, 'digests.json')
        with open(path) as f:
            sets = [s for s in json.load(f) if s['name'] != 'config3iii']
        with open(path, 'w') as f:
            json.dump(sets + [d], f, separators=(',', ':'))
            f.write('\n')
        return
    if '--ranks-extra' in sys.argv:
        # the small per-rank shards and config 3 (ii) at 2 / 4 / 8 ranks, added to ranks.json
        path = os.path.join(HERE, 'ranks.json')
        with open(path) as f:
            d = json.load(f)
        d['small'] = make_ranks_small()
        if '--no-3ii' not in sys.argv:
            d['config3ii'] = make_config3ii_worlds()
            for c in d['config3ii']:
                print('config3ii world', c['world'], c['chunks'], c['sha256'][:16], flush=True)
        with open(path, 'w') as f:
            json.dump(d, f, indent=1)
            f.write('\n')
        return
    if '--ranks' in sys.argv:
        d = make_ranks()
        with open(os.path.join(HERE, 'ranks.json'), 'w') as f:
            json.dump(d, f, indent=1)
            f.write('\n')
        return
    if '--config4' in sys.argv:
        c4 = make_config4()
        print('config4', [g['sha256'][:16] for g in c4['per_gpu']], flush=True)
        with open(os.path.join(HERE, 'config4.json'), 'w') as f:
            json.dump(c4, f, separators=(',', ':'))
            f.write('\n')
        return
    if '--large' in sys.argv:
        with mp.get_context('fork').Pool(8) as pool:
            r3 = pool.apply_async(make_config3ii)
            c5 = make_config5(pool)
            print('config5', c5['dedup_ratio_edited'], c5['original_sha256'], flush=True)
            c3 = r3.get()
            print('config3ii', c3['chunks'], c3['sha256'], flush=True)
        with open(os.path.join(HERE, 'large.json'), 'w') as f:
            json.dump([c3, c5], f, separators=(',', ':'))
            f.write('\n')
        return
    if '--snapshots-only' in sys.argv:
        with open(os.path.join(HERE, 'snapshots.json'), 'w') as f:
            json.dump(make_snapshots(), f, separators=(',', ':'))
            f.write('\n')
        return
    if '--surface-only' in sys.argv:
        with open(os.path.join(HERE, 'surface.json'), 'w') as f:
            json.dump(make_surface(), f, indent=0)
            f.write('\n')
        return
    def dump(name, obj):
        with open(os.path.join(HERE, name), 'w') as f:
            json.dump(obj, f, separators=(',', ':'))
            f.write('\n')
    dump('surface.json', make_surface())
    dump('snapshots.json', make_snapshots())
    dump('small_cases.json', make_small_cases())
    dump('known_answers.json', make_known_answers())
    with mp.get_context('fork').Pool(8) as pool:
        dump('streams.json', make_streams(pool))
        dump('digests.json', make_digests(pool, quick))


if __name__ == '__main__':
    main()
