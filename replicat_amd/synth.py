"""Synthetic stream bytes shared by the tests, the golden-fixture script and bench.py.

Stream ``s`` of a workload with seed ``seed`` is the little-endian concatenation of the
64-bit words ``sm64(base ^ i)``, ``i = 0, 1, ...``, where ``base = (seed * GOLDEN) ^ (s << 34)``
and ``sm64`` is the splitmix64 finaliser.  The device generator in
``replicat_amd/csrc/chunker.hip`` (``rc_fill_splitmix``) and ``oracle/gclmul_oracle.c``
(``oc_fill_splitmix``) write exactly the same bytes, so a multi-GiB stream never needs
to cross PCIe to be checked.  ("splitmix64 counter stream (seed 0x5eed,
stream id in high bits)".)
"""
import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1
DEFAULT_SEED = 0x5EED


def stream_base(seed: int, stream: int) -> int:
    return ((seed * GOLDEN) & M64) ^ ((stream << 34) & M64)


def splitmix_words(base: int, start: int, count: int) -> np.ndarray:
    """Words ``start .. start+count-1`` of the counter stream with the given base."""
    with np.errstate(over='ignore'):
        z = np.arange(start, start + count, dtype=np.uint64)
        z ^= np.uint64(base)
        z += np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z


def stream_bytes(nbytes: int, seed: int = DEFAULT_SEED, stream: int = 0) -> np.ndarray:
    """``nbytes`` bytes of synthetic stream ``stream`` as a uint8 array."""
    words = splitmix_words(stream_base(seed, stream), 0, (nbytes + 7) // 8)
    return words.view('<u1')[:nbytes].copy() if nbytes % 8 else words.view('<u1')


def seeded_key(seed: int) -> bytes:
    """A 16-byte chunker key (k0 != 0) derived from ``seed`` -- the 'generic key' leg."""
    w = splitmix_words(stream_base(seed, 0x3FFF), 0, 2)
    if int(w[0]) == 0:
        w[0] = np.uint64(1)
    return w.astype('<u8').tobytes()


# ------------------------------------------- the reference's own benchmark stream (harness)

HARNESS_NUMBER = 10          # repository.py:1984 _benchmark_chunker(number=10, ...)
HARNESS_SIZE = 512_000_000   # ... size=512_000_000
HARNESS_PIECE = 16_777_216   # repository.py:1992 method(16_777_216)


def harness_buffers(number: int = HARNESS_NUMBER, size: int = HARNESS_SIZE, seed: int = 0):
    """The pieces ``Repository._benchmark_chunker`` feeds the chunker adapter
    (/root/reference/replicat/repository.py:1984-1999): one ``random.Random(seed)`` (what
    ``replicat.utils.compat.Random`` is on Python >= 3.9), and per piece 16 MiB ``randbytes``
    appended until ``size`` bytes, the excess dropped.  Each piece is one adapter piece, so the
    stream is ``number * size`` bytes whose last piece starts at ``(number - 1) * size``."""
    import random
    method = random.Random(seed).randbytes
    for _ in range(number):
        buf = bytearray()
        while len(buf) < size:
            buf += method(HARNESS_PIECE)
        del buf[size:]
        yield buf


# ------------------------------------------------------------------ config 5: edited copies

EDIT_KINDS = ('overwrite1', 'insert4', 'insert1')


def edit_plan(n_streams: int = 1024, n_edit: int = 512, size: int = 64 << 20, seed: int = 5):
    """``n_edit`` of the ``n_streams`` synthetic streams (a seeded
    choice) get one edit each at a seeded offset, cycling through a 1-byte overwrite (XOR 0x5a),
    a 4-byte insert and a 1-byte insert.  Returns ``[(stream, kind, offset, payload)]`` sorted
    by stream; ``payload`` is the inserted bytes (empty for an overwrite)."""
    import random
    rnd = random.Random(seed)
    ids = sorted(rnd.sample(range(n_streams), n_edit))
    plan = []
    for k, sid in enumerate(ids):
        kind = EDIT_KINDS[k % 3]
        if kind == 'overwrite1':
            plan.append((sid, kind, rnd.randrange(size), b''))
        else:
            n = 4 if kind == 'insert4' else 1
            plan.append((sid, kind, rnd.randrange(size + 1), rnd.randbytes(n)))
    return plan


def apply_edit(data: np.ndarray, kind: str, offset: int, payload: bytes) -> np.ndarray:
    """The edited copy of a stream (a new array; ``data`` is left alone)."""
    if kind == 'overwrite1':
        out = data.copy()
        out[offset] ^= 0x5A
        return out
    ins = np.frombuffer(payload, dtype=np.uint8)
    return np.concatenate([data[:offset], ins, data[offset:]])
