"""One stream over several ranks (replicat_amd/split.py) on the CPU: the
window plan, the splice (including the exact fallback when the halo holds no shared position)
and the gloo world-size-2 protocol.  The oracle plays the per-rank chunker here; on the GPU
bench.py's Config3ii does the same with the HIP chunker."""
import os
import random
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from replicat_amd import split, synth


def _oracle():
    from oracle import oracle as o
    o.lib()
    return o


def oracle_window(data, mn, mx, key):
    """chunk_window for the oracle: the chain from `entry` over window w of `data`."""
    o = _oracle()

    def chunk_window(w, entry):
        seg = np.ascontiguousarray(data[entry:w.end])
        if w.open:
            # RC_OPEN semantics: the final-call chain with P = L, cut while L - s >= max
            full = o.chunk_stream(seg, mn, mx, key, len(seg))
            out, s = [], 0
            for e in full:
                if len(seg) - s < mx:
                    break
                out.append(e)
                s = e
        else:
            out = o.chunk_stream(seg, mn, mx, key, max(0, w.last_piece - (entry - w.start)))
        return [entry + int(e) for e in out]
    return chunk_window


def run_local(data, P, world, mn, mx, key, halo=None):
    windows = split.plan_windows(len(data), P, world, mx, halo=halo)
    fn = oracle_window(data, mn, mx, key)
    chains = [(w.start, fn(w, w.start)) for w in windows]
    rounds = 0
    while True:
        ends, r, entry = split.splice(windows, chains)
        if r is None:
            return ends, rounds
        rounds += 1
        chains[r] = (entry, fn(windows[r], entry))


def test_plan_windows():
    L, P, mx = 10_000_000, 9_000_000, 100_000
    ws = split.plan_windows(L, P, 4, mx)
    assert ws[0].start == 0 and ws[-1].end == L and not ws[-1].open
    assert all(w.start % 64 == 0 for w in ws)
    for a, b in zip(ws, ws[1:]):
        assert a.end >= b.start + split.halo_bytes(mx) or a.end == L
        assert a.open == (a.end + mx <= L)
    assert ws[-1].last_piece == P - ws[-1].start
    # a window that would reach within max of the end becomes final
    ws = split.plan_windows(1_000_000, 0, 3, 200_000)
    assert all(w.end == 1_000_000 for w in ws[1:]) or ws[1].end + 200_000 <= 1_000_000


@pytest.mark.parametrize('world', [1, 2, 3, 5])
@pytest.mark.parametrize('seed', [1, 2])
def test_splice_matches_whole_stream(world, seed):
    o = _oracle()
    mn, mx = 500, 10_000
    key = synth.seeded_key(seed)
    rnd = random.Random(seed)
    L = 400_000 + rnd.randrange(1000)
    data = synth.stream_bytes(L, synth.DEFAULT_SEED, 40 + seed)
    P = rnd.choice([0, L - 7_000, L // 2])
    exp = o.chunk_stream(data, mn, mx, key, P)
    got, rounds = run_local(data, P, world, mn, mx, key)
    assert got == exp
    assert rounds == 0  # chains meet inside a 4 x max halo on random data


@pytest.mark.parametrize('world', [2, 4])
def test_splice_fallback_is_exact(world):
    """Chains that never meet (here: speculative lists shifted off the 4-byte grid) force the
    recompute-from-the-true-position path, which must still give the exact chain."""
    o = _oracle()
    mn, mx = 2_000, 10_000
    key = b'\xff' * 16
    data = synth.stream_bytes(300_000, synth.DEFAULT_SEED, 77)
    exp = o.chunk_stream(data, mn, mx, key, 0)
    windows = split.plan_windows(len(data), 0, world, mx)
    fn = oracle_window(data, mn, mx, key)
    chains = [(w.start, fn(w, w.start)) for w in windows]
    chains = [chains[0]] + [(a, [e + 2 for e in ends]) for a, ends in chains[1:]]
    rounds = 0
    while True:
        ends, r, entry = split.splice(windows, chains)
        if r is None:
            break
        rounds += 1
        assert windows[r].start <= entry < windows[r].end and entry % 4 == 0
        chains[r] = (entry, fn(windows[r], entry))
    assert ends == exp
    assert rounds == world - 1


def test_splice_on_repetitive_data():
    """Zero bytes: every key is k1, so every chain cuts at roundup4(min); speculative chains
    from aligned segment starts land on the true grid or not, both must splice exactly."""
    o = _oracle()
    mn, mx = 1_000, 8_000
    key = b'\x11' * 16
    data = np.zeros(200_000, dtype=np.uint8)
    exp = o.chunk_stream(data, mn, mx, key, 0)
    for world in (2, 3, 7):
        got, _ = run_local(data, 0, world, mn, mx, key)
        assert got == exp


# ------------------------------------------------------------------ gloo, world size 2

def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mn, mx = 500, 10_000
    key = synth.seeded_key(9)
    L = 333_333
    data = synth.stream_bytes(L, synth.DEFAULT_SEED, 5)
    P = L - 4_096
    windows = split.plan_windows(L, P, world, mx)

    def gather(obj):
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    ends, rounds = split.chunk_split(oracle_window(data, mn, mx, key), windows, rank, gather)
    q.put((rank, ends, rounds))
    dist.barrier()
    dist.destroy_process_group()


def test_chunk_split_gloo_two_ranks():
    world, port = 2, _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o = _oracle()
    L = 333_333
    data = synth.stream_bytes(L, synth.DEFAULT_SEED, 5)
    exp = o.chunk_stream(data, 500, 10_000, synth.seeded_key(9), L - 4_096)
    assert res[0][1] == exp and res[1][1] == exp


@pytest.mark.parametrize('world', [2, 3, 5])
@pytest.mark.parametrize('k', [4, 64])
def test_merge_points_compact_exchange(world, k):
    """bench.py's compact exchange: from each window's first and last k cut ends alone, the
    slice bounds reproduce the whole stream's cut list (or ask for the full protocol)."""
    o = _oracle()
    mn, mx = 500, 10_000
    key = synth.seeded_key(world)
    L = 600_000 + 13 * world
    data = synth.stream_bytes(L, synth.DEFAULT_SEED, 70 + world)
    P = L - 7_000
    windows = split.plan_windows(L, P, world, mx)
    fn = oracle_window(data, mn, mx, key)
    lists = [fn(w, w.start) for w in windows]
    info = [(w.start, c[:k], c[-k:]) for w, c in zip(windows, lists)]
    bounds = split.merge_points(windows, info)
    if bounds is None:  # 4 cuts need not span the halo (~8 chunks here): the caller falls back
        assert k == 4
        return
    ends = []
    for r, c in enumerate(lists):
        hi = bounds[r + 1] if r + 1 < world else None
        ends += [p for p in c if p > bounds[r] and (hi is None or p <= hi)]
    assert ends == o.chunk_stream(data, mn, mx, key, P)
    # nothing exchanged past the entries: no bounds, the caller falls back
    assert split.merge_points(windows, [(w.start, [], []) for w in windows]) is None
