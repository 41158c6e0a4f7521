"""CPU model of the segment-parallel chain's join (kernels.hip: rc_spec_kernel, rc_merge_kernel
with boundary repair, rc_scan_kernel's entry recurrence, rc_copy_kernel), restated over the
oracle's chains: for random streams, segment lengths and extension counts -- including
extensions that run past the next segment's merge, where the true chain skips a list -- the
spliced lists must be the stream's own cut list.  Test infrastructure: checks the algorithm the
GPU kernels implement (the GPU tests check the kernels)."""
import random

import numpy as np
import pytest

from oracle import oracle as o

NO_MERGE = None


def chain_from(data, mn, mx, key, P, g):
    """Every cut of the chain that starts at chunk start g (the oracle on the stream's suffix:
    chunk starts and key offsets are 4-aligned, so the suffix's keys are the stream's)."""
    return [g + e for e in o.chunk_stream(data[g:], mn, mx, key, max(P - g, 0))]


def spec_lists(data, mn, mx, key, P, seg, ext):
    """rc_spec_kernel: segment i walks from i*seg until it has taken `ext` steps from a cut at or
    past its segment's end (or its chain ended); returns (lists, terminated flags)."""
    L = len(data)
    n_seg = (max(L - 1, 0)) // seg + 1
    lists, terms = [], []
    for i in range(n_seg):
        full = chain_from(data, mn, mx, key, P, i * seg)
        out, pos, taken, term = [], i * seg, 0, True
        for c in full:
            if pos >= (i + 1) * seg:
                if taken >= ext:
                    term = False
                    break
                taken += 1
            out.append(c)
            pos = c
        lists.append(out)
        terms.append(term)
    return lists, terms


def merge(lists, terms, data, mn, mx, key, P, seg, repair=True, max_repair=64):
    """rc_merge_kernel: per boundary k, (a, b) -- list k-1's first a entries lead to list k's
    entry b -- or NO_MERGE; with repair, list k-1 is extended in place until the lists meet, or
    given up once its chain passes list k's last entry (the meeting lies beyond what list k
    holds: the stream takes the sequential join)."""
    counts = [len(x) for x in lists]  # what the scan reads (rc_spec_kernel's seg_rcount copy)
    out = [None]
    for k in range(1, len(lists)):
        A, B, g = lists[k - 1][:], lists[k], k * seg
        res = NO_MERGE
        for ia, p in enumerate(A):
            if p < g:
                continue
            if p == g:
                res = (ia + 1, 0)
                break
            if p in B[:64]:
                res = (ia + 1, B.index(p) + 1)
                break
        if res is NO_MERGE and repair and A and not terms[k - 1] and len(B) <= 64:
            full = chain_from(data, mn, mx, key, P, (k - 1) * seg)
            ext = full[len(A):len(A) + max_repair]
            for c in ext:
                A.append(c)
                if c == g:
                    res = (len(A), 0)
                    break
                if c in B[:64]:
                    res = (len(A), B.index(c) + 1)
                    break
                if B and c > B[-1]:
                    break
            if res is NO_MERGE and len(A) == len(full):
                terms[k - 1] = True
            lists[k - 1] = A
            counts[k - 1] = len(A)
        out.append(res)
    return out, counts


def scan_copy(lists, terms, merges, counts):
    """rc_scan_kernel + rc_copy_kernel: entry_k = max(b_k, entry_{k-1} + b_k - a_k); list k's
    slice [entry_k, a_{k+1}) (to its end when the chain ends in it).  None = the stream would take
    the sequential join."""
    out, entry = [], 0
    for k in range(len(lists)):
        if k > 0:
            if merges[k] is NO_MERGE:
                return None
            a, b = merges[k]
            entry = max(b, entry + b - a)
        ends = k + 1 == len(lists) or merges[k + 1] is NO_MERGE
        hi = counts[k] if ends else merges[k + 1][0]
        if ends:
            if not terms[k] or entry > counts[k]:
                return None
            out += lists[k][entry:hi]
            return out
        out += lists[k][entry:hi]
    return out


@pytest.mark.parametrize('seed', range(24))
def test_join_model_vs_chain(seed):
    rnd = random.Random(seed)
    mx = rnd.choice([256, 512, 1024])
    mn = rnd.choice([4, mx // 8, mx // 2])
    key = rnd.randbytes(16)
    if key[:8] == bytes(8):
        key = b'\x01' + key[1:]
    L = rnd.randrange(20 * mx, 60 * mx)
    kind = seed % 3  # random, periodic, two-valued bytes
    data = (np.frombuffer(rnd.randbytes(L), np.uint8) if kind == 0 else
            np.resize(np.frombuffer(rnd.randbytes(rnd.randrange(1, 3 * mx)), np.uint8), L) if kind == 1
            else np.frombuffer(bytes(rnd.randrange(2) for _ in range(L)), np.uint8))
    P = rnd.choice([0, L, rnd.randrange(0, L + 1)])
    exp = o.chunk_stream(data, mn, mx, key, P)
    for seg_mult in (0.25, 1, 2, 3):
        for ext in (0, 1, 2, 4):
            seg = int(seg_mult * mx) // 4 * 4
            lists, terms = spec_lists(data, mn, mx, key, P, seg, ext)
            merges, counts = merge(lists, terms, data, mn, mx, key, P, seg)
            got = scan_copy(lists, terms, merges, counts)
            if got is None:  # the sequential join (rc_join_kernel) takes the stream
                # not with the defaults' margins on random data (a floor of 2 max_lengths,
                # 2 extension steps)
                assert kind != 0 or seg_mult < 2 or ext < 2, (seg_mult, ext)
                continue
            assert got == exp, (seg_mult, ext)


def test_join_model_repairs_and_skips():
    """The cases the round-3 join adds do occur: boundaries repaired (list k-1 extended) and
    lists skipped (an extension past the next boundary's merge), over the model's streams."""
    repaired = skipped = total = 0
    for seed in range(12):
        rnd = random.Random(1000 + seed)
        mx, mn = 512, 64
        key = rnd.randbytes(16)
        data = np.frombuffer(rnd.randbytes(rnd.randrange(30 * mx, 60 * mx)), np.uint8)
        L = len(data)
        exp = o.chunk_stream(data, mn, mx, key, L)
        # segments shorter than a chunk: an extension often runs past the next merge
        for seg, ext in ((mx // 4, 2), (mx // 2, 3), (mx, 1), (2 * mx, 0), (2 * mx, 4)):
            lists, terms = spec_lists(data, mn, mx, key, L, seg, ext)
            orig = [len(x) for x in lists]
            merges, counts = merge(lists, terms, data, mn, mx, key, L, seg)
            got = scan_copy(lists, terms, merges, counts)
            if got is None:
                continue
            assert got == exp
            total += 1
            repaired += sum(c != n for c, n in zip(counts, orig))
            entry = 0
            for k in range(1, len(merges)):
                if merges[k] is None:
                    break
                a, b = merges[k]
                skipped += entry > a
                entry = max(b, entry + b - a)
    assert total > 0 and repaired > 0 and skipped > 0, (total, repaired, skipped)
