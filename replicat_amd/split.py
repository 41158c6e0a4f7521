"""One long stream across several devices (config 3 (ii)).

A snapshot is ONE stream (repository.py:1352,1413-1452): its cuts form a chain in which every
cut depends on the previous one.  To spread one stream over G devices, the stream is split into
contiguous segments; device r chunks its segment plus a halo of the next one with a
*speculative* chain that starts at the segment start o_r as if a chunk began there.  Chains that
share one position coincide from there on (the next cut is a function of the position alone),
and the true chain, followed from device r-1's list into the halo, meets device r's speculative
chain after about one chunk.  The host splices the lists; the exchange is a handful of u64
offsets per device (a host-side gather, no device collective).  When no shared position exists
in the halo, the owner of the segment recomputes its chain from the true position (an exact
fallback, never needed on random data at a 4 x max halo).

Framing of a window [a, e) of a stream (L bytes, last piece at P), following the closed form of
SURVEY.md §8 (a0) S4 (argmax at s iff P - s >= max or L - s >= 2 max, adapters.py:290-305):

* an interior window (e + max <= L) is chunked OPEN (cut while e - s >= max): at every such s,
  L - s >= 2 max, so the true rule is argmax whatever P is;
* the last window (e = L) is final, with last piece at max(0, P - a).
"""
from dataclasses import dataclass


@dataclass(frozen=True)
class Window:
    start: int        # o_r: first byte of the segment (a multiple of `align`)
    end: int          # end of the bytes chunked (segment end + halo, or L)
    last_piece: int   # P relative to `start` (final windows)
    open: bool        # interior window: non-final prefix semantics (RC_OPEN)


def halo_bytes(max_length: int) -> int:
    return 4 * max_length


def plan_windows(L: int, P: int, world: int, max_length: int, align: int = 64, halo=None):
    """The window of every rank, segment starts aligned (cuts are multiples of 4 from 0)."""
    halo = halo_bytes(max_length) if halo is None else halo
    starts = [(L * r // world) // align * align for r in range(world)] + [L]
    out = []
    for r in range(world):
        a = starts[r]
        e = starts[r + 1] + halo
        if r == world - 1 or e + max_length > L:
            out.append(Window(a, L, max(0, P - a), False))
        else:
            out.append(Window(a, e, 0, True))
    return out


def splice(windows, chains):
    """Join per-window chains into the true chain.

    ``chains[r] = (entry, ends)``: absolute cut ends of the chain that starts at ``entry``
    inside window r (``entry = windows[r].start`` for a speculative chain; windows[0] is the
    true start).  Returns ``(ends, None, None)`` when the chains join, otherwise
    ``(None, r, entry)``: window r must be recomputed from the true position ``entry``."""
    entry0, ends0 = chains[0]
    assert entry0 == 0 and windows[0].start == 0
    true_pos = [0] + [int(e) for e in ends0]   # positions: chunk starts, then the final end
    for r in range(1, len(windows)):
        entry, ends = chains[r]
        pos_r = [int(entry)] + [int(e) for e in ends]
        index = {p: i for i, p in enumerate(pos_r)}
        k = next((i for i, t in enumerate(true_pos) if t >= entry and t in index), None)
        if k is None:
            # the true chain stopped (end of window r-1) without meeting chain r: continue it
            # from its last position, which lies inside window r (halo > max_length)
            return None, r, true_pos[-1]
        true_pos = true_pos[:k + 1] + pos_r[index[true_pos[k]] + 1:]
    return true_pos[1:], None, None


def chunk_split(chunk_window, windows, rank, gather):
    """The multi-process protocol.  ``chunk_window(window, entry)`` chunks this rank's window
    from ``entry`` and returns absolute cut ends; ``gather(obj)`` returns every rank's ``obj``
    (a host-side all-gather).  Every rank returns the whole true cut list."""
    w = windows[rank]
    chains = gather((w.start, chunk_window(w, w.start)))
    rounds = 0
    while True:
        ends, r, entry = splice(windows, chains)
        if r is None:
            return ends, rounds
        rounds += 1
        mine = (entry, chunk_window(windows[r], entry)) if rank == r else None
        chains[r] = gather(mine)[r]


def merge_points(windows, info):
    """Slice bounds from a compact exchange: ``info[r] = (entry, head, tail)`` with ``head`` the
    first cut ends of window r's chain from ``entry`` and ``tail`` its last ones (absolute).
    Returns ``bounds`` (rank r keeps its cuts p with bounds[r] < p <= bounds[r + 1], the last
    rank to its end), or None when a boundary cannot be settled from the exchanged cuts (the
    caller then runs chunk_split).  At boundary r the true chain, followed in window r - 1's
    tail, meets window r's speculative chain at a position both hold: from there they are the
    same chain, so any common position after window r - 1's own merge is a valid splice."""
    bounds = [0]
    for r in range(1, len(windows)):
        entry, head, _ = info[r]
        spec = {int(entry)}
        spec.update(int(p) for p in head)
        tail_prev = [int(p) for p in info[r - 1][2]]
        p = next((t for t in tail_prev if t >= entry and t in spec and t > bounds[-1]), None)
        if p is None:
            return None
        bounds.append(p)
    return bounds

