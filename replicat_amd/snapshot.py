"""replicat's snapshot stream, chunked on the device (SURVEY.md §8 f rank 1; S6 framing).

replicat chunks ONE stream per snapshot (repository.py:1340-1452): the files sorted by
(size, path) (:1352), each read in pieces of at most 16 MiB (:1413, :1440), a zero piece of
(-len) % 4 bytes after every file but the last (:1415-1424), empty files contributing nothing.
Chunks straddle file boundaries and are mapped back to per-file byte ranges (:1374-1411).

`stream_pieces` restates that framing; `chunk_snapshot` feeds it to the batching shim
(replicat_amd.adapters.gclmulchunker), so the chunks equal the reference's for the same
files, parameters and key.
"""
import bisect
import os
from dataclasses import dataclass, field
from typing import Iterator, List, Optional, Sequence

from .adapters import gclmulchunker

PIECE = 16_777_216     # repository.py:1413 (_stream_files chunk_size)
ALIGNMENT = 4          # gclmulchunker.alignment, adapters.py:261


@dataclass
class SnapshotFile:
    path: str
    stream_start: int
    stream_end: int


@dataclass
class SnapshotChunk:
    stream_start: int
    stream_end: int
    data: bytes = field(repr=False)


def sort_files(paths: Sequence[os.PathLike]) -> List[str]:
    """repository.py:1352: small files first, ties by path string."""
    return sorted((str(p) for p in paths), key=lambda p: (os.stat(p).st_size, p))


def stream_pieces(paths: Sequence[str], files_out: Optional[List[SnapshotFile]] = None,
                  read=None) -> Iterator[bytes]:
    """The pieces replicat's _stream_files yields for already-sorted `paths`."""
    pos = 0
    prev = None
    for path in paths:
        if prev is not None:
            pad = -(prev.stream_end - prev.stream_start) % ALIGNMENT
            if pad:
                pos += pad
                yield bytes(pad)
        f = SnapshotFile(path=str(path), stream_start=pos, stream_end=pos)
        if files_out is not None:
            files_out.append(f)
        prev = f
        with (read(path) if read else open(path, 'rb')) as src:
            while piece := src.read(PIECE):
                pos += len(piece)
                f.stream_end += len(piece)
                yield piece


def chunk_snapshot(paths: Sequence[os.PathLike], *, min_length: int = gclmulchunker.MIN_LENGTH,
                   max_length: int = gclmulchunker.MAX_LENGTH, params: Optional[bytes] = None,
                   chunker: Optional[gclmulchunker] = None):
    """Chunk a snapshot's files as one stream.  Returns (files, chunks)."""
    chunker = chunker or gclmulchunker(min_length=min_length, max_length=max_length)
    files: List[SnapshotFile] = []
    chunks: List[SnapshotChunk] = []
    pos = 0
    for data in chunker(stream_pieces(sort_files(paths), files), params=params):
        chunks.append(SnapshotChunk(pos, pos + len(data), data))
        pos += len(data)
    return files, chunks


def file_ranges(files: Sequence[SnapshotFile], chunks: Sequence[SnapshotChunk]):
    """Per file, the (chunk index, [part_start, part_end]) list -- repository.py:1374-1411."""
    starts = [(f.stream_start, i) for i, f in enumerate(files)]
    out = {f.path: [] for f in files}
    for ci, c in enumerate(chunks):
        point = bisect.bisect_left(starts, (c.stream_end + 1,))
        for index in range(point - 1, -1, -1):
            f = files[starts[index][1]]
            if f.stream_end < c.stream_start:
                break
            part_start = max(f.stream_start - c.stream_start, 0)
            part_end = min(f.stream_end, c.stream_end) - c.stream_start
            out[f.path].append((ci, [part_start, part_end]))
    return out
