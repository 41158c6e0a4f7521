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
import io
import os
import stat
import threading
from dataclasses import dataclass, field
from typing import Iterator, List, Optional, Sequence, Tuple

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


_READ_POOL = None
_READ_POOL_LOCK = threading.Lock()
READ_SPLIT = 4 << 20   # the smallest part of a piece read by one thread


def _read_pool():
    global _READ_POOL
    with _READ_POOL_LOCK:
        if _READ_POOL is None:
            from concurrent.futures import ThreadPoolExecutor
            _READ_POOL = ThreadPoolExecutor(max_workers=8, thread_name_prefix='rc-read')
        return _READ_POOL


def _pread_full(fd, view, off) -> int:
    """Read view's length from fd at off (os.preadv releases the GIL); short only at EOF."""
    done, n = 0, len(view)
    while done < n:
        r = os.preadv(fd, [view[done:]], off + done)
        if r == 0:
            break
        done += r
    return done


class PieceReader:
    """The pieces replicat's _stream_files yields (repository.py:1413-1447) for already-sorted
    `paths`, read on demand into a caller's buffer: files in order, each in reads of at most
    PIECE bytes (one ``read(PIECE)`` per piece, as the reference; a buffered file or BytesIO is
    read straight into the buffer with ``readinto``, which returns the same bytes), and a zero
    piece of (-len) % 4 bytes after every file that is followed by another.

    `files` receives a record (``record(path=, stream_start=, stream_end=)``) when a file is
    opened, and its stream_end grows as the file is read; `on_open(record, file_object)` runs
    once per opened file.  Both stream_pieces and the device snapshot producer
    (replicat_amd/pipeline.py) frame the stream through this one class.

    `threads` > 1: a piece of a regular file opened in binary mode is read as up to `threads`
    parts of at least READ_SPLIT bytes, in parallel (positional reads from a shared pool) --
    the same bytes as one read(PIECE) at the file's position: the piece ends at the first part
    that comes back short (end of file), and the file's next piece starts after it."""

    def __init__(self, paths: Sequence[str], files: Optional[list] = None, read=None,
                 record=None, on_open=None, threads: int = 1):
        self._threads = max(1, int(threads))
        self._fd = None     # a regular file read with positional reads (threads > 1)
        self._off = 0
        self._paths = iter(paths)
        self.files = files if files is not None else []
        self._open = read if read else (lambda p: open(p, 'rb'))
        self._record = record or SnapshotFile
        self._on_open = on_open
        self._cm = self._src = None
        self._next = None   # the path after the current file (known before its padding)
        self._pad = 0       # padding owed after the last closed file
        self.pos = 0        # stream bytes so far

    def read_into(self, dst) -> Optional[Tuple[int, int, Optional[int]]]:
        """Place the next piece at the start of `dst` (writable, at least PIECE bytes).  Returns
        (length, tag, file index) -- tag = the number of files known to be complete (data of
        file f: f; padding after file f: f + 1), file index None for padding -- or None at the
        end of the stream."""
        mv = memoryview(dst).cast('B')
        while True:
            if self._src is not None:
                n = self._read(mv)
                if n:
                    fi = len(self.files) - 1
                    self.files[fi].stream_end += n
                    self.pos += n
                    return n, fi, fi
                self.close()
                f = self.files[-1]
                self._pad = -(f.stream_end - f.stream_start) % ALIGNMENT
            if self._next is None:
                self._next = next(self._paths, None)
                if self._next is None:
                    return None
            if self._pad:
                pad, self._pad = self._pad, 0
                mv[:pad] = bytes(pad)
                self.pos += pad
                return pad, len(self.files), None
            path, self._next = self._next, None
            f = self._record(path=str(path), stream_start=self.pos, stream_end=self.pos)
            self.files.append(f)
            self._cm = self._open(path)
            self._src = self._cm.__enter__()
            self._fd = None
            if self._threads > 1 and isinstance(self._src, (io.BufferedReader, io.FileIO)):
                try:
                    fd = self._src.fileno()
                    if stat.S_ISREG(os.fstat(fd).st_mode):
                        self._fd, self._off = fd, self._src.tell()
                except (OSError, ValueError):
                    self._fd = None
            if self._on_open is not None:
                self._on_open(f, self._src)

    def _read(self, mv) -> int:
        if self._fd is not None:
            return self._pread(mv)
        src = self._src
        if isinstance(src, (io.BufferedReader, io.BytesIO)):
            return src.readinto(mv[:PIECE]) or 0
        piece = src.read(PIECE)
        mv[:len(piece)] = piece
        return len(piece)

    def _pread(self, mv) -> int:
        want = min(PIECE, len(mv))
        parts = max(1, min(self._threads, want // READ_SPLIT))
        step = -(-want // parts)
        ranges = [(a, min(a + step, want)) for a in range(0, want, step)]
        if len(ranges) == 1:
            got = [_pread_full(self._fd, mv[:want], self._off)]
        else:
            pool = _read_pool()
            futs = [pool.submit(_pread_full, self._fd, mv[a:b], self._off + a) for a, b in ranges]
            got = [f.result() for f in futs]
        n = 0
        for (a, b), g in zip(ranges, got):
            n += g
            if g < b - a:  # end of file: what later parts read (a file growing) is not this piece
                break
        self._off += n
        return n

    def close(self):
        self._fd = None
        cm, self._cm, self._src = self._cm, None, None
        if cm is not None:
            cm.__exit__(None, None, None)


def stream_pieces(paths: Sequence[str], files_out: Optional[List[SnapshotFile]] = None,
                  read=None, threads: int = 1) -> Iterator[bytes]:
    """The pieces replicat's _stream_files yields for already-sorted `paths`."""
    reader = PieceReader(paths, files_out, read, threads=threads)
    buf = bytearray(PIECE)
    try:
        while (got := reader.read_into(buf)) is not None:
            yield bytes(memoryview(buf)[:got[0]])
    finally:
        reader.close()


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


def file_parts(files, chunks):
    """(chunk index, file index, [part_start, part_end]) for every piece of a file inside a
    chunk, in the order _chunk_done records them (repository.py:1374-1411): chunks in stream
    order, the files a chunk touches from its last one backwards."""
    starts = [(f.stream_start, i) for i, f in enumerate(files)]
    for ci, c in enumerate(chunks):
        point = bisect.bisect_left(starts, (c.stream_end + 1,))
        for index in range(point - 1, -1, -1):
            fi = starts[index][1]
            f = files[fi]
            if f.stream_end < c.stream_start:
                break
            yield ci, fi, [max(f.stream_start - c.stream_start, 0),
                           min(f.stream_end, c.stream_end) - c.stream_start]


def file_ranges(files: Sequence[SnapshotFile], chunks: Sequence[SnapshotChunk]):
    """Per file, the (chunk index, [part_start, part_end]) list -- repository.py:1374-1411."""
    out = {f.path: [] for f in files}
    for ci, fi, part in file_parts(files, chunks):
        out[files[fi].path].append((ci, part))
    return out
