"""replicat's snapshot chunk producer on the device (SURVEY.md §8 f, ranks 1-4 together).

What it replaces, in /root/reference/replicat/repository.py:

* ``_stream_files`` (:1413-1452): files sorted by (size, path), read in 16 MiB pieces, zero
  padding to 4 bytes between files, and a ``blake2b`` incremental hasher per file (:1433-1446);
* ``_chunk_producer`` (:1454-1505): ``chunkify`` over that ONE stream, ``hash_digest`` of every
  chunk (:1462), the digest -> table-index dedup map (:1464-1468), for an encrypted repository
  ``encrypt(chunk, derive_shared_subkey(digest))`` (:1470-1473), the chunk counter and stream
  offsets (:1457-1459, :1477-1485);
* ``_chunk_done``'s file -> chunk-range map (:1374-1411).

The stream is gathered into host batches (``batch_bytes``, pinned) exactly as the batching shim
does (replicat_amd/adapters.py): every batch but the last is chunked as an OPEN prefix (the
reference's non-final ``next_cut`` calls), the last with its real framing, and the uncut tail
is carried into the next batch.  ``slots`` batches (default 3) are in flight, each on its own
HIP stream with its own digest / cipher handles: the files are read straight into one pinned
batch (``readinto``) while the device works on the others, so the BLAKE2b floor of one batch
(its longest chunk's chain, ~55 ms for a 5.12 MB chunk) overlaps the next
batches' uploads, cuts and digests instead of serialising the pipeline.  Each batch is uploaded ONCE and everything runs on the bytes in HBM: the cut chain (rc_chunk_device), the chunk digests (rc_blake2b_chunks), the per-file
incremental digests of small files (rc_blake2b_update_device: each file's bytes are fed once, in
the batch that first holds them; a file's state lives in HBM across batches) and, with ``encryption``, every
chunk's subkey (rc_blake2b_derive_chunks) and its AES-GCM encryption (rc_gcm_encrypt_chunks).
Only cut offsets, digests and -- what replicat uploads -- the chunk contents come back: sliced
from the host batch, or the device's nonce || C || T when encrypted.

Memory held per producer: ``slots`` x (one pinned host batch + its HBM copy) of ``capacity`` =
batch_bytes + max_length + 16 MiB + 128 bytes each (~1.02 GiB at the default 1 GiB batch, so ~2.1
GiB pinned and ~3.1 GiB HBM with the default 3 slots, ~2.1 with 2); with ``encryption`` each slot
also holds a pinned and an HBM ciphertext buffer of the same size plus 28 bytes per chunk (~6.1
GiB pinned in all with 3 slots).  Smaller ``batch_bytes`` or ``slots`` shrink it linearly.
Round 5 made 3 slots the default again: with large files the producer is bound by the host's
per-file BLAKE2b chains and page-cache copies, and with 2 slots a slot's round trip (fill, then
~75 ms of upload + chunk digests on the device) set the pace instead -- 8 GiB in 128 files,
15.4 GiB/s with 2 slots, 16.9 with 3, against 18.8 GiB/s for the files' digests alone on the
same 16 host threads (profiles/r05/producer/).

Two ways to consume the chunks:

* ``run(paths)`` returns the whole ``SnapshotStream``; every ``ChunkRecord.contents`` is a copy
  (bytes) made on the collector thread -- the host copies were ~0.46 s of an 8 GiB snapshot
  (DESIGN.md §5c);
* ``stream(paths)`` yields the ``ChunkRecord``s batch by batch as replicat's upload queue takes
  ``_SnapshotChunk``s (repository.py:1492, :1507-1554), with ``contents`` a read-only
  memoryview INTO the pinned batch (or the pinned ciphertexts): no copy.  The consumer calls
  ``record.release()`` when it is done with the contents (an upload worker, after its upload); a
  batch's pinned buffer is refilled only once every record of it has been released (or
  garbage-collected), so a view never changes under its reader.

The dedup table and the chunk -> file range map are host bookkeeping on a few integers per
chunk, as in the reference.  Per-file digests of files of 1 MiB and more are hashed on host
threads from the pinned batch, piece by piece as the pieces are read, while the device works
(``file_digests='auto'``): a file digest is
one sequential chain, which a host core advances ~10x faster than one device chain (measured,
DESIGN.md §5c); ``file_digests='device'`` keeps every file on the device.  There is no CPU
fallback: every cut, chunk digest, subkey and ciphertext comes from the HIP library, and a
missing library raises.
"""
import collections
import io
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from .chunker import (MAX_LENGTH, MIN_LENGTH, GpuChunker, QueueStream, _current_device,
                      check_counts, normalize_params)
from .hashing import SLOT, GpuBlake2b, state_init
from .snapshot import PIECE, PieceReader, file_parts, sort_files

# The device time of a batch has a floor: the BLAKE2b chain of its longest chunk (~55 ms for a
# 5.12 MB chunk), whatever the batch size; 1 GiB batches amortize it (256 MiB ones
# spent ~58 ms per batch on the device, measured).
DEFAULT_BATCH = 1 << 30


@dataclass
class FileRecord:
    """repository.py:1427-1432 (_SnapshotFile) plus the digest of :1445."""
    path: str
    stream_start: int
    stream_end: int
    digest: Optional[bytes] = None
    size: Optional[int] = None   # at open time (fstat of the opened file), when it tells


class _Lease:
    """Records of one batch whose contents still view its pinned buffer (stream())."""

    def __init__(self):
        self.n = 0
        self.cv = threading.Condition()

    def take(self, k):
        with self.cv:
            self.n += k

    def drop(self):
        with self.cv:
            self.n -= 1
            if self.n == 0:
                self.cv.notify_all()

    def wait(self, abort, timeout=None, warn_after=60.0):
        """Until every record is released; False if `abort` (an Event) was set first,
        TimeoutError after `timeout` seconds.  A consumer that keeps records without releasing
        them stalls the producer: say so once."""
        t0, warned = time.monotonic(), False
        with self.cv:
            while self.n:
                if abort.is_set():
                    return False
                self.cv.wait(0.05)
                if timeout is not None and time.monotonic() - t0 > timeout:
                    raise TimeoutError(f'{self.n} ChunkRecord(s) of a batch unreleased for '
                                       f'{timeout} s: release() each record when done with it')
                if not warned and time.monotonic() - t0 > warn_after:
                    warned = True
                    import warnings
                    warnings.warn(f'DeviceSnapshotProducer.stream: {self.n} ChunkRecord(s) of a '
                                  'batch still unreleased; the producer waits to refill its '
                                  'buffer (release() each record when done with it)',
                                  RuntimeWarning, stacklevel=2)
        return True


@dataclass
class ChunkRecord:
    """repository.py:1477-1485 (_SnapshotChunk) without the upload location.  ``contents`` is
    what replicat uploads: the chunk bytes, or nonce || C || T for an encrypted repository --
    bytes from run(), a read-only memoryview into the producer's pinned batch from stream()
    (valid until release())."""
    counter: int
    stream_start: int
    stream_end: int
    digest: bytes
    table_index: int
    contents: Optional[object] = field(default=None, repr=False)
    _lease: Optional[_Lease] = field(default=None, repr=False, compare=False)

    def release(self):
        """Done with ``contents`` (a stream() record): its batch buffer may be refilled.
        Idempotent; a record dropped without it releases when it is garbage-collected."""
        lease, self._lease = self._lease, None
        if lease is not None:
            self.contents = None
            lease.drop()

    def __del__(self):
        try:
            self.release()
        except Exception:  # interpreter shutdown
            pass


@dataclass
class ChunkEncryption:
    """What an encrypted repository's snapshot loop needs to encrypt chunks
    (repository.py:1470-1473): KeyProps.params['shared_key'] and ['shared_kdf_params']
    (repository.py:132-137) and the cipher's aes_gcm settings (adapters.py:151-158).  The shared
    KDF is blake2b(length=key_bits // 8) (repository.py:623-627)."""
    shared_key: bytes
    shared_kdf_params: bytes
    key_bits: int = 256
    nonce_bits: int = 96


@dataclass
class SnapshotStream:
    files: List[FileRecord]
    chunks: List[ChunkRecord]
    chunks_table: Dict[bytes, int]

    def snapshot_files(self):
        """The ``snapshot_files`` dict _chunk_done builds (repository.py:1374-1411): per file,
        its chunk parts ({'range', 'index', 'counter'}) and digest (metadata not collected)."""
        out = {}
        for ci, fi, part in file_parts(self.files, self.chunks):
            f, c = self.files[fi], self.chunks[ci]
            d = out.setdefault(f.path, {'path': f.path, 'chunks': [], 'digest': None})
            d['chunks'].append({'range': part, 'index': c.table_index, 'counter': c.counter})
            if c.stream_end >= f.stream_end:
                d['digest'] = f.digest
        return out


def _fstat_size(record, src):
    try:
        record.size = os.fstat(src.fileno()).st_size
    except (AttributeError, OSError, ValueError, io.UnsupportedOperation):
        record.size = None  # a read hook without a file descriptor


class _Pending:
    """Host digest pieces still to be hashed from one slot's bytes."""

    def __init__(self):
        self.n, self.err = 0, None
        self.cv = threading.Condition()

    def add(self):
        with self.cv:
            self.n += 1

    def done(self, err=None):
        with self.cv:
            self.n -= 1
            self.err = self.err or err
            self.cv.notify_all()

    def wait(self):
        with self.cv:
            while self.n:
                self.cv.wait()
            if self.err is not None:
                raise self.err


class _HostHash:
    """A file digest on host threads: its pieces are hashed in order by one drain job at a time
    (hashlib releases the GIL while it hashes), so files proceed in parallel and no pool thread
    ever waits for another file's piece."""

    def __init__(self, h):
        self.h = h
        self.q = collections.deque()
        self.busy = False
        self.lock = threading.Lock()

    def push(self, view, pending, pool):
        pending.add()
        with self.lock:
            self.q.append((view, pending))
            if self.busy:
                return
            self.busy = True
        pool.submit(self._drain)

    def _drain(self):
        while True:
            with self.lock:
                if not self.q:
                    self.busy = False
                    return
                view, pending = self.q.popleft()
            try:
                self.h.update(view)
            except BaseException as e:  # reported by the slot's wait
                pending.done(e)
            else:
                pending.done()


def fill_batch(reader, look_buf, look, buf, head, batch_bytes, on_piece):
    """Fill one batch at buf[head:] (a uint8 array): the piece read ahead (`look`, in
    look_buf), then whole pieces straight from the files (PieceReader) while fewer than
    batch_bytes new bytes are in place, then the next piece into look_buf: it tells whether the
    batch is final and which files it closes.  on_piece(file index or None, offset, length)
    follows every piece placed.  Returns (the next look, new bytes, offset of the last piece)."""
    n = last_rel = 0
    mv = memoryview(buf)
    while look is not None and (n < batch_bytes or n == 0):
        ln, _, fi = look
        at = head + n
        buf[at:at + ln] = np.frombuffer(look_buf, dtype=np.uint8, count=ln)
        on_piece(fi, at, ln)
        last_rel, n = n, n + ln
        # further pieces straight into the batch; the one after a full batch into look_buf
        while n < batch_bytes:
            got = reader.read_into(mv[head + n:])
            if got is None:
                look = None
                break
            ln, _, fi = got
            on_piece(fi, head + n, ln)
            last_rel, n = n, n + ln
        else:
            look = reader.read_into(look_buf)
            continue
        break
    return look, n, last_rel


class _Slot:
    """One batch in flight: its pinned host bytes, their device copy, the cut / digest outputs
    and the HIP stream its work is queued on.  The batch's bytes sit at host[off:off + blen]:
    the previous batch's uncut tail in the head room before `head`, the new pieces from `head`."""

    def __init__(self, prod, torch):
        dev = prod.dev
        # per-slot native handles: a handle's staging workspaces are reused every other call, so
        # a shared one would make the host wait for batch k's digests before queuing batch k + 2's
        self.hasher = GpuBlake2b(length=prod.digest_size, device=prod.device)
        self.file_hasher = GpuBlake2b(length=prod.digest_size, device=prod.device)
        self.host = torch.empty(prod.capacity, dtype=torch.uint8, pin_memory=True)
        self.hnp = self.host.numpy()
        self.dbuf = torch.empty(prod.capacity, dtype=torch.uint8, device=dev)
        self.d_cuts = torch.zeros(max(prod.cut_cap, 1), dtype=torch.int64, device=dev)
        self.d_count = torch.zeros(1, dtype=torch.int64, device=dev)
        self.d_digests = torch.zeros((max(prod.cut_cap, 1), SLOT), dtype=torch.uint8, device=dev)
        self.h_meta = torch.zeros(2, dtype=torch.int64, pin_memory=True)  # count, last cut end
        # queues='own': a HIP stream with a hardware queue of its own (rc_stream_create), so this
        # batch's ~55 ms digest chain never holds up the next batch's kernels on a shared queue
        # (HIP's default GPU_MAX_HW_QUEUES=4 put a third slot stream behind the first, DESIGN.md
        # §3b); 'shared': a torch stream on the process's shared queues
        self.qs = QueueStream.acquire(prod.device) if prod.queues == 'own' else None
        self.stream = self.qs.torch if self.qs is not None else torch.cuda.Stream(device=dev)
        # timing events when the producer records a per-batch timeline (prod.timeline)
        tm = bool(getattr(prod, 'timeline', False))
        self.ev_start, self.ev_up, self.ev_cut, self.ev_upd, self.ev_done = (
            torch.cuda.Event(enable_timing=tm) for _ in range(5))
        self.t_enqueue = 0.0
        if prod.encryption is not None:
            nb, total = prod.cipher.nonce_bytes, max(prod.cut_cap, 1)
            self.d_keys = torch.zeros((total, SLOT), dtype=torch.uint8, device=dev)
            self.h_nonces = torch.empty(total * nb, dtype=torch.uint8, pin_memory=True)
            self.d_nonces = torch.empty(total * nb, dtype=torch.uint8, device=dev)
            self.d_enc = torch.empty(max(prod.enc_cap, 1), dtype=torch.uint8, device=dev)
            self.h_enc = torch.empty(max(prod.enc_cap, 1), dtype=torch.uint8, pin_memory=True)
            from .cipher import GpuAesGcm
            self.kdf_hasher = GpuBlake2b(length=prod.digest_size, device=prod.device)
            self.cipher = GpuAesGcm(key_bits=prod.encryption.key_bits,
                                    nonce_bits=prod.encryption.nonce_bits, device=prod.device)
        self.lease = _Lease()  # stream(): records still viewing host / h_enc
        self.reset(prod.head)

    def close(self):
        for h in ('hasher', 'file_hasher', 'kdf_hasher', 'cipher'):
            obj = getattr(self, h, None)
            if obj is not None and hasattr(obj, 'close'):
                obj.close()
        qs, self.qs = getattr(self, 'qs', None), None
        if qs is not None:
            self.stream.synchronize()
            qs.release()  # pooled, never destroyed: torch may still record events on it

    def reset(self, head):
        self.off = head          # host offset of the batch's first byte
        self.blen = 0            # bytes in the batch (carried tail + new pieces)
        self.buf_start = 0       # stream offset of the batch's first byte
        self.final = False
        self.closed = 0          # files [0, closed) are complete within this batch
        self.host_jobs = _Pending()  # host digest pieces reading this slot's bytes
        self.items = []          # device file-digest items: (file index, final)
        self.file_digests = None


class DeviceSnapshotProducer:
    """Chunks, chunk digests, file digests and (optionally) encrypted chunks of a snapshot's
    stream on one HIP device."""

    def __init__(self, *, min_length: int = MIN_LENGTH, max_length: int = MAX_LENGTH,
                 params: Optional[bytes] = None, digest_size: int = 64,
                 batch_bytes: int = DEFAULT_BATCH, device=None, keep_contents: bool = True,
                 encryption: Optional[ChunkEncryption] = None, file_digests: str = 'auto',
                 slots: int = 3, queues: str = 'own', read_threads: int = 4,
                 timeline: bool = False):
        import torch
        if device is None:
            device = _current_device()
        if min_length > max_length:
            raise ValueError(f'Minimum length ({min_length}) is greater '
                             f'than the maximum one ({max_length})')
        if int(slots) < 2:
            raise ValueError('slots must be at least 2 (one batch filled while one is on the device)')
        if queues not in ('own', 'shared'):
            raise ValueError(f'queues must be own or shared, not {queues!r}')
        self.queues = queues
        if int(read_threads) < 1:
            raise ValueError('read_threads must be at least 1')
        # a piece of a regular file is read as up to read_threads parallel positional reads
        # (snapshot.PieceReader): the page-cache copy, not the device, bounds the producer
        self.read_threads = int(read_threads)
        # timeline: per-batch device phases in self.profile['timeline'] (HIP timing events on
        # the slot streams; a measurement switch)
        self.timeline = bool(timeline)
        self.device = int(device)
        self.dev = torch.device('cuda', self.device)
        self.chunker = GpuChunker(min_length, max_length, normalize_params(params), device=self.device)
        self.min_length, self.max_length = min_length, max_length
        self.digest_size = digest_size
        self.batch_bytes = max(int(batch_bytes), 2 * max_length + 16)
        self.keep_contents = keep_contents
        if file_digests not in ('auto', 'device', 'host'):
            raise ValueError(f'file_digests must be auto, device or host, not {file_digests!r}')
        self.file_digests = file_digests
        self._pool = None
        # head room for the carried tail (an OPEN batch leaves < max_length bytes uncut), one
        # batch of new pieces, one piece of overshoot
        self.head = (max_length + 127) // 64 * 64
        self.capacity = self.head + self.batch_bytes + PIECE + 64
        self.cut_cap, _ = self.chunker.capacity([self.capacity])
        self._init_state = np.frombuffer(state_init(digest_size), dtype=np.uint8)
        self.encryption = encryption
        if encryption is not None:
            from .cipher import GpuAesGcm
            # the layout of the ciphertexts (nonce || C || T per chunk); each slot encrypts with
            # its own handle
            self.cipher = GpuAesGcm(key_bits=encryption.key_bits, nonce_bits=encryption.nonce_bits,
                                    device=self.device)
            kdf = state_init(self.cipher.key_bytes, key=encryption.shared_key,
                             salt=encryption.shared_kdf_params)
            self.d_kdf = torch.from_numpy(np.frombuffer(kdf, dtype=np.uint8).copy()).to(self.dev)
            self.enc_cap, _ = self.cipher.chunks_layout(self.chunker, [self.capacity])
        # `slots` batches in flight: the host fills one while the device works on the others
        self._slots = [_Slot(self, torch) for _ in range(int(slots))]
        self._busy = threading.Lock()  # held by the one _produce at a time
        self._look = bytearray(PIECE)  # the piece after a full batch (tells whether it is final)

    # ------------------------------------------------------------------- file digests

    # A file digest is ONE sequential BLAKE2b chain over the whole file.  On the device a chain
    # advances one 128-byte block per ~1.4 us (the dependent-instruction latency of a quad of
    # lanes); a host core does ~1 GB/s.  Many small files hash in parallel on the
    # device within a batch, but a large file's chain would set the batch time (a 256 MiB file:
    # 2.9 s on the device, 0.27 s on a host core), so 'auto' hashes files of at least
    # HOST_DIGEST_MIN bytes on host threads, piece by piece as they are read, overlapped with
    # the reads and the device work; 'device' and 'host' force one engine.
    HOST_DIGEST_MIN = 1 << 20

    def _on_host(self, fi, f, hstates, engine):
        """Whether file fi's digest runs on a host thread; decided once per file (its bytes must
        all go to one engine): in 'auto' by the size fstat gave when the file was opened, or,
        for a read hook with no file descriptor, by the bytes read when it is first seen."""
        if fi not in engine:
            if self.file_digests == 'auto':
                size = f.size if f.size is not None else f.stream_end - f.stream_start
                engine[fi] = size >= self.HOST_DIGEST_MIN
            else:
                engine[fi] = self.file_digests == 'host'
            if engine[fi]:
                import hashlib
                hstates[fi] = _HostHash(hashlib.blake2b(digest_size=self.digest_size))
        return engine[fi]

    def close(self):
        """Release the pinned batches, their device copies and the host threads (the object is
        unusable afterwards; also on leaving a `with` block)."""
        for pool in (self._pool, getattr(self, '_collect_pool', None)):
            if pool is not None:
                pool.shutdown(wait=True)
        self._pool = self._collect_pool = None
        for sl in self._slots:
            sl.close()
        self._slots = []
        for h in ('chunker', 'cipher'):
            obj = getattr(self, h, None)
            if obj is not None and hasattr(obj, 'close'):
                obj.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def _collector(self):
        if getattr(self, '_collect_pool', None) is None:
            from concurrent.futures import ThreadPoolExecutor
            self._collect_pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix='rc-collect')
        return self._collect_pool

    def _host_pool(self):
        if self._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=max(1, min(16, os.cpu_count() or 1)),
                                            thread_name_prefix='rc-file-digest')
        return self._pool

    # ------------------------------------------------------------------------------ run

    def run(self, paths: Sequence[os.PathLike], read=None) -> SnapshotStream:
        """The whole snapshot stream, every chunk's contents copied out (bytes)."""
        files: List[FileRecord] = []
        run = self._produce(paths, read, files, zero_copy=False, sink=None,
                            abort=threading.Event())
        return SnapshotStream(files=files, chunks=run.chunks, chunks_table=run.table)

    def stream(self, paths: Sequence[os.PathLike], read=None,
               stall_timeout: Optional[float] = None) -> 'ChunkStream':
        """The chunks as they are produced (a ``ChunkStream``: iterate it for ``ChunkRecord``s
        whose ``contents`` view the pinned batches -- release() each when done), produced on a
        thread of its own like replicat's chunk-producer thread (repository.py:1358,1556).
        The records must be released by someone other than the loop that waits for the next
        one (upload workers, as replicat's _worker coroutines), or right away: a loop that
        holds more records than the other slots can carry waits for itself.  stall_timeout:
        seconds the producer waits for a batch's records before it fails the stream with a
        TimeoutError (None: it waits, and warns after a minute)."""
        return ChunkStream(self, paths, read, stall_timeout)

    def _produce(self, paths, read, files, zero_copy, sink, abort, stall_timeout=None):
        """Batch k + 1 is read from the files while the device cuts and digests batch k, and
        batch k's records are built while the device works on batch k + 1.  The uncut tail of
        batch k (known once its cut chain is done, long before its digests) is copied to the
        head of batch k + 1 on the host, so every batch is uploaded once.  zero_copy: records
        view the slot (sink(records) gets every batch's; the slot is refilled once all are
        released)."""
        import torch
        if not self._slots:
            raise RuntimeError('DeviceSnapshotProducer is closed')
        # one run at a time: two would fill the same slots (an abandoned stream() whose producer
        # thread still runs -- close() it, or let its iterator go -- fails the next run here)
        if not self._busy.acquire(blocking=False):
            raise RuntimeError('DeviceSnapshotProducer: another run() or stream() is still '
                               'producing on this producer (close() the ChunkStream first)')
        try:
            return self._produce_locked(torch, paths, read, files, zero_copy, sink, abort,
                                        stall_timeout)
        finally:
            self._busy.release()

    def _produce_locked(self, torch, paths, read, files, zero_copy, sink, abort, stall_timeout):
        run = _Run(self, torch, files, zero_copy, sink)
        reader = PieceReader(sort_files(paths), files, read, record=FileRecord, on_open=_fstat_size,
                             threads=self.read_threads)
        # fill / wait_cut / enqueue / collect_join: this thread; collect_wait / records /
        # host_digest_wait: the collector thread (overlapping the next fill)
        prof = self.profile = {'fill': 0.0, 'wait_cut': 0.0, 'enqueue': 0.0, 'collect_join': 0.0,
                               'collect_wait': 0.0, 'records': 0.0, 'host_digest_wait': 0.0,
                               'release_wait': 0.0, 'batches': 0, 't0': time.perf_counter()}
        clock = time.perf_counter
        prev, look, k = None, None, 0
        # records are built on a collector thread (they copy chunk contents, holding the GIL)
        # while this thread reads the next batch (the reads release it)
        ns = len(self._slots)
        collected = [None] * ns  # per slot: the collection of its last batch
        collector = self._collector()
        try:
            look = reader.read_into(self._look)
            while True:
                s = self._slots[k % ns]
                if collected[k % ns] is not None:  # the slot's previous batch is fully consumed
                    t = clock()
                    collected[k % ns].result()
                    collected[k % ns] = None
                    prof['collect_join'] += clock() - t
                # and every stream() record viewing its bytes released (also across runs)
                t = clock()
                if not s.lease.wait(abort, stall_timeout):
                    raise _Aborted()
                prof['release_wait'] += clock() - t
                s.reset(self.head)
                # ---- fill: the piece read ahead, then whole pieces up to batch_bytes of new bytes
                t0 = clock()
                look, n, last_rel = fill_batch(reader, self._look, look, s.hnp, self.head,
                                               self.batch_bytes,
                                               lambda fi, at, ln: run.host_piece(s, fi, at, ln))
                s.final = look is None
                s.closed = len(files) if s.final else look[1]
                new_lo = reader.pos - n - (look[0] if look is not None else 0)
                t1 = clock()
                prof['fill'] += t1 - t0
                # ---- the previous batch's uncut tail to the head of this one
                T, buf_start = 0, new_lo
                if prev is not None:
                    prev.ev_cut.synchronize()
                    cnt, cut_end = int(prev.h_meta[0]), int(prev.h_meta[1])
                    check_counts([cnt])  # overflow, or the tile kernel's fail-safe stop
                    cut_end = cut_end if cnt else 0
                    T = prev.blen - cut_end
                    if T > self.head:
                        raise RuntimeError(f'uncut tail of {T} bytes exceeds the head room')
                    s.hnp[self.head - T:self.head] = prev.hnp[prev.off + cut_end:prev.off + prev.blen]
                    buf_start = prev.buf_start + cut_end
                t2 = clock()
                prof['wait_cut'] += t2 - t1
                s.off, s.blen, s.buf_start = self.head - T, T + n, buf_start
                run.enqueue(s, prev, T, T + last_rel, new_lo, new_lo + n)
                prof['batches'] += 1
                prof['enqueue'] += clock() - t2
                if prev is not None:
                    collected[(k - 1) % ns] = collector.submit(run.collect, prev)
                if s.final:
                    collected[k % ns] = collector.submit(run.collect, s)
                    for f in collected:
                        if f is not None:
                            f.result()
                    break
                prev = s
                k += 1
        finally:
            reader.close()
            for f in collected:
                if f is not None:
                    try:
                        f.result()
                    except BaseException:
                        pass
            for sl in self._slots:  # nothing of this run may still be queued or hashing
                sl.stream.synchronize()
                try:
                    sl.host_jobs.wait()
                except BaseException:
                    pass
        return run


class _Run:
    """The bookkeeping of one DeviceSnapshotProducer.run: per-file digest states and engines,
    the dedup table, the chunk records."""

    def __init__(self, prod, torch, files, zero_copy=False, sink=None):
        self.p, self.torch, self.files = prod, torch, files
        self.zero_copy, self.sink = zero_copy, sink
        self.chunks: List[ChunkRecord] = []  # zero_copy: records without contents
        self.table: Dict[bytes, int] = {}
        self.states = {}     # file index -> device state (open device-engine files)
        self.hstates = {}    # file index -> _HostHash (host-engine files)
        self.engine = {}     # file index -> its digest runs on the host (decided once)
        self.finalized = 0   # files [0, finalized) have their digest

    def host_piece(self, s, fi, at, n):
        """A file piece just placed at s.hnp[at:at + n]: hashed now on a host thread if the
        file's digest is a host one."""
        if fi is None or not self.p._on_host(fi, self.files[fi], self.hstates, self.engine):
            return
        self.hstates[fi].push(memoryview(s.hnp)[at:at + n], s.host_jobs, self.p._host_pool())

    def enqueue(self, s, prev, T, last_start, new_lo, new_hi):
        """Upload batch s and queue, on s.stream: its cuts, the device file digests of its new
        bytes, its chunk digests, and subkeys + ciphertexts.  The file digests go before the
        chunk digests: the next batch's file digests wait for them (a file's state advances
        batch after batch), and must not wait behind this batch's ~55 ms digest floor."""
        torch, p = self.torch, self.p
        hs = s.stream.cuda_stream
        ptr = s.dbuf.data_ptr()
        timeline = p.timeline
        s.t_enqueue = time.perf_counter()
        with torch.cuda.stream(s.stream):
            if timeline:
                s.ev_start.record(s.stream)
            if s.blen:
                s.dbuf[:s.blen].copy_(s.host[s.off:s.off + s.blen], non_blocking=True)
            if timeline:
                s.ev_up.record(s.stream)
            p.chunker.chunk_device([ptr], [s.blen], [last_start], s.d_cuts.data_ptr(),
                                   s.d_count.data_ptr(), hs, open_=not s.final)
            # count and last cut end to pinned memory: the next batch's head needs them
            s.h_meta[0:1].copy_(s.d_count, non_blocking=True)
            last = torch.index_select(s.d_cuts, 0, (s.d_count - 1).clamp_(min=0))
            s.h_meta[1:2].copy_(last, non_blocking=True)
            s.ev_cut.record(s.stream)
            # device file digests over the new bytes [T, blen): a file's state in HBM is
            # advanced batch after batch, so this stream first waits for the previous batch's
            # (files below prev.closed were closed by earlier batches, collected or not)
            items = []
            for fi in range(max(self.finalized, prev.closed if prev is not None else 0),
                            len(self.files)):
                f = self.files[fi]
                a, b = max(f.stream_start, new_lo), min(f.stream_end, new_hi)
                n = b - a if b > a else 0
                is_final = fi < s.closed
                if n == 0 and not is_final:
                    continue
                if p._on_host(fi, f, self.hstates, self.engine):
                    continue
                items.append((fi, ptr + T + (a - new_lo) if n else 0, n, is_final))
            if items:
                if prev is not None:
                    s.stream.wait_event(prev.ev_upd)
                for fi, _, _, _ in items:
                    if fi not in self.states:
                        self.states[fi] = torch.from_numpy(p._init_state.copy()).to(p.dev)
                    else:
                        self.states[fi].record_stream(s.stream)
                scratch = torch.zeros((len(items), SLOT), dtype=torch.uint8, device=p.dev)
                s.file_hasher.update_device([self.states[fi].data_ptr() for fi, _, _, _ in items],
                                            [q for _, q, _, _ in items],
                                            [n for _, _, n, _ in items],
                                            [1 if fin else 0 for _, _, _, fin in items],
                                            scratch.data_ptr(), hs)
                s.file_digests = scratch
                s.items = [(fi, fin) for fi, _, _, fin in items]
            elif prev is not None:
                s.stream.wait_event(prev.ev_upd)  # keep the file-state order transitive
            s.ev_upd.record(s.stream)
            s.hasher.digest_chunks(p.chunker, [ptr], [s.blen], s.d_cuts.data_ptr(),
                                   s.d_count.data_ptr(), s.d_digests.data_ptr(), hs)
            if p.encryption is not None:
                # derive_shared_subkey(digest) and encrypt, per chunk, still in HBM; one
                # os.urandom nonce per chunk as the adapter draws them (adapters.py:133)
                s.kdf_hasher.derive_chunks(p.chunker, [s.blen], s.d_count.data_ptr(),
                                           p.d_kdf.data_ptr(), s.d_digests.data_ptr(),
                                           s.d_keys.data_ptr(), hs)
                s.h_nonces.numpy()[:] = np.frombuffer(os.urandom(s.h_nonces.numel()),
                                                      dtype=np.uint8)
                s.d_nonces.copy_(s.h_nonces, non_blocking=True)
                s.cipher.encrypt_chunks(p.chunker, [ptr], [s.blen], s.d_cuts.data_ptr(),
                                        s.d_count.data_ptr(), s.d_keys.data_ptr(),
                                        s.d_nonces.data_ptr(), s.d_enc.data_ptr(), hs)
            s.ev_done.record(s.stream)

    def collect(self, s):
        """Wait for batch s and turn it into records: cut ends, digests, dedup indices, contents
        (sliced from the host batch, or the device's nonce || C || T), finished file digests."""
        torch, p, prof, clock = self.torch, self.p, self.p.profile, time.perf_counter
        t0 = clock()
        s.ev_done.synchronize()
        count = int(s.h_meta[0])
        check_counts([count])
        # every device read on the slot's own stream: the legacy NULL stream would wait for
        # every blocking (own-queue) slot stream, i.e. for the later batches' digests too
        with torch.cuda.stream(s.stream):
            ends = s.d_cuts[:count].cpu().numpy().view(np.uint64).astype(np.int64)
            digs = s.d_digests[:count, :p.digest_size].cpu().numpy()
            fd = (s.file_digests[:, :p.digest_size].cpu().numpy()
                  if s.file_digests is not None else None)
        enc = over = None
        if p.encryption is not None:
            over = p.cipher.nonce_bytes + 16
            n_out = (int(ends[-1]) if count else 0) + count * over
            with torch.cuda.stream(s.stream):
                s.h_enc[:n_out].copy_(s.d_enc[:n_out], non_blocking=True)
            s.stream.synchronize()
            enc = s.h_enc[:n_out].numpy()
        if fd is not None:
            for j, (fi, fin) in enumerate(s.items):
                if fin:
                    self.files[fi].digest = fd[j].tobytes()
                    del self.states[fi]
        t1 = clock()
        prof['collect_wait'] += t1 - t0
        if p.timeline:
            # one batch's device phases (HIP events on its stream) and its host latency
            ms = lambda a, b: round(a.elapsed_time(b), 3)  # noqa: E731
            prof.setdefault('timeline', []).append({
                'bytes': s.blen, 'upload_ms': ms(s.ev_start, s.ev_up),
                'chunk_ms': ms(s.ev_up, s.ev_cut), 'file_digest_ms': ms(s.ev_cut, s.ev_upd),
                'digest_ms': ms(s.ev_upd, s.ev_done), 'device_ms': ms(s.ev_start, s.ev_done),
                'enqueue_to_done_ms': round((t1 - s.t_enqueue) * 1e3, 3),
                'start_at_ms': round((s.t_enqueue - prof['t0']) * 1e3, 3),
                'collected_at_ms': round((t1 - prof['t0']) * 1e3, 3)})
        chunks, table, hnp = self.chunks, self.table, s.hnp
        zc = self.zero_copy and p.keep_contents
        # zero copy: read-only views into the pinned batch (or ciphertexts), leased per batch
        view = memoryview(enc if enc is not None else hnp).toreadonly() if zc else None
        out = [] if self.sink is not None else None
        prev = 0
        for k, e in enumerate(ends.tolist()):
            d = digs[k].tobytes()
            idx = table.get(d)
            if idx is None:
                idx = table[d] = len(table)
            if enc is not None:  # nonce || C || T of chunk k at prev + k (nonce_bytes + 16)
                o = prev + k * over
                contents = view[o:o + (e - prev) + over] if zc else enc[o:o + (e - prev) + over].tobytes()
            elif not p.keep_contents:
                contents = None
            else:
                contents = view[s.off + prev:s.off + e] if zc else hnp[s.off + prev:s.off + e].tobytes()
            rec = ChunkRecord(counter=len(chunks) + 1, stream_start=s.buf_start + prev,
                              stream_end=s.buf_start + e, digest=d, table_index=idx,
                              contents=None if zc else contents)
            chunks.append(rec)
            if out is not None:
                if zc:  # the consumer's copy of the record carries the view and the lease
                    rec = ChunkRecord(rec.counter, rec.stream_start, rec.stream_end, d, idx,
                                      contents, s.lease)
                out.append(rec)
            prev = e
        if out is not None:
            if zc:
                s.lease.take(len(out))
            self.sink(out)
        t2 = clock()
        prof['records'] += t2 - t1
        s.host_jobs.wait()  # every host piece of this slot, before it is refilled
        for fi in range(self.finalized, s.closed):
            if self.engine.get(fi) and self.files[fi].digest is None:
                self.files[fi].digest = self.hstates.pop(fi).h.digest()
        prof['host_digest_wait'] += clock() - t2
        while self.finalized < s.closed and self.files[self.finalized].digest is not None:
            self.finalized += 1
        if s.final and prev != s.blen:
            raise RuntimeError(f'final batch left {s.blen - prev} bytes uncut')


class _Aborted(Exception):
    """The consumer of a ChunkStream went away: the producer thread stops."""


class ChunkStream:
    """The chunks of one snapshot, produced on a thread of its own (DeviceSnapshotProducer
    .stream): iterate it for ``ChunkRecord``s in stream order; ``contents`` views the producer's
    pinned batch until ``release()``.  Once exhausted, ``files`` and ``chunks_table`` are the
    run's (``snapshot()`` gives the ``SnapshotStream``, records without contents).  ``close()``
    stops the producer; so does leaving a ``with`` block, abandoning the iteration (``break``:
    the iterator's ``finally``) or dropping the stream (the producer thread holds only the queue,
    the abort event and a result box, never the stream).  Records the consumer still holds keep
    their batch's buffer until released (the next run waits for them)."""

    _END = object()

    def __init__(self, prod, paths, read=None, stall_timeout=None):
        import queue
        self.files: List[FileRecord] = []
        self._q = q = queue.Queue()
        self._abort = abort = threading.Event()
        self._box = box = {}  # 'run': the finished _Run
        self._done = False
        files, end = self.files, self._END

        def work():
            try:
                box['run'] = prod._produce(paths, read, files, zero_copy=True, sink=q.put,
                                           abort=abort, stall_timeout=stall_timeout)
                q.put(end)
            except _Aborted:
                q.put(end)
            except BaseException as e:  # re-raised in the consumer
                q.put(e)

        self._thread = threading.Thread(target=work, name='rc-chunk-producer', daemon=True)
        self._thread.start()

    @property
    def _run(self):
        return self._box.get('run')

    def __iter__(self):
        try:
            while not self._done:
                item = self._q.get()
                if item is self._END:
                    self._done = True
                    self._thread.join()
                    return
                if isinstance(item, BaseException):
                    self._done = True
                    self._thread.join()
                    raise item
                yield from item
                del item
        finally:
            if not self._done:  # abandoned: stop the producer (its queued records are dropped)
                self.close()

    @property
    def chunks_table(self):
        return self._run.table if self._run is not None else {}

    def snapshot(self) -> SnapshotStream:
        if not self._done or self._run is None:
            raise RuntimeError('ChunkStream not exhausted')
        return SnapshotStream(files=self.files, chunks=self._run.chunks,
                              chunks_table=self._run.table)

    def close(self):
        if threading.current_thread() is self._thread:
            # finalised on the producer thread itself (a cyclic GC pass may run there): it cannot
            # wait for itself -- ask it to stop and release what is queued; it ends on its own
            self._abort.set()
            self._drain_queued()
            return
        if self._thread.is_alive():
            self._abort.set()
            while self._thread.is_alive():  # drain (drops unconsumed records, releasing them)
                try:
                    item = self._q.get(timeout=0.05)
                except Exception:
                    continue
                self._drop(item)
            self._thread.join()
        # what the producer queued before it stopped: release those records now (round 5: with
        # 3 slots a whole batch of them could sit here, holding its slot's lease, until this
        # stream was garbage-collected -- and the next run on the producer waited for it)
        self._drain_queued()
        self._done = True

    def _drain_queued(self):
        import queue
        while True:
            try:
                self._drop(self._q.get_nowait())
            except queue.Empty:
                break

    @staticmethod
    def _drop(item):
        if isinstance(item, list):
            for rec in item:
                rec.release()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def snapshot_stream(paths, **kw) -> SnapshotStream:
    """One-shot helper: DeviceSnapshotProducer(**kw).run(paths)."""
    return DeviceSnapshotProducer(**kw).run(paths)


__all__ = ['DeviceSnapshotProducer', 'SnapshotStream', 'ChunkStream', 'FileRecord', 'ChunkRecord',
           'ChunkEncryption', 'snapshot_stream', 'DEFAULT_BATCH']
