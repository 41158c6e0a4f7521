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
is carried into the next batch.  Each batch is uploaded ONCE and everything runs on the bytes in
HBM: the cut chain (rc_chunk_device), the chunk digests (rc_blake2b_chunks), the per-file
incremental digests of small files (rc_blake2b_update_device: each file's bytes are fed once, in
the batch that first holds them; a file's state lives in HBM across batches) and, with ``encryption``, every
chunk's subkey (rc_blake2b_derive_chunks) and its AES-GCM encryption (rc_gcm_encrypt_chunks).
Only cut offsets, digests and -- what replicat uploads -- the chunk contents come back: sliced
from the host batch, or the device's nonce || C || T when encrypted.

The dedup table and the chunk -> file range map are host bookkeeping on a few integers per
chunk, as in the reference.  Per-file digests of files of 1 MiB and more are hashed on host
threads from the pinned batch while the device works (``file_digests='auto'``): a file digest is
one sequential chain, which a host core advances ~10x faster than one device chain (measured,
DESIGN.md §5c); ``file_digests='device'`` keeps every file on the device.  There is no CPU
fallback: every cut, chunk digest, subkey and ciphertext comes from the HIP library, and a
missing library raises.
"""
import bisect
import os
import time
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .chunker import MAX_LENGTH, MIN_LENGTH, GpuChunker, _current_device, normalize_params
from .hashing import SLOT, STATE_BYTES, GpuBlake2b, state_init
from .snapshot import ALIGNMENT, PIECE, sort_files

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


@dataclass
class ChunkRecord:
    """repository.py:1477-1485 (_SnapshotChunk) without the upload location.  ``contents`` is
    what replicat uploads: the chunk bytes, or nonce || C || T for an encrypted repository."""
    counter: int
    stream_start: int
    stream_end: int
    digest: bytes
    table_index: int
    contents: Optional[bytes] = field(default=None, repr=False)


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
        starts = [(f.stream_start, i) for i, f in enumerate(self.files)]
        out = {}
        for c in self.chunks:
            point = bisect.bisect_left(starts, (c.stream_end + 1,))
            for index in range(point - 1, -1, -1):
                f = self.files[starts[index][1]]
                if f.stream_end < c.stream_start:
                    break
                d = out.setdefault(f.path, {'path': f.path, 'chunks': [], 'digest': None})
                d['chunks'].append({'range': [max(f.stream_start - c.stream_start, 0),
                                              min(f.stream_end, c.stream_end) - c.stream_start],
                                    'index': c.table_index, 'counter': c.counter})
                if c.stream_end >= f.stream_end:
                    d['digest'] = f.digest
        return out


def tagged_pieces(paths: Sequence[str], files: List[FileRecord], read=None
                  ) -> Iterator[Tuple[bytes, int]]:
    """repository.py:1413-1447's pieces for already-sorted paths, each with the number of files
    known to be complete when it is yielded (data of file f: f; padding after file f: f + 1).
    `files` receives a FileRecord when a file is opened; stream_end grows as it is read."""
    pos = 0
    prev = None
    for path in paths:
        if prev is not None:
            pad = -(prev.stream_end - prev.stream_start) % ALIGNMENT
            if pad:
                pos += pad
                yield bytes(pad), len(files)
        f = FileRecord(path=str(path), stream_start=pos, stream_end=pos)
        files.append(f)
        prev = f
        with (read(path) if read else open(path, 'rb')) as src:
            try:
                f.size = os.fstat(src.fileno()).st_size
            except (AttributeError, OSError, ValueError):
                f.size = None  # a read hook without a file descriptor
            while piece := src.read(PIECE):
                pos += len(piece)
                f.stream_end += len(piece)
                yield piece, len(files) - 1


class DeviceSnapshotProducer:
    """Chunks, chunk digests, file digests and (optionally) encrypted chunks of a snapshot's
    stream on one HIP device."""

    def __init__(self, *, min_length: int = MIN_LENGTH, max_length: int = MAX_LENGTH,
                 params: Optional[bytes] = None, digest_size: int = 64,
                 batch_bytes: int = DEFAULT_BATCH, device=None, keep_contents: bool = True,
                 encryption: Optional[ChunkEncryption] = None, file_digests: str = 'auto'):
        import torch
        if device is None:
            device = _current_device()
        if min_length > max_length:
            raise ValueError(f'Minimum length ({min_length}) is greater '
                             f'than the maximum one ({max_length})')
        self.device = int(device)
        self.dev = torch.device('cuda', self.device)
        self.chunker = GpuChunker(min_length, max_length, normalize_params(params), device=self.device)
        self.hasher = GpuBlake2b(length=digest_size, device=self.device)
        self.min_length, self.max_length = min_length, max_length
        self.digest_size = digest_size
        self.batch_bytes = max(int(batch_bytes), 2 * max_length + 16)
        self.keep_contents = keep_contents
        if file_digests not in ('auto', 'device', 'host'):
            raise ValueError(f'file_digests must be auto, device or host, not {file_digests!r}')
        self.file_digests = file_digests
        self._pool = None
        # one batch plus the carried tail (< max_length) plus one piece of overshoot
        self.capacity = self.batch_bytes + max_length + PIECE + 64
        self.host = torch.empty(self.capacity, dtype=torch.uint8, pin_memory=True)
        self.dbuf = torch.empty(self.capacity, dtype=torch.uint8, device=self.dev)
        total, caps = self.chunker.capacity([self.capacity])
        self.cut_cap = total
        self.d_cuts = torch.zeros(max(total, 1), dtype=torch.int64, device=self.dev)
        self.d_count = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.d_digests = torch.zeros((max(total, 1), SLOT), dtype=torch.uint8, device=self.dev)
        self._init_state = np.frombuffer(state_init(digest_size), dtype=np.uint8)
        self.encryption = encryption
        if encryption is not None:
            from .cipher import GpuAesGcm
            self.cipher = GpuAesGcm(key_bits=encryption.key_bits, nonce_bits=encryption.nonce_bits,
                                    device=self.device)
            kdf = state_init(self.cipher.key_bytes, key=encryption.shared_key,
                             salt=encryption.shared_kdf_params)
            self.d_kdf = torch.from_numpy(np.frombuffer(kdf, dtype=np.uint8).copy()).to(self.dev)
            self.d_keys = torch.zeros((max(total, 1), SLOT), dtype=torch.uint8, device=self.dev)
            nb = self.cipher.nonce_bytes
            self.h_nonces = torch.empty(max(total, 1) * nb, dtype=torch.uint8, pin_memory=True)
            self.d_nonces = torch.empty(max(total, 1) * nb, dtype=torch.uint8, device=self.dev)
            out_total, _ = self.cipher.chunks_layout(self.chunker, [self.capacity])
            self.d_enc = torch.empty(max(out_total, 1), dtype=torch.uint8, device=self.dev)
            self.h_enc = torch.empty(max(out_total, 1), dtype=torch.uint8, pin_memory=True)

    # ------------------------------------------------------------------- file digests

    # A file digest is ONE sequential BLAKE2b chain over the whole file.  On the device a chain
    # advances one 128-byte block per ~1.4 us (the dependent-instruction latency of a quad of
    # lanes); a host core does ~1 GB/s.  Many small files hash in parallel on the
    # device within a batch, but a large file's chain would set the batch time (a 256 MiB file:
    # 2.9 s on the device, 0.27 s on a host core), so 'auto' hashes files of at least
    # HOST_DIGEST_MIN bytes on host threads from the pinned batch, overlapped with the device
    # work; 'device' and 'host' force one engine.
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
                hstates[fi] = hashlib.blake2b(digest_size=self.digest_size)
        return engine[fi]

    def _host_pool(self):
        if self._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=max(1, min(16, os.cpu_count() or 1)),
                                            thread_name_prefix='rc-file-digest')
        return self._pool

    # ------------------------------------------------------------------------------ run

    def run(self, paths: Sequence[os.PathLike], read=None) -> SnapshotStream:
        import torch
        stream = torch.cuda.current_stream(self.dev)
        hs = stream.cuda_stream
        files: List[FileRecord] = []
        chunks: List[ChunkRecord] = []
        table: Dict[bytes, int] = {}
        states = {}              # file index -> device state (open files only)
        hstates = {}             # file index -> host hasher (open large files only)
        engine = {}              # file index -> its digest runs on the host (decided once)
        finalized = 0            # files [0, finalized) have their digest
        hnp = self.host.numpy()
        buf_start = 0            # stream offset of host[0]
        blen = 0                 # bytes in the batch buffer
        fed = 0                  # host[0:fed] already fed to the file digests
        it = tagged_pieces(sort_files(paths), files, read)
        nxt = next(it, None)
        prof = self.profile = {'fill': 0.0, 'device': 0.0, 'host_digest_wait': 0.0, 'records': 0.0,
                               'batches': 0}
        clock = time.perf_counter
        while True:
            t0 = clock()
            prof['batches'] += 1
            last_start = blen
            while nxt is not None and (blen < self.batch_bytes or blen == 0):
                piece, _ = nxt
                last_start = blen
                hnp[blen:blen + len(piece)] = np.frombuffer(piece, dtype=np.uint8)
                blen += len(piece)
                nxt = next(it, None)
            final = nxt is None
            closed = len(files) if final else nxt[1]
            t1 = clock()
            prof['fill'] += t1 - t0
            # ---- host: per-file digests of the large files, hashed from the pinned batch while
            # the device works on it (see _on_host)
            lo_stream, hi_stream = buf_start + fed, buf_start + blen
            host_jobs = []       # (file index, future or None, final)
            for fi in range(finalized, len(files)):
                if not self._on_host(fi, files[fi], hstates, engine):
                    continue
                f = files[fi]
                a, b = max(f.stream_start, lo_stream), min(f.stream_end, hi_stream)
                is_final = fi < closed
                if b <= a and not is_final:
                    continue
                fut = None
                if b > a:
                    fut = self._host_pool().submit(hstates[fi].update,
                                                   memoryview(hnp)[a - buf_start:b - buf_start])
                host_jobs.append((fi, fut, is_final))
            # ---- device: upload, cut chain, chunk digests
            if blen:
                self.dbuf[:blen].copy_(self.host[:blen], non_blocking=True)
            ptr = self.dbuf.data_ptr()
            self.chunker.chunk_device([ptr], [blen], [last_start], self.d_cuts.data_ptr(),
                                      self.d_count.data_ptr(), hs, open_=not final)
            self.hasher.digest_chunks(self.chunker, [ptr], [blen], self.d_cuts.data_ptr(),
                                      self.d_count.data_ptr(), self.d_digests.data_ptr(), hs)
            if self.encryption is not None:
                # derive_shared_subkey(digest) and encrypt, per chunk, still in HBM; one
                # os.urandom nonce per chunk as the adapter draws them (adapters.py:133)
                self.hasher.derive_chunks(self.chunker, [blen], self.d_count.data_ptr(),
                                          self.d_kdf.data_ptr(), self.d_digests.data_ptr(),
                                          self.d_keys.data_ptr(), hs)
                self.h_nonces.numpy()[:] = np.frombuffer(os.urandom(self.h_nonces.numel()),
                                                         dtype=np.uint8)
                self.d_nonces.copy_(self.h_nonces, non_blocking=True)
                self.cipher.encrypt_chunks(self.chunker, [ptr], [blen], self.d_cuts.data_ptr(),
                                           self.d_count.data_ptr(), self.d_keys.data_ptr(),
                                           self.d_nonces.data_ptr(), self.d_enc.data_ptr(), hs)
            # ---- device: per-file incremental digests over the fresh bytes [fed, blen)
            items = []           # (file index, device ptr, length, final)
            for fi in range(finalized, len(files)):
                if engine.get(fi):
                    continue
                f = files[fi]
                a, b = max(f.stream_start, lo_stream), min(f.stream_end, hi_stream)
                n = b - a if b > a else 0
                is_final = fi < closed
                if n == 0 and not is_final:
                    continue
                items.append((fi, ptr + (a - buf_start) if n else 0, n, is_final))
            file_digests = None
            if items:
                for fi, _, _, _ in items:
                    if fi not in states:
                        states[fi] = torch.from_numpy(self._init_state.copy()).to(self.dev)
                scratch = torch.zeros((len(items), SLOT), dtype=torch.uint8, device=self.dev)
                self.hasher.update_device([states[fi].data_ptr() for fi, _, _, _ in items],
                                          [p for _, p, _, _ in items], [n for _, _, n, _ in items],
                                          [1 if fin else 0 for _, _, _, fin in items],
                                          scratch.data_ptr(), hs)
                file_digests = scratch
            # ---- results back
            count = int(self.d_count.cpu()[0])
            if count < 0:
                raise RuntimeError('cut capacity overflow')
            ends = self.d_cuts[:count].cpu().numpy().view(np.uint64).astype(np.int64)
            digs = self.d_digests[:count, :self.digest_size].cpu().numpy()
            enc = None
            if self.encryption is not None:
                over = self.cipher.nonce_bytes + 16
                n_out = (int(ends[-1]) if count else 0) + count * over
                self.h_enc[:n_out].copy_(self.d_enc[:n_out], non_blocking=True)
                stream.synchronize()
                enc = self.h_enc[:n_out].numpy()
            if file_digests is not None:
                fd = file_digests[:, :self.digest_size].cpu().numpy()
                for j, (fi, _, _, fin) in enumerate(items):
                    if fin:
                        files[fi].digest = fd[j].tobytes()
                        del states[fi]
            t2 = clock()
            prof['device'] += t2 - t1
            for fi, fut, fin in host_jobs:  # before the batch buffer is reused
                if fut is not None:
                    fut.result()
                if fin:
                    files[fi].digest = hstates.pop(fi).digest()
            t3 = clock()
            prof['host_digest_wait'] += t3 - t2
            while finalized < closed and files[finalized].digest is not None:
                finalized += 1
            prev = 0
            for k, e in enumerate(ends.tolist()):
                d = digs[k].tobytes()
                idx = table.get(d)
                if idx is None:
                    idx = table[d] = len(table)
                if enc is not None:  # nonce || C || T of chunk k at prev + k (nonce_bytes + 16)
                    o = prev + k * over
                    contents = enc[o:o + (e - prev) + over].tobytes()
                else:
                    contents = hnp[prev:e].tobytes() if self.keep_contents else None
                chunks.append(ChunkRecord(counter=len(chunks) + 1, stream_start=buf_start + prev,
                                          stream_end=buf_start + e, digest=d, table_index=idx,
                                          contents=contents))
                prev = e
            prof['records'] += clock() - t3
            if final:
                if prev != blen:
                    raise RuntimeError(f'final batch left {blen - prev} bytes uncut')
                break
            # carry the uncut tail (< max_length bytes) to the front of the buffer
            tail = blen - prev
            if tail:
                hnp[:tail] = hnp[prev:blen].copy()
            buf_start += prev
            blen = tail
            fed = blen
        return SnapshotStream(files=files, chunks=chunks, chunks_table=table)


def snapshot_stream(paths, **kw) -> SnapshotStream:
    """One-shot helper: DeviceSnapshotProducer(**kw).run(paths)."""
    return DeviceSnapshotProducer(**kw).run(paths)


__all__ = ['DeviceSnapshotProducer', 'SnapshotStream', 'FileRecord', 'ChunkRecord', 'ChunkEncryption',
           'tagged_pieces', 'snapshot_stream', 'DEFAULT_BATCH']
