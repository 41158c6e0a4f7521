"""Device helpers for the -m gpu tests: streams live in torch CUDA (HIP) tensors; the chunker
is called through the C ABI (replicat_amd.chunker -> libreplicat_chunker.so)."""
import hashlib
import os

import numpy as np
import torch

from replicat_amd.chunker import GpuChunker, fill_splitmix


def device_streams(sizes, seed=None, fill=None, datas=None, ids=None):
    """One 16-byte aligned torch allocation per stream (splitmix synthetic bytes, a constant
    fill, or host data copied in)."""
    out = []
    for i, n in enumerate(sizes):
        t = torch.empty(max(int(n), 1) + 16, dtype=torch.uint8, device='cuda')
        if datas is not None:
            if n:
                # a writable copy: torch.from_numpy warns on (and may not own) read-only
                # buffers such as np.frombuffer over bytes
                t[:n].copy_(torch.from_numpy(np.array(datas[i], dtype=np.uint8, copy=True)))
        elif fill is not None:
            t.fill_(fill)
        else:
            fill_splitmix(t.data_ptr(), int(n), seed, ids[i] if ids else i,
                          torch.cuda.current_stream().cuda_stream)
        out.append(t)
    return out


def chunk_device(ch: GpuChunker, tensors, sizes, last=None, open_=False, pipelined=False):
    total, caps = ch.capacity(sizes)
    cuts = torch.zeros(max(total, 1), dtype=torch.int64, device='cuda')
    counts = torch.zeros(len(sizes), dtype=torch.int64, device='cuda')
    hs = torch.cuda.current_stream().cuda_stream
    ch.chunk_device([t.data_ptr() for t in tensors], sizes, last, cuts.data_ptr(),
                    counts.data_ptr(), hs, open_, pipelined=pipelined)
    if pipelined:
        ch.wait(hs)
    torch.cuda.synchronize()
    cuts = cuts.cpu().numpy().view(np.uint64)
    counts = counts.cpu().numpy()
    base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    assert (counts >= 0).all(), 'cut capacity overflow'
    return [cuts[b:b + c].tolist() for b, c in zip(base, counts)]


_EXPECTED = {}


def _oracle_threads():
    # the GPU box's host share (OMP_NUM_THREADS there); nproc shows the whole machine
    return max(1, min(16, int(os.environ.get('OMP_NUM_THREADS') or 0) or (os.cpu_count() or 1)))


def expected_cuts(datas, mn, mx, key, lasts):
    """The oracle's cut END lists of many streams at once (oracle.chunk_streams_mt: the C
    restatement, one host thread per stream), memoised per (bytes, params, last piece): tests
    that vary only a device knob over the same streams compute their expectations once.
    lasts[i] is the stream's last-piece start (len: the whole stream is one non-final piece)."""
    from oracle import oracle as o
    ids = [(hashlib.blake2b(memoryview(np.ascontiguousarray(d, dtype=np.uint8)), digest_size=16).digest(),
            len(d), mn, mx, key, int(P)) for d, P in zip(datas, lasts)]
    todo = [i for i, k in enumerate(ids) if k not in _EXPECTED]
    if todo:
        bufs = []
        for i in todo:
            b = np.zeros(len(datas[i]) + 16, np.uint8)
            b[:len(datas[i])] = np.asarray(datas[i], dtype=np.uint8)
            bufs.append(b)
        got = o.chunk_streams_mt(bufs, [len(datas[i]) for i in todo], [int(lasts[i]) for i in todo],
                                 mn, mx, key, threads=_oracle_threads())
        for i, g in zip(todo, got):
            _EXPECTED[ids[i]] = g
    if len(_EXPECTED) > 20000:  # bounded: a long session keeps only the latest
        for k in list(_EXPECTED)[:10000]:
            del _EXPECTED[k]
    return [_EXPECTED[k] for k in ids]


def open_prefix(full, n, mx):
    """RC_OPEN (non-final prefix): the argmax cuts of the stream's full list only, while at
    least max_length bytes remain (no tail rule)."""
    exp, s = [], 0
    for e in full:
        if n - s < mx:
            break
        exp.append(e)
        s = e
    return exp
