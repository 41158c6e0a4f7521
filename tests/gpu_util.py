"""Device helpers for the -m gpu tests: streams live in torch CUDA (HIP) tensors; the chunker
is called through the C ABI (replicat_amd.chunker -> libreplicat_chunker.so)."""
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
