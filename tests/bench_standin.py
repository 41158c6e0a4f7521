"""A CPU stand-in for bench.py's device calls (test infrastructure: its chunker is the oracle).

Used two ways:
* imported -- ``bench.main(argv, backend=CpuBackend)`` inside gloo ranks the test spawns;
* as a script -- ``python tests/bench_standin.py --gpus N ...`` is bench.py's own command line
  (``bench.cli``): with no launcher around it, it starts the N ranks itself as a child
  ``torch.distributed.run`` over THIS script, so every rank runs the stand-in.

``RC_STANDIN_DEVICES=k`` makes the stand-in expose only k distinct devices (ranks wrap round,
as Backend does on a box with fewer GPUs than ranks)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


class OracleChunker:
    """GpuChunker's surface as bench.py uses it, over host memory, computed by the oracle."""

    def __init__(self, min_length, max_length, key, log):
        from oracle import oracle as o
        self.o, self.log = o, log
        self.min_length, self.max_length, self.key = min_length, max_length, key
        self.calls = 0
        self.pipelined_calls_n = 0

    def overlap(self, reserve_cus=0):
        return reserve_cus or 32

    def overlap_cus(self):
        return 32

    def wait(self, stream=0):
        pass

    def check(self):  # the oracle has no tile kernel, so no fail-safe stop
        pass

    def pipelined_calls(self):
        return self.pipelined_calls_n

    def capacity(self, lens):
        step = max(4, (self.min_length + 3) & ~3)
        caps = np.array([int(L) // step + 3 for L in lens], dtype=np.uint64)
        return int(caps.sum()), caps

    def chunk_device(self, ptrs, lens, last, cuts_ptr, counts_ptr, stream=0, open_=False,
                     pipelined=False, end=False):
        self.pipelined_calls_n += bool(pipelined)
        _, caps = self.capacity(lens)
        base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
        n = len(lens)
        cuts = np.ctypeslib.as_array((ctypes.c_uint64 * int(caps.sum())).from_address(cuts_ptr))
        counts = np.ctypeslib.as_array((ctypes.c_int64 * n).from_address(counts_ptr))
        for i, (p, L) in enumerate(zip(ptrs, lens)):
            data = np.frombuffer(ctypes.string_at(int(p), int(L)), dtype=np.uint8)
            P = int(L) if open_ else (int(last[i]) if last is not None else 0)
            ends = self.o.chunk_stream(data, self.min_length, self.max_length, self.key, P)
            if open_:  # non-final prefix: cut while L - s >= max (RC_OPEN)
                out, s = [], 0
                for e in ends:
                    if L - s < self.max_length:
                        break
                    out.append(e)
                    s = e
                ends = out
            cuts[base[i]:base[i] + len(ends)] = ends
            counts[i] = len(ends)
            self.log.append(bytes(data[:16]))
        self.calls += 1

    def timing(self, enable):
        if enable:
            self.calls = 0

    def read_kernel_timing(self):
        return 1.0 * self.calls, 0.1 * self.calls, 0.2 * self.calls, self.calls


class CpuBackend:
    device = 'cpu'

    def __init__(self, local_rank):
        k = int(os.environ.get('RC_STANDIN_DEVICES', '0') or 0)
        self.index = local_rank % k if k > 0 else local_rank
        self.log = []

    def identity(self):
        return {'device': self.index, 'pci': '0000:%02x:00' % (0x10 + self.index),
                'uuid': 'standin-%d' % self.index, 'name': 'cpu stand-in', 'visible': None}

    def empty(self, nbytes):
        return torch.empty(nbytes, dtype=torch.uint8)

    def zeros_i64(self, n):
        return torch.zeros(max(n, 1), dtype=torch.int64)

    def stream(self):
        return 0

    def synchronize(self):
        pass

    def chunker(self, min_len, max_len, key):
        return OracleChunker(min_len, max_len, key, self.log)

    def fill_streams(self, ptr, n, size, slot, seed, first_id, id_step):
        from oracle import oracle as o
        for k in range(n):
            b = o.fill_splitmix(size, seed, first_id + k * id_step)
            ctypes.memmove(ptr + k * slot, b.ctypes.data, size)

    def fill_at(self, ptr, nbytes, seed, stream_id, word0):
        from replicat_amd import synth
        w = synth.splitmix_words(synth.stream_base(seed, stream_id), word0, (nbytes + 7) // 8)
        ctypes.memmove(ptr, w.view(np.uint8).ctypes.data, nbytes)


if __name__ == '__main__':
    sys.exit(bench.cli(backend=CpuBackend, script=os.path.abspath(__file__)))
