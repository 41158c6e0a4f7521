"""bench.main's N > 1 control flow on the CPU: world size 2 over gloo (what bench.py uses on the
GPU box too -- the data path has no collective), with the device calls replaced by a CPU
stand-in whose chunker is the oracle.  Checks device selection per LOCAL_RANK, the shards each
rank fills and chunks, the weak-scaling value formula, the max-over-ranks timing, per-rank
parity gathering, and config 3 (ii)'s split + gather + splice of one stream over two ranks."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import bench

GIB = 1 << 30


class OracleChunker:
    """GpuChunker's surface as bench.py uses it, over host memory, computed by the oracle."""

    def __init__(self, min_length, max_length, key, log):
        from oracle import oracle as o
        self.o, self.log = o, log
        self.min_length, self.max_length, self.key = min_length, max_length, key
        self.calls = 0

    def capacity(self, lens):
        step = max(4, (self.min_length + 3) & ~3)
        caps = np.array([int(L) // step + 3 for L in lens], dtype=np.uint64)
        return int(caps.sum()), caps

    def chunk_device(self, ptrs, lens, last, cuts_ptr, counts_ptr, stream=0, open_=False):
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
    used = []

    def __init__(self, local_rank):
        self.index = local_rank
        self.log = []

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


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, argv, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    try:
        res = bench.main(argv, backend=CpuBackend)
        last = bench.LAST
        ends = [np.asarray(e).tolist() for e in last['ends']] if last.get('ends') is not None else None
        q.put((rank, res, last['device'], ends, last['parity']))
    except Exception as e:  # noqa: BLE001 - report to the parent
        q.put((rank, repr(e), None, None, None))
        raise


def _run(argv, world=2):
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, argv, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_config2_two_ranks():
    n, mib, steps = 3, 1, 2
    out = _run(['--config', '2', '--streams', str(n), '--stream-mib', str(mib), '--steps',
                str(steps), '--warmup', '1', '--cpu-streams', '0', '--min-length', '2000',
                '--max-length', '80000'])
    from oracle import oracle as o
    from replicat_amd import synth
    (r0, res0, dev0, ends0, _), (r1, res1, dev1, ends1, _) = out
    assert (dev0, dev1) == (0, 1)                              # device = LOCAL_RANK
    assert isinstance(res0, dict) and res1 is None             # rank 0 prints the line
    assert res0['n_gpus'] == 2 and res0['scaling'] == 'weak'
    size = mib << 20
    # value = all ranks' bytes / the slowest rank's time
    per_step = res0['ms_per_step'] / 1e3
    assert res0["value"] == pytest.approx(2 * n * size / per_step / GIB, rel=1e-2)  # both rounded
    # kernel times are the max over ranks of the stand-in's per-call figures
    assert res0['roofline']['kernel_ms'] == pytest.approx(1.0)
    assert res0['roofline']['chain_kernel_ms'] == pytest.approx(0.2)
    # each rank chunked its own shard: stream ids rank * n ..
    for rank, ends in ((0, ends0), (1, ends1)):
        ids = bench.shard_ids('2', rank, n)
        assert ids == list(range(rank * n, rank * n + n))
        for i, e in zip(ids, ends):
            data = synth.stream_bytes(size, synth.DEFAULT_SEED, i)
            assert e == o.chunk_stream(data, 2000, 80000, None, 0)


def test_config3ii_split_over_two_ranks():
    """One stream split in two windows, chunked per rank, gathered and spliced: every rank ends
    with the whole true cut list of the stream."""
    mib = 4
    out = _run(['--config', '3ii', '--stream-mib', str(mib), '--steps', '1', '--warmup', '0',
                '--cpu-streams', '0', '--min-length', '2000', '--max-length', '80000'])
    from oracle import oracle as o
    from replicat_amd import synth
    L = 2 * (mib << 20)
    exp = o.chunk_stream(synth.stream_bytes(L, synth.DEFAULT_SEED, 0), 2000, 80000, None,
                         L - (1 << 20))
    for _, res, _, ends, _ in out:
        assert ends[0] == exp
    assert out[0][1]['config']['parallelism'] == 'one stream split over 2 ranks'


def test_parity_flags_gathered_for_config4():
    """Config 4's parity is the AND of every rank's own-shard check; a workload the fixtures do
    not cover (here 2 x 1 MiB per rank) carries no flag on any rank and none in the line."""
    out = _run(['--config', '4', '--streams', '2', '--stream-mib', '1', '--steps', '1',
                '--warmup', '0', '--cpu-streams', '0'])
    (_, res0, _, ends0, p0), (_, _, _, ends1, p1) = out
    assert p0 is None and p1 is None  # not the config-4 sizes: no fixture, no flag
    assert res0['parity_sha256'] is None
    # round-robin shards: rank r holds streams r, r + 8
    assert bench.shard_ids('4', 1, 2) == [1, 9]
