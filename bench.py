"""bench.py -- device-resident chunking throughput of the MI355X chunker (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY.md §8 d config 2): per GPU, 1024 synthetic
splitmix64 streams x 64 MiB (64 GiB resident in HBM), replicat's default chunk parameters
(min 128,000 / max 5,120,000), unencrypted key (0xff * 16), one piece per stream.
One step = one pass of the hot path over the whole batch: rc_chunk_device (tile kernel over
every byte + chain kernel per stream), cut offsets left in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

Ranks shard the work per stream (stream ids rank*1024 ..), with no data-path collective:
"scaling": "weak".  Rank 0 prints one JSON line.  Parity is checked in-run: rank 0's cut lists
hash to the reference's SHA-256 for config 2 (tests/golden/digests.json).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = 1 << 30
MIN_LEN, MAX_LEN = 128_000, 5_120_000
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=10)
    p.add_argument('--warmup', type=int, default=2)
    p.add_argument('--config', choices=['2', '3i', '3iii', '4'], default='2',
                   help='2: 1024 x 64 MiB (the metric); 3i: 65536 x 1 MiB default params '
                        '(degenerate: tail rule only); 3iii: 65536 x 1 MiB, min 2000 / max 80000; '
                        '4: 16 x 8 GiB per GPU (streams rank, rank+8, ...)')
    p.add_argument('--streams', type=int, default=None)
    p.add_argument('--stream-mib', type=int, default=None)
    p.add_argument('--calibrate', action='store_true',
                   help='also time a pure streaming read of the same bytes (rc_read_probe)')
    p.add_argument('--key', choices=['ff', 'seeded'], default='ff')
    p.add_argument('--cpu-streams', type=int, default=256,
                   help='bounded CPU-baseline sample (64 MiB streams); 0 = skip')
    p.add_argument('--cpu-procs', type=int, default=16)
    p.add_argument('--e2e', action='store_true', help='also time the host-resident path')
    p.add_argument('--no-verify', action='store_true')
    return p.parse_args()


def cut_digest(cuts_dev, counts_dev, caps):
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import golden_util as G
    cuts = cuts_dev.cpu().numpy().view(np.uint64)
    counts = counts_dev.cpu().numpy()
    base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    ends = [cuts[b:b + c] for b, c in zip(base, counts)]
    return G.cutlist_digest(ends), int(counts.sum()), ends


# ------------------------------------------------------------------------ CPU baseline

def _cpu_worker(args):
    kind, ids, size, seed = args
    from replicat_amd import synth
    out = []
    if kind == 'reference':
        sys.path.insert(0, os.path.join(ROOT, 'oracle', '_ref'))
        import _replicat_adapters as ref  # the reference's own chunker, built by oracle/Makefile
        ch = ref._gclmulchunker(MIN_LEN, MAX_LEN, b'\xff' * 16)
        t = 0.0
        for i in ids:
            data = synth.stream_bytes(size, seed, i)
            mv = memoryview(data)
            t0 = time.perf_counter()
            pos, ends = 0, []
            while pos < size:  # next_cut on a zero-copy view: the native scan alone
                c = ch.next_cut(mv[pos:], True)
                if not c:
                    break
                pos += c
                ends.append(pos)
            t += time.perf_counter() - t0
            out.append(ends)
        return t, out
    from oracle import oracle as o
    t = 0.0
    for i in ids:
        data = synth.stream_bytes(size, seed, i)
        t0 = time.perf_counter()
        out.append(o.chunk_stream(data, MIN_LEN, MAX_LEN, None, 0))
        t += time.perf_counter() - t0
    return t, out


def cpu_baseline(n_streams, size, seed, procs):
    import multiprocessing as mp
    import glob
    kind = 'reference' if glob.glob(os.path.join(ROOT, 'oracle', '_ref', '_replicat_adapters*.so')) \
        else 'port'
    if kind == 'port':
        from oracle import oracle as o
        o.lib()
    procs = max(1, min(procs, n_streams))
    shards = [list(range(r, n_streams, procs)) for r in range(procs)]
    t0 = time.perf_counter()
    with mp.get_context('fork').Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(kind, s, size, seed) for s in shards])
    wall = time.perf_counter() - t0
    busiest = max(r[0] for r in res)  # scan time of the slowest process (generation excluded)
    ends = {}
    for s, (_, out) in zip(shards, res):
        for i, e in zip(s, out):
            ends[i] = e
    gibs = n_streams * size / busiest / GIB
    return {'value': round(gibs, 3), 'unit': 'GiB/s', 'cores': procs, 'kind': kind,
            'sample': f'{n_streams} x {size >> 20} MiB of the same synthetic streams '
                      f'(ids 0..{n_streams - 1}), one process per core, '
                      f'native next_cut scan time of the slowest process ({busiest:.2f} s; '
                      f'{wall:.1f} s wall incl. data generation)'}, ends


# ------------------------------------------------------------------- multi-GPU plumbing

def shard_ids(config, rank, n):
    """Stream ids a rank chunks (weak scaling: every rank has its own n streams).  Config 4
    follows the north star's round-robin: stream i lives on GPU i mod 8."""
    if config == '4':
        return [rank + 8 * i for i in range(n)]
    return [rank * n + i for i in range(n)]


def reduce_max(values, dist, device):
    """Max over ranks of a few floats (elapsed time, kernel times): the job is as slow as its
    slowest rank.  The only collective the bench uses besides its barriers."""
    import torch
    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


# ------------------------------------------------------------------------------ main

def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    from replicat_amd import synth
    from replicat_amd.chunker import GpuChunker, fill_splitmix, read_probe
    key = b'\xff' * 16 if args.key == 'ff' else synth.seeded_key(1)
    cfg = {'2': (1024, 64, MIN_LEN, MAX_LEN), '3i': (65536, 1, MIN_LEN, MAX_LEN),
           '3iii': (65536, 1, 2_000, 80_000), '4': (16, 8192, MIN_LEN, MAX_LEN)}[args.config]
    n = args.streams or cfg[0]
    size = (args.stream_mib or cfg[1]) << 20
    min_len, max_len = cfg[2], cfg[3]
    ch = GpuChunker(min_len, max_len, key, device=local)
    stream = torch.cuda.current_stream()
    hs = stream.cuda_stream
    pool = torch.empty(n * size, dtype=torch.uint8, device='cuda')  # one 16-B aligned arena
    base_ptr = pool.data_ptr()
    ptrs = [base_ptr + i * size for i in range(n)]
    ids = shard_ids(args.config, rank, n)
    for p, i in zip(ptrs, ids):
        fill_splitmix(p, size, synth.DEFAULT_SEED, i, hs)
    lens = [size] * n
    total_cap, caps = ch.capacity(lens)
    cuts = torch.zeros(total_cap, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    torch.cuda.synchronize()

    def step():
        ch.chunk_device(ptrs, lens, None, cuts.data_ptr(), counts.data_ptr(), hs)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ch.timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ch.timing(False)
    a_ms, b_ms, calls = ch.read_timing()
    if world > 1:
        elapsed, a_ms, b_ms = reduce_max([elapsed, a_ms, b_ms], dist, 'cuda')

    bytes_per_step = n * size
    value = world * bytes_per_step * args.steps / elapsed / GIB
    ms_per_step = elapsed * 1e3 / args.steps
    a_avg = a_ms / max(calls, 1)
    b_avg = b_ms / max(calls, 1)
    achieved = bytes_per_step / (a_avg * 1e-3) / 1e9  # GB/s, ΣL per tile-kernel launch

    parity = None
    ends = None
    if not args.no_verify and rank == 0:
        digest, nchunks, ends = cut_digest(cuts, counts, caps)
        sys.path.insert(0, os.path.join(ROOT, 'tests'))
        import golden_util as G
        gold = {d['name']: d for d in G.load('digests.json')}
        if args.key == 'ff' and n == 1024 and size == 64 << 20 and args.config == '2':
            parity = digest == gold['config2_ff']['sha256']
        elif args.key == 'ff' and args.config == '3iii' and n >= 4096:
            parity = G.cutlist_digest(ends[:4096]) == gold['config3iii_first4096']['sha256']
    if world > 1:
        dist.barrier()

    result = None
    if rank == 0:
        cpu = None
        if args.cpu_streams and world == 1 and args.key == 'ff' and args.config == '2':
            cpu, cpu_ends = cpu_baseline(min(args.cpu_streams, n), size, synth.DEFAULT_SEED,
                                         args.cpu_procs)
            if ends is not None:
                same = all(np.array_equal(np.asarray(cpu_ends[i], np.uint64), ends[i])
                           for i in cpu_ends)
                cpu['matches_gpu'] = bool(same)
        e2e = None
        if args.e2e:  # host-resident streams: copies in, chunking, cut offsets out
            m = min(n, 64)
            hbufs = [synth.stream_bytes(size, synth.DEFAULT_SEED, i) for i in range(m)]
            pinned = torch.empty(m * size, dtype=torch.uint8).pin_memory()
            pv = pinned.numpy()
            for i, b in enumerate(hbufs):
                pv[i * size:(i + 1) * size] = b
            pbufs = [pv[i * size:(i + 1) * size] for i in range(m)]
            e2e = {}
            for label, bufs in (('pageable', hbufs), ('pinned', pbufs)):
                ch.chunk_host(bufs[:2])
                t1 = time.perf_counter()
                ch.chunk_host(bufs)
                e2e[label] = round(m * size / (time.perf_counter() - t1) / GIB, 2)
            e2e['streams'] = m
        calib = None
        if args.calibrate:
            out = torch.zeros(4, dtype=torch.int32, device='cuda')
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(2):
                read_probe(base_ptr, n * size, out.data_ptr(), hs)
            ev0.record(stream)
            for _ in range(5):
                read_probe(base_ptr, n * size, out.data_ptr(), hs)
            ev1.record(stream)
            torch.cuda.synchronize()
            calib = round(5 * n * size / (ev0.elapsed_time(ev1) * 1e-3) / 1e9, 1)
        result = {
            'metric': 'GiB/s chunked, device-resident streams',
            'value': round(value, 2),
            'unit': 'GiB/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms_per_step, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'u8',
            'data': 'synthetic (splitmix64 counter streams generated in HBM)',
            'config': {'workload': 'config%s: %d x %d MiB streams per GPU, min %d, max %d, key %s'
                                   % (args.config, n, size >> 20, min_len, max_len, args.key),
                       'streams_per_gpu': n, 'stream_bytes': size, 'parallelism': f'streams/{world} ranks'},
            'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4),
                         'traffic': None, 'kernel': 'rc_tile_kernel',
                         'kernel_ms': round(a_avg, 3), 'chain_kernel_ms': round(b_avg, 3)},
            'cpu_baseline': cpu,
            'parity_sha256': parity,
        }
        if calib is not None:
            result['read_probe_gbs'] = calib
        if e2e is not None:
            result['e2e_host_gibs'] = e2e
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return result


if __name__ == '__main__':
    main()
