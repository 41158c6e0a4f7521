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
    p.add_argument('--streams', type=int, default=1024)
    p.add_argument('--stream-mib', type=int, default=64)
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
    from replicat_amd.chunker import GpuChunker, fill_splitmix
    key = b'\xff' * 16 if args.key == 'ff' else synth.seeded_key(1)
    ch = GpuChunker(MIN_LEN, MAX_LEN, key, device=local)

    n, size = args.streams, args.stream_mib << 20
    stream = torch.cuda.current_stream()
    hs = stream.cuda_stream
    pool = torch.empty(n * size, dtype=torch.uint8, device='cuda')  # one 16-B aligned arena
    base_ptr = pool.data_ptr()
    ptrs = [base_ptr + i * size for i in range(n)]
    ids = [rank * n + i for i in range(n)]
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
        t = torch.tensor([elapsed, a_ms, b_ms], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, a_ms, b_ms = t.tolist()

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
        if args.key == 'ff' and n == 1024 and size == 64 << 20:
            parity = digest == gold['config2_ff']['sha256']
    if world > 1:
        dist.barrier()

    result = None
    if rank == 0:
        cpu = None
        if args.cpu_streams and world == 1 and args.key == 'ff':
            cpu, cpu_ends = cpu_baseline(min(args.cpu_streams, n), size, synth.DEFAULT_SEED,
                                         args.cpu_procs)
            if ends is not None:
                same = all(np.array_equal(np.asarray(cpu_ends[i], np.uint64), ends[i])
                           for i in cpu_ends)
                cpu['matches_gpu'] = bool(same)
        e2e = None
        if args.e2e:
            hbufs = [synth.stream_bytes(size, synth.DEFAULT_SEED, i) for i in range(16)]
            ch.chunk_host(hbufs[:2])
            t1 = time.perf_counter()
            ch.chunk_host(hbufs)
            e2e = round(16 * size / (time.perf_counter() - t1) / GIB, 2)
        result = {
            'metric': 'GiB/s chunked, device-resident streams (config 2: 1024 x 64 MiB per GPU)',
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
            'config': {'workload': 'config2: %d x %d MiB streams per GPU, min %d, max %d, key %s'
                                   % (n, size >> 20, MIN_LEN, MAX_LEN, args.key),
                       'streams_per_gpu': n, 'stream_bytes': size, 'parallelism': f'streams/{world} ranks'},
            'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4),
                         'traffic': None, 'kernel': 'rc_tile_kernel',
                         'kernel_ms': round(a_avg, 3), 'chain_kernel_ms': round(b_avg, 3)},
            'cpu_baseline': cpu,
            'parity_config2_sha256': parity,
        }
        if e2e is not None:
            result['e2e_host_gibs'] = e2e
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return result


if __name__ == '__main__':
    main()
