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
    p.add_argument('--config', choices=['2', '3i', '3ii', '3iii', '4', '5'], default='2',
                   help='2: 1024 x 64 MiB (the metric); 3i: 65536 x 1 MiB default params '
                        '(degenerate: tail rule only); 3ii: ONE 64 GiB stream, last piece the '
                        'final 1 MiB (snapshot framing, segment-parallel chain); 3iii: 65536 x '
                        '1 MiB, min 2000 / max 80000; 4: 16 x 8 GiB per GPU (streams rank, '
                        'rank+8, ...); 5: re-chunk of config 2 with 512 edited copies + dedup '
                        'ratio check')
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


# ---------------------------------------------------------------- PMC traffic (profiles/)

def pmc_traffic(args, n, size):
    """HBM bytes per rc_tile_kernel launch from the committed rocprofv3 PMC summary of this same
    command (scripts/gpu_profile.sh -> scripts/summarize_profile.py: separate --pmc passes,
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM, WRITE_SIZE as is), or None when no summary
    covers this workload.  bench.py cannot read counters itself (that needs rocprofv3)."""
    if not (args.config == '2' and args.key == 'ff' and n == 1024 and size == 64 << 20):
        return None, None
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*', 'pmc_summary.json')),
                    reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        t = d.get('rc_tile_kernel', {})
        if d.get('workload') == 'config2' and 'hbm_read_bytes_corrected' in t:
            return (t['hbm_read_bytes_corrected'] + t.get('hbm_write_bytes', 0.0),
                    os.path.relpath(f, ROOT))
    return None, None


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


# ------------------------------------------------------------------- config 5 (dedup)

class Config5:
    """config 2's streams, of which 512 (synth.edit_plan) get one edit
    each; the edited set is re-chunked and its dedup ratio against the original set computed.

    Content identity on the device: an edited-set chunk can only equal an original chunk of the
    same stream at the same bytes -- before the edit at the same offsets, after it shifted by the
    insert length -- so those candidates are looked up by offset and confirmed by comparing the
    bytes in HBM (torch.equal).  The reference value (tests/golden/large.json) looks every chunk
    up by BLAKE2b-512 content digest over the whole original set instead, so the two agree only
    if no other coincidence exists."""

    def __init__(self, ch, pool, slot, n, size, rank, hs):
        import torch
        from replicat_amd import synth
        self.size, self.slot, self.n = size, slot, n
        self.orig = pool
        base = pool.data_ptr()
        olens = [size] * n
        cap, ocaps = ch.capacity(olens)
        ocuts = torch.zeros(cap, dtype=torch.int64, device='cuda')
        ocounts = torch.zeros(n, dtype=torch.int64, device='cuda')
        ch.chunk_device([base + i * slot for i in range(n)], olens, None, ocuts.data_ptr(),
                        ocounts.data_ptr(), hs)
        self.orig_digest, _, self.orig_ends = cut_digest(ocuts, ocounts, ocaps)
        plan = synth.edit_plan(n, n // 2, size) if rank == 0 and n == 1024 else []
        self.plan = {sid: (kind, off, payload) for sid, kind, off, payload in plan}
        self.edited = sorted(self.plan)
        self.buf = torch.empty(n * slot + 64, dtype=torch.uint8, device='cuda')
        self.lens = []
        for i in range(n):
            src = pool[i * slot:i * slot + size]
            dst = self.buf[i * slot:]
            kind, off, payload = self.plan.get(i, (None, 0, b''))
            if kind is None:
                dst[:size].copy_(src)
            elif kind == 'overwrite1':
                dst[:size].copy_(src)
                dst[off:off + 1] ^= 0x5A
            else:
                k = len(payload)
                dst[:off].copy_(src[:off])
                dst[off:off + k].copy_(torch.tensor(list(payload), dtype=torch.uint8))
                dst[off + k:size + k].copy_(src[off:])
            self.lens.append(size + len(payload))
        self.ptrs = [self.buf.data_ptr() + i * slot for i in range(n)]

    def dedup(self, ends):
        """Dedup bytes of the edited streams (integers, comparable with the reference's)."""
        dup = total = 0
        for sid in self.edited:
            kind, off, payload = self.plan[sid]
            d = len(payload)
            lo_end = off            # a chunk ending at or before this is untouched
            hi_start = off + max(d, 1)  # a chunk starting here or later is shifted by d
            orig = self.orig_ends[sid]
            ostarts, prev = {}, 0
            for e in orig:
                ostarts[prev] = int(e)
                prev = int(e)
            a = 0
            for e in ends[sid]:
                e = int(e)
                if e <= lo_end:
                    oa, ob = a, e
                elif a >= hi_start:
                    oa, ob = a - d, e - d
                else:
                    oa = ob = None
                if oa is not None and ostarts.get(oa) == ob:
                    x = self.orig[sid * self.slot + oa:sid * self.slot + ob]
                    y = self.buf[sid * self.slot + a:sid * self.slot + e]
                    if bool((x == y).all()):
                        dup += e - a
                a = e
            total += a
        return {'dup_bytes_edited': dup, 'total_bytes_edited': total,
                'dedup_ratio_edited': round(dup / total, 6) if total else None}


# -------------------------------------------------------- config 3 (ii): one long stream

class Config3ii:
    """ONE stream of world x 64 GiB (last piece = the final 1 MiB) split over the ranks
    (replicat_amd/split.py): each rank fills and chunks its window (segment + halo) with a
    speculative chain, the ranks exchange their cut lists through a host-side (gloo) gather and
    splice them.  One rank: the plain single-stream path (segment-parallel chain on one GPU)."""

    def __init__(self, ch, size, rank, world, hs, dist):
        import torch
        from replicat_amd import split, synth
        from replicat_amd.chunker import fill_splitmix_at
        self.ch, self.rank, self.world, self.hs = ch, rank, world, hs
        self.L = size * world
        self.P = self.L - (1 << 20)
        self.windows = split.plan_windows(self.L, self.P, world, ch.max_length)
        w = self.windows[rank]
        self.w = w
        self.buf = torch.empty(w.end - w.start + 64, dtype=torch.uint8, device='cuda')
        fill_splitmix_at(self.buf.data_ptr(), w.end - w.start, synth.DEFAULT_SEED, 0,
                         w.start // 8, hs)
        self.lens = [w.end - w.start]
        _, caps = ch.capacity(self.lens)
        self.cap = int(caps[0])
        self.cuts = torch.zeros(self.cap + 1, dtype=torch.int64, device='cuda')
        self.counts = torch.zeros(1, dtype=torch.int64, device='cuda')
        self.group = dist.new_group(backend='gloo') if world > 1 else None
        self.dist = dist
        self.ends = None
        self.rounds = 0

    def chunk_window(self, w, entry):
        import torch
        off = entry - w.start
        src, n = self.buf.data_ptr() + off, w.end - entry
        tmp = None
        if src % 16:  # a fallback entry (rare): re-base the bytes on an aligned buffer
            tmp = torch.empty(n + 64, dtype=torch.uint8, device='cuda')
            tmp[:n].copy_(self.buf[off:off + n])
            src = tmp.data_ptr()
        _, caps = self.ch.capacity([n])
        cuts = self.cuts if int(caps[0]) <= self.cap else \
            torch.zeros(int(caps[0]), dtype=torch.int64, device='cuda')
        self.ch.chunk_device([src], [n], [max(0, w.last_piece - off) if not w.open else 0],
                             cuts.data_ptr(), self.counts.data_ptr(), self.hs, open_=w.open)
        c = int(self.counts.item())
        return (cuts[:c].cpu().numpy() + entry).tolist()

    def gather(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def step(self):
        from replicat_amd import split
        self.ends, self.rounds = split.chunk_split(self.chunk_window, self.windows, self.rank,
                                                   self.gather)


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
           '3ii': (1, 64 << 10, MIN_LEN, MAX_LEN), '3iii': (65536, 1, 2_000, 80_000),
           '4': (16, 8192, MIN_LEN, MAX_LEN), '5': (1024, 64, MIN_LEN, MAX_LEN)}[args.config]
    n = args.streams or cfg[0]
    size = (args.stream_mib or cfg[1]) << 20
    min_len, max_len = cfg[2], cfg[3]
    ch = GpuChunker(min_len, max_len, key, device=local)
    stream = torch.cuda.current_stream()
    hs = stream.cuda_stream
    last = None
    edit = long = None
    if args.config == '3ii':
        long = Config3ii(ch, size, rank, world, hs, dist)
        n, lens = 1, long.lens
        base_ptr = long.buf.data_ptr()
    else:
        # stream slots 64-B aligned; config 5's inserts grow a stream by up to 4 bytes
        slot = (size + (64 if args.config == '5' else 0) + 63) // 64 * 64
        pool = torch.empty(n * slot + 64, dtype=torch.uint8, device='cuda')  # one arena
        base_ptr = pool.data_ptr()
        ptrs = [base_ptr + i * slot for i in range(n)]
        for p, i in zip(ptrs, shard_ids(args.config, rank, n)):
            fill_splitmix(p, size, synth.DEFAULT_SEED, i, hs)
        lens = [size] * n
        if args.config == '5':
            # the original set is chunked once (untimed); the step re-chunks the edited set
            edit = Config5(ch, pool, slot, n, size, rank, hs)
            ptrs, lens = edit.ptrs, edit.lens
    total_cap, caps = ch.capacity(lens)
    cuts = torch.zeros(total_cap, dtype=torch.int64, device='cuda')
    counts = torch.zeros(n, dtype=torch.int64, device='cuda')
    torch.cuda.synchronize()

    def step():
        if long is not None:
            long.step()
        else:
            ch.chunk_device(ptrs, lens, last, cuts.data_ptr(), counts.data_ptr(), hs)

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

    bytes_per_step = sum(lens) if long is None else long.L // world
    value = world * bytes_per_step * args.steps / elapsed / GIB
    ms_per_step = elapsed * 1e3 / args.steps
    a_avg = a_ms / max(calls, 1)
    b_avg = b_ms / max(calls, 1)
    achieved = bytes_per_step / (a_avg * 1e-3) / 1e9  # GB/s, ΣL per tile-kernel launch

    parity = None
    ends = None
    if not args.no_verify and rank == 0:
        sys.path.insert(0, os.path.join(ROOT, 'tests'))
        import golden_util as G
        if long is not None:
            ends = [np.asarray(long.ends, dtype=np.uint64)]
            digest = G.cutlist_digest(ends)
        else:
            digest, nchunks, ends = cut_digest(cuts, counts, caps)
        gold = {d['name']: d for d in G.load('digests.json')}
        if args.key == 'ff' and n == 1024 and size == 64 << 20 and args.config == '2':
            parity = digest == gold['config2_ff']['sha256']
        elif args.key == 'ff' and args.config == '3iii' and n >= 4096:
            parity = G.cutlist_digest(ends[:4096]) == gold['config3iii_first4096']['sha256']
        elif args.key == 'ff' and long is not None and long.L == 64 << 30:
            large = {d['name']: d for d in G.load('large.json')}
            parity = digest == large['config3ii']['sha256']
        elif edit is not None and args.key == 'ff' and n == 1024 and size == 64 << 20:
            large = {d['name']: d for d in G.load('large.json')}
            dedup = edit.result = edit.dedup(ends)
            g5 = large['config5']
            parity = (G.cutlist_digest([ends[i] for i in edit.edited]) == g5['edited_sha256']
                      and edit.orig_digest == g5['original_sha256']
                      and dedup['dup_bytes_edited'] == g5['dup_bytes_edited']
                      and dedup['total_bytes_edited'] == g5['total_bytes_edited'])
    if world > 1:
        dist.barrier()

    if long is not None:
        workload = ('config3ii: ONE stream of %d GiB (last piece = final 1 MiB) split over %d '
                    'rank(s), min %d, max %d, key %s' % (long.L >> 30, world, min_len, max_len,
                                                         args.key))
    else:
        workload = ('config%s: %d x %d MiB streams per GPU, min %d, max %d, key %s'
                    % (args.config, n, size >> 20, min_len, max_len, args.key))
        if edit is not None:
            workload += ' (512 of the 1024 edited, re-chunk + dedup check)'
    traffic, traffic_src = pmc_traffic(args, n, size)
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
        if args.e2e and long is None:  # host-resident streams: copies in, chunking, cut offsets out
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
            probe = sum(lens) // 16 * 16
            for _ in range(2):
                read_probe(base_ptr, probe, out.data_ptr(), hs)
            ev0.record(stream)
            for _ in range(5):
                read_probe(base_ptr, probe, out.data_ptr(), hs)
            ev1.record(stream)
            torch.cuda.synchronize()
            calib = round(5 * probe / (ev0.elapsed_time(ev1) * 1e-3) / 1e9, 1)
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
            'config': {'workload': workload,
                       'streams_per_gpu': n, 'stream_bytes': size, 'parallelism': f'streams/{world} ranks'},
            'roofline': {'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4),
                         'traffic': None if traffic is None else round(traffic),
                         'traffic_source': traffic_src,
                         'algorithmic_bytes': bytes_per_step, 'kernel': 'rc_tile_kernel',
                         'kernel_ms': round(a_avg, 3), 'chain_kernel_ms': round(b_avg, 3)},
            'cpu_baseline': cpu,
            'parity_sha256': parity,
        }
        if edit is not None and getattr(edit, 'result', None) is not None:
            result['dedup'] = edit.result
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
