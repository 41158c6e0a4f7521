"""bench.py -- device-resident chunking throughput of the MI355X chunker (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY.md §8 d config 2): per GPU, 1024 synthetic
splitmix64 streams x 64 MiB (64 GiB resident in HBM), replicat's default chunk parameters
(min 128,000 / max 5,120,000), unencrypted key (0xff * 16), one piece per stream.
One step = one pass of the hot path over the whole batch: rc_chunk_device (tile kernel over
every needed byte + chain kernel per stream), cut offsets left in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3i|3ii|3iii|4|5|harness]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

`--gpus N` with N > 1 and no launcher around it (WORLD_SIZE unset) starts the N ranks itself:
a child `python -m torch.distributed.run --nproc-per-node N` over this same script, before
anything touches the GPU; bench.py exits with the child's status.  Every rank checks that the
world size equals --gpus and that the ranks hold N DISTINCT devices (PCI bus id / UUID
gathered into the line); ranks sharing a device exit non-zero unless --share-gpus is given (a
one-GPU rehearsal), and then the roofline is null (the ranks' HIP events time each other).

Ranks shard the work per stream (config 2: stream ids rank*1024 ..; config 4: stream i on
GPU i mod 8) with no data-path collective: "scaling": "weak".  The process group is gloo and
carries only the barriers, the max-over-ranks time and the parity flags -- never stream data.
Rank 0 prints one JSON line.  Parity is checked in-run by EVERY rank against the reference's
cut-list digests of that rank's own shard (tests/golden/ranks.json for ranks 0..7: config 2
with key ff and the seeded key's first 128 streams, 3 (iii), 5; config4.json; the harness;
3 (i) by its closed form; 3 (ii) for the stream lengths large.json / ranks.json hold); the
line's flag is the AND over ranks, null when any rank has no fixture.  The CPU baseline runs
on rank 0 over N x the per-GPU host-core share.

`--config harness` is the reference's own benchmark (Repository._benchmark_chunker,
/root/reference/replicat/repository.py:1984-2008): 10 x 512,000,000 Random(0) bytes as one
stream of 10 pieces, here chunked on the device in one call; its cpu_baseline is that harness
itself -- the reference's native chunker (oracle/_ref) under replicat's adapter loop.
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

# name -> (streams per GPU, MiB per stream, min_length, max_length)
CONFIGS = {'2': (1024, 64, MIN_LEN, MAX_LEN), '3i': (65536, 1, MIN_LEN, MAX_LEN),
           '3ii': (1, 64 << 10, MIN_LEN, MAX_LEN), '3iii': (65536, 1, 2_000, 80_000),
           '4': (16, 8192, MIN_LEN, MAX_LEN), '5': (1024, 64, MIN_LEN, MAX_LEN),
           'harness': (1, 0, MIN_LEN, MAX_LEN)}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=10)
    p.add_argument('--warmup', type=int, default=None,
                   help='untimed steps before the timed ones (default: 2; 50 for the harness '
                        'and 3 i, whose sub-millisecond steps would otherwise be timed while '
                        'the GPU is still ramping its clock after the host-side setup)')
    p.add_argument('--config', choices=sorted(CONFIGS), default='2',
                   help='2: 1024 x 64 MiB (the metric); 3i: 65536 x 1 MiB default params '
                        '(degenerate: tail rule only); 3ii: ONE 64 GiB stream, last piece the '
                        'final 1 MiB (snapshot framing, segment-parallel chain); 3iii: 65536 x '
                        '1 MiB, min 2000 / max 80000; 4: 16 x 8 GiB per GPU (streams rank, '
                        'rank+8, ...); 5: re-chunk of config 2 with 512 edited copies + dedup '
                        'ratio check; harness: the reference benchmark stream (10 x 512 MB)')
    p.add_argument('--streams', type=int, default=None)
    p.add_argument('--stream-mib', type=int, default=None)
    p.add_argument('--calibrate', action='store_true',
                   help='also time a pure streaming read of the same bytes (rc_read_probe)')
    p.add_argument('--min-length', type=int, default=None, help='override the config\'s min')
    p.add_argument('--max-length', type=int, default=None, help='override the config\'s max')
    p.add_argument('--key', choices=['ff', 'seeded'], default='ff')
    p.add_argument('--cpu-streams', type=int, default=None,
                   help='CPU-baseline sample in streams (default: all of config 2); 0 = skip')
    p.add_argument('--cpu-procs', type=int, default=None,
                   help='CPU-baseline processes (default: the cores this process may use)')
    p.add_argument('--e2e', action='store_true', help='also time the host-resident path')
    p.add_argument('--no-verify', action='store_true')
    p.add_argument('--pipeline', choices=['on', 'off'], default='on',
                   help='on: steps are RC_PIPELINED calls -- the tile kernel on all but '
                        '--reserve-cus CUs, edge + chain kernels on those, so one step\'s chain '
                        'runs beside the next step\'s tile kernel; off: every kernel of a step '
                        'on one stream, in sequence')
    p.add_argument('--reserve-cus', type=int, default=0,
                   help='CUs kept for the chain kernels in pipelined steps (0: the library '
                        'default)')
    p.add_argument('--share-gpus', action='store_true',
                   help='allow ranks to share a device (a rehearsal of the N-rank path on a '
                        'smaller box; the line then carries no roofline)')
    args = p.parse_args(argv)
    if args.warmup is None:
        # round 5 (profiles/r05/warmup/): the harness line after 2 warm-up steps (~2 ms of GPU
        # work after seconds of host-side data generation) ran its tile kernel at 0.857 ms,
        # after 50 at 0.792 and after 200 at 0.791 -- the clock ramp, not the kernel; config 2's
        # 9.3 ms steps (and its 64 GiB device fill) measure the same after 2, 10 or 30
        args.warmup = WARMUP_SHORT if args.config in ('harness', '3i') else 2
    return args


WARMUP_SHORT = 50  # warm-up steps of sub-millisecond configurations (parse)
WARM_MS = 100.0       # warm-up runs at least this long (main), whatever --warmup says
WARM_MAX_STEPS = 2000


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv, script=None):
    """Run the N ranks of `--gpus N` as one child `torch.distributed.run` over this script
    (one process per GPU; the driver's own N > 1 command has the same shape).  Nothing here
    touches the GPU -- the children initialise their devices themselves -- and the parent
    waits for the child instead of replacing itself.  Returns the child's exit status."""
    import subprocess
    script = os.path.abspath(script or sys.argv[0])
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           f'--nproc-per-node={args.gpus}', '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), script] + list(argv)
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return subprocess.call(cmd, env=env)


def cli(argv=None, backend=None, script=None):
    """The command line: N > 1 without a launcher starts the ranks; otherwise this process is
    one rank (or the only one).  Returns an exit status."""
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        return launch_ranks(args, argv, script)
    try:
        main(argv, backend=backend or Backend)
    except RankMismatch as e:
        print(f'bench.py: {e}', file=sys.stderr, flush=True)
        return 3
    return 0


class RankMismatch(RuntimeError):
    """The ranks do not match the request: world size != --gpus, or ranks sharing a device
    without --share-gpus."""


# ------------------------------------------------------------------ device plumbing

class Backend:
    """Everything bench.py does on a GPU: device selection, memory, synthetic fills, the chunker.
    tests/test_bench_ranks.py substitutes a CPU stand-in to run main() under gloo ranks."""

    device = 'cuda'

    def __init__(self, local_rank):
        import torch
        self.torch = torch
        # one GPU per local rank; with fewer visible devices than ranks they wrap round, and
        # main() refuses that (distinct physical devices checked) unless --share-gpus
        self.index = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(self.index)

    def use_own_stream(self):
        """Make every later bench op run on one non-blocking stream (main() calls this before
        it allocates anything): the legacy NULL stream would synchronise with the chunker's
        CU-masked streams (blocking streams) and serialise pipelined steps.  Not done in
        __init__: tests build a Backend inside their own stream context."""
        self.torch.cuda.set_stream(self.torch.cuda.Stream())

    def identity(self):
        """The physical device this rank runs on: ordinal, PCI location, UUID, name."""
        p = self.torch.cuda.get_device_properties(self.index)
        pci = '%04x:%02x:%02x' % (getattr(p, 'pci_domain_id', 0), getattr(p, 'pci_bus_id', 0),
                                  getattr(p, 'pci_device_id', 0))
        return {'device': self.index, 'pci': pci, 'uuid': str(getattr(p, 'uuid', '')),
                'name': p.name, 'visible': os.environ.get('HIP_VISIBLE_DEVICES')
                or os.environ.get('ROCR_VISIBLE_DEVICES') or os.environ.get('CUDA_VISIBLE_DEVICES')}

    def empty(self, nbytes):
        return self.torch.empty(nbytes, dtype=self.torch.uint8, device=self.device)

    def zeros_i64(self, n):
        return self.torch.zeros(max(n, 1), dtype=self.torch.int64, device=self.device)

    def stream(self):
        return self.torch.cuda.current_stream().cuda_stream

    def synchronize(self):
        self.torch.cuda.synchronize()

    def chunker(self, min_len, max_len, key):
        from replicat_amd.chunker import GpuChunker
        return GpuChunker(min_len, max_len, key, device=self.index)

    def fill_streams(self, ptr, n, size, slot, seed, first_id, id_step):
        from replicat_amd.chunker import fill_splitmix_streams
        fill_splitmix_streams(ptr, n, size, slot, seed, first_id, id_step, self.stream())

    def fill_at(self, ptr, nbytes, seed, stream_id, word0):
        from replicat_amd.chunker import fill_splitmix_at
        fill_splitmix_at(ptr, nbytes, seed, stream_id, word0, self.stream())

    def upload(self, dst_tensor, host_bytes):
        dst_tensor[:len(host_bytes)].copy_(self.torch.frombuffer(host_bytes, dtype=self.torch.uint8))

    def read_probe_gbs(self, ptr, nbytes):
        from replicat_amd.chunker import read_probe
        torch = self.torch
        out = torch.zeros(4, dtype=torch.int32, device=self.device)
        st = torch.cuda.current_stream()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        probe = nbytes // 16 * 16
        for _ in range(2):
            read_probe(ptr, probe, out.data_ptr(), self.stream())
        ev0.record(st)
        for _ in range(5):
            read_probe(ptr, probe, out.data_ptr(), self.stream())
        ev1.record(st)
        torch.cuda.synchronize()
        return round(5 * probe / (ev0.elapsed_time(ev1) * 1e-3) / 1e9, 1)


class Ranks:
    """The process group of a multi-GPU run: gloo (host) only.  The data path has no exchange;
    this carries the start/stop barriers, the max-over-ranks time and small host objects."""

    def __init__(self):
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        self.local = int(os.environ.get('LOCAL_RANK', str(self.rank)))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group('gloo')
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, values):
        if not self.dist:
            return list(values)
        import torch
        t = torch.tensor(values, dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return t.tolist()

    def gather(self, obj):
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist and self.dist.is_initialized():
            self.dist.destroy_process_group()


def shard_ids(config, rank, n):
    """Stream ids a rank chunks (weak scaling: every rank has its own n streams).  Config 4
    follows the north star's round-robin: stream i lives on GPU i mod 8."""
    if config == '4':
        return [rank + 8 * i for i in range(n)]
    return [rank * n + i for i in range(n)]


def cut_digest(cuts_dev, counts_dev, caps):
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import golden_util as G
    from replicat_amd.chunker import check_counts
    cuts = cuts_dev.cpu().numpy().view(np.uint64)
    counts = counts_dev.cpu().numpy()[:len(caps)]
    check_counts(counts)  # a fail-safe stop (RC_COUNT_FAULT) or an overflow raises
    base = np.concatenate([[0], np.cumsum(caps)[:-1]]).astype(np.int64)
    ends = [cuts[b:b + c] for b, c in zip(base, counts)]
    return G.cutlist_digest(ends), int(counts.sum()), ends


def bytes_needed(max_length, lens, last):
    """Bytes the tile kernel must read: per stream, bytes [0, 4 jneed + 4) with jneed the last
    key any argmax window reaches (rc_keys_needed; 0 = tail rule only, nothing read)."""
    from replicat_amd.chunker import keys_needed
    memo, total = {}, 0
    for L, P in zip(lens, last if last is not None else [0] * len(lens)):
        k = (int(L), int(P))
        if k not in memo:
            j = keys_needed(max_length, k[0], k[1])
            memo[k] = min(k[0], 4 * j + 4) if j else 0
        total += memo[k]
    return total


# ------------------------------------------------------------------------ CPU baseline

def cpu_share(world=1):
    """(cores to use, cores in the affinity mask): the mask, capped by the CPU share the node
    grants the line's GPUs -- OMP_NUM_THREADS per GPU there (nproc and the mask show the whole
    machine), times the ranks, so an N-GPU line is set against N GPUs' host cores."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get('OMP_NUM_THREADS')
    if cap and cap.isdigit() and int(cap) > 0:
        return min(n, int(cap) * max(1, world)), n
    return n, n


def _ref_chunker(min_len, max_len, key):
    """The reference's own chunker, compiled from /root/reference/src/adapters.cpp into
    oracle/_ref by oracle/Makefile (built in the build container, shipped with the tree)."""
    import glob
    import importlib.machinery
    import importlib.util
    so = glob.glob(os.path.join(ROOT, 'oracle', '_ref', '_replicat_adapters*.so'))
    if not so:
        return None
    loader = importlib.machinery.ExtensionFileLoader('_replicat_adapters', so[0])
    spec = importlib.util.spec_from_loader('_replicat_adapters', loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod._gclmulchunker(min_len, max_len, key)


def _stream(size, seed, sid):
    from oracle import oracle as o
    return o.fill_splitmix(size, seed, sid)


def _scan_worker(args):
    """Native next_cut scan (the reference's, else the oracle port) over whole streams, on a
    zero-copy view: exactly the adapter's calls for a single piece (adapters.py:290-305)."""
    kind, ids, size, seed, min_len, max_len = args
    from oracle import oracle as o
    ref = _ref_chunker(min_len, max_len, b'\xff' * 16) if kind == 'reference' else None
    t, out = 0.0, []
    for i in ids:
        data = _stream(size, seed, i)
        t0 = time.perf_counter()
        if ref is not None:
            mv, pos, ends = memoryview(data), 0, []
            while pos < size:
                c = ref.next_cut(mv[pos:], True)
                if not c:
                    break
                pos += c
                ends.append(pos)
        else:
            ends = o.chunk_stream(data, min_len, max_len, None, 0)
        t += time.perf_counter() - t0
        out.append((i, ends))
    return t, out


def _adapter_worker(args):
    """replicat's adapter loop (oracle/adapter_loop.py) over the reference's native chunker,
    fed 16 MiB pieces as Repository.snapshot reads files (repository.py:1413,1440)."""
    ids, size, seed, min_len, max_len = args
    from oracle.adapter_loop import adapter_chunks
    t = 0.0
    for i in ids:
        data = _stream(size, seed, i)
        pieces = [data[k:k + (16 << 20)].tobytes() for k in range(0, size, 16 << 20)]
        ref = _ref_chunker(min_len, max_len, b'\xff' * 16)
        t0 = time.perf_counter()
        n = sum(len(c) for c in adapter_chunks(ref, pieces))
        t += time.perf_counter() - t0
        assert n == size
    return t


def _pool_map(fn, jobs):
    import multiprocessing as mp
    with mp.get_context('fork').Pool(len(jobs)) as pool:
        return pool.map(fn, jobs)


def cpu_baseline(n_streams, size, seed, procs, min_len=MIN_LEN, max_len=MAX_LEN, extras=True):
    """the reference's native scan on the box's host cores, one process per
    core, over `n_streams` of the same synthetic streams; the adapter-loop rate beside it; and
    the speed ratio of the reference build to the oracle port on the same sample."""
    import glob
    from oracle import oracle as o
    o.lib()
    kind = 'reference' if glob.glob(os.path.join(ROOT, 'oracle', '_ref', '_replicat_adapters*.so')) \
        else 'port'
    procs = max(1, min(procs, n_streams))
    shards = [list(range(r, n_streams, procs)) for r in range(procs)]
    t0 = time.perf_counter()
    res = _pool_map(_scan_worker, [(kind, s, size, seed, min_len, max_len) for s in shards])
    wall = time.perf_counter() - t0
    busiest = max(r[0] for r in res)  # scan time of the slowest process (generation excluded)
    ends = {i: e for _, out in res for i, e in out}
    out = {'value': round(n_streams * size / busiest / GIB, 3), 'unit': 'GiB/s', 'cores': procs,
           'kind': kind,
           'sample': f'{n_streams} x {size >> 20} MiB of the same synthetic streams (ids '
                     f'0..{n_streams - 1}), one process per core, native next_cut scan time of '
                     f'the slowest process ({busiest:.2f} s; {wall:.1f} s wall incl. data '
                     f'generation)'}
    if kind == 'reference' and extras:
        # the adapter loop: one stream per core (16 MiB pieces), and the reference-vs-port
        # time ratio on two streams in this process
        k = min(procs, n_streams)
        ta = max(_pool_map(_adapter_worker, [([i], size, seed, min_len, max_len) for i in range(k)]))
        out['adapter_loop'] = {'value': round(k * size / ta / GIB, 3), 'unit': 'GiB/s',
                               'cores': k, 'sample': f'{k} x {size >> 20} MiB in 16 MiB pieces '
                               f'through adapters.py:290-305 (restated, oracle/adapter_loop.py)'}
        tr, _ = _scan_worker(('reference', [0, 1], size, seed, min_len, max_len))
        tp, _ = _scan_worker(('port', [0, 1], size, seed, min_len, max_len))
        out['reference_time_over_port_time'] = round(tr / tp, 3)
    return out, ends


def harness_cpu(pieces, min_len, max_len):
    """The reference harness itself on one host core: its native chunker under replicat's adapter
    loop over the 10 pre-built pieces (generation outside the clock, as repository.py:2001-2003)."""
    from oracle.adapter_loop import harness_rate
    ref = _ref_chunker(min_len, max_len, b'\xff' * 16)
    if ref is None:
        return None, None
    nbytes, secs, lengths = harness_rate(ref, pieces)
    return ({'value': round(nbytes / secs / GIB, 3), 'unit': 'GiB/s', 'cores': 1,
             'kind': 'reference', 'rate_GBps': round(nbytes / secs / 1e9, 3),
             'sample': f'the whole harness stream ({nbytes} B, 10 pieces) through the adapter '
                       f'loop, {secs:.2f} s, generation excluded (repository.py:1984-2008)'},
            lengths)


# ---------------------------------------------------------------- PMC traffic (profiles/)

def workload_key(args, n, size, custom, long):
    """The profiles/ name of a line's workload (one rocprofv3 PMC entry per BASELINE line), or
    None for a workload without one (custom sizes or parameters; 3 (i) reads nothing)."""
    if custom or args.streams is not None or args.stream_mib is not None:
        return None
    if args.config == '2':
        return 'config2' if args.key == 'ff' else 'config2_seeded'
    if args.key != 'ff':
        return None
    return {'3ii': 'config3ii' if long is not None and long.world == 1 else None,
            '3iii': 'config3iii', '4': 'config4', '5': 'config5',
            'harness': 'harness'}.get(args.config)


def pmc_traffic(workload, build_id):
    """HBM bytes per rc_tile_kernel launch from the committed rocprofv3 PMC summary of this same
    workload (scripts/gpu_pmc_all.sh -> scripts/summarize_profile.py: separate --pmc passes,
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM, WRITE_SIZE as is).  Only a summary of the
    SAME library build counts: it is stamped with rc_build_id(), and a stale one is refused.
    bench.py cannot read counters itself (that needs rocprofv3)."""
    if workload is None:
        return None, 'no PMC summary for this workload'
    import glob
    stale = None
    for f in sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*', 'pmc_summary.json')),
                    reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if workload in d.get('workloads', {}):
            t = d['workloads'][workload].get('rc_tile_kernel', {})
        elif d.get('workload') == workload:  # the round-4 layout (config 2 only)
            t = d.get('rc_tile_kernel', {})
        else:
            continue
        if 'hbm_read_bytes_corrected' not in t:
            continue
        if d.get('build_id') != build_id:
            stale = stale or f'{os.path.relpath(f, ROOT)} is of build {d.get("build_id")}, not {build_id}'
            continue
        PROFILE.clear()
        if t.get('steady_avg_ns'):
            PROFILE.update(steady_ns=t['steady_avg_ns'], median_ns=t.get('median_ns'),
                           launches=t.get('launches'))
        return (t['hbm_read_bytes_corrected'] + t.get('hbm_write_bytes', 0.0),
                os.path.relpath(f, ROOT) + f' [{workload}]')
    return None, stale or f'no PMC summary of {workload} under profiles/'


PROFILE = {}  # the tile kernel's launch times in the PMC summary pmc_traffic() accepted


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

    def __init__(self, ch, pool, slot, n, size, rank, hs, device='cuda'):
        import torch
        from replicat_amd import synth
        self.size, self.slot, self.n = size, slot, n
        self.orig = pool
        base = pool.data_ptr()
        olens = [size] * n
        cap, ocaps = ch.capacity(olens)
        ocuts = torch.zeros(cap, dtype=torch.int64, device=device)
        ocounts = torch.zeros(n, dtype=torch.int64, device=device)
        ch.chunk_device([base + i * slot for i in range(n)], olens, None, ocuts.data_ptr(),
                        ocounts.data_ptr(), hs)
        self.orig_digest, _, self.orig_ends = cut_digest(ocuts, ocounts, ocaps)
        # every rank edits its own shard: rank 0 the single-GPU plan (seed 5), rank r seed 5 + r
        # (tests/golden/make_golden.py rank_edit_plan; ranks.json holds each rank's reference)
        plan = synth.edit_plan(n, n // 2, size, seed=5 + rank) if n == 1024 else []
        self.plan = {sid: (kind, off, payload) for sid, kind, off, payload in plan}
        self.edited = sorted(self.plan)
        self.buf = torch.empty(n * slot + 64, dtype=torch.uint8, device=device)
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

    def __init__(self, ch, size, ranks, be, pipelined=False):
        from replicat_amd import split, synth
        self.ch, self.ranks, self.be = ch, ranks, be
        self.pipelined = pipelined
        self.rank, self.world = ranks.rank, ranks.world
        self.hs = be.stream()
        self.L = size * self.world
        self.P = self.L - (1 << 20)
        self.windows = split.plan_windows(self.L, self.P, self.world, ch.max_length)
        w = self.windows[self.rank]
        self.w = w
        self.buf = be.empty(w.end - w.start + 64)
        be.fill_at(self.buf.data_ptr(), w.end - w.start, synth.DEFAULT_SEED, 0, w.start // 8)
        self.lens = [w.end - w.start]
        _, caps = ch.capacity(self.lens)
        self.cap = int(caps[0])
        self.cuts = be.zeros_i64(self.cap + 1)
        self.counts = be.zeros_i64(1)
        self.ends = None
        self.rounds = 0

    def enqueue(self, w, entry, pipelined=False, last=False):
        """Chunk window w from ``entry`` on the device (cut ends relative to entry in
        self.cuts / the returned tensor); enqueue only (pipelined: ch.wait orders the outputs)."""
        off = entry - w.start
        src, n = self.buf.data_ptr() + off, w.end - entry
        tmp = None
        if src % 16:  # a fallback entry (rare): re-base the bytes on an aligned buffer
            tmp = self.be.empty(n + 64)
            tmp[:n].copy_(self.buf[off:off + n])
            src = tmp.data_ptr()
        _, caps = self.ch.capacity([n])
        cuts = self.cuts if int(caps[0]) <= self.cap else self.be.zeros_i64(int(caps[0]))
        self.ch.chunk_device([src], [n], [max(0, w.last_piece - off) if not w.open else 0],
                             cuts.data_ptr(), self.counts.data_ptr(), self.hs, open_=w.open,
                             pipelined=pipelined, end=last)
        self._tmp = tmp
        return cuts

    def count(self):
        from replicat_amd.chunker import counts_host
        return int(counts_host(self.counts)[0])

    def chunk_window(self, w, entry):
        """The whole cut list of window w from ``entry``, absolute, on the host."""
        cuts = self.enqueue(w, entry)
        c = self.count()
        return (cuts[:c].cpu().numpy() + entry).tolist()

    EXCHANGE = 64  # cut ends of each window's head and tail in the compact exchange

    def step(self, last=False):
        """One GPU: the stream is chunked on the device and its cuts stay there.  Several: each
        rank chunks its window, and the ranks exchange only the first and last EXCHANGE cuts of
        their chains (a host gather of a few KB) to find where the true chain meets each
        window's speculative one -- the whole lists only when that fails (split.chunk_split)."""
        from replicat_amd import split
        self.ends, self._bounds = None, None
        # one rank: steps pipeline (nothing is read back between them); several: each step
        # reads its window's head and tail back, so its calls run in sequence
        cuts = self.enqueue(self.w, self.w.start, pipelined=self.pipelined and self.world == 1,
                            last=last)
        self._cuts = cuts
        if self.world == 1:
            return
        c = self.count()
        k = self.EXCHANGE
        head = (cuts[:min(c, k)].cpu().numpy() + self.w.start).tolist()
        tail = (cuts[max(0, c - k):c].cpu().numpy() + self.w.start).tolist()
        bounds = split.merge_points(self.windows, self.ranks.gather((self.w.start, head, tail)))
        if bounds is None:
            self.ends, self.rounds = split.chunk_split(self.chunk_window, self.windows, self.rank,
                                                       self.ranks.gather)
            return
        self._bounds = bounds

    def finish(self):
        """The whole true cut list on every rank (parity; outside the timed region)."""
        if self.ends is not None:
            return
        c = self.count()
        mine = (self._cuts[:c].cpu().numpy() + self.w.start).tolist()
        if self.world == 1:
            self.ends = mine
            return
        lo = self._bounds[self.rank]
        hi = self._bounds[self.rank + 1] if self.rank + 1 < self.world else None
        part = [p for p in mine if p > lo and (hi is None or p <= hi)]
        self.ends = [p for prt in self.ranks.gather(part) for p in prt]


# ------------------------------------------------------------------------------ main

def _golden():
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import golden_util as G
    return G


def check_parity(args, n, size, rank, long, edit, ends, digest):
    """(flag, scope) of THIS rank's cut lists against the reference's digests of this rank's
    own shard (tests/golden/ranks.json: every rank of an up-to-8-GPU line; rank 0's entries are
    the single-GPU fixtures), or (None, None) when no fixture covers the workload.  main() ANDs
    the ranks' flags into the line's (null when any rank has none)."""
    cfg = CONFIGS[args.config]
    if (args.min_length not in (None, cfg[2])) or (args.max_length not in (None, cfg[3])):
        return None, None  # every fixture is of the config's own chunk parameters
    G = _golden()
    R = G.load('ranks.json')
    ff = args.key == 'ff'
    mine = rank < R['ranks']
    c2 = size == 64 << 20 and n == 1024
    if args.config == '2' and ff and c2 and mine:
        g = R['config2_ff'][rank]
        return digest == g['sha256'], f'streams {g["first_id"]}..{g["first_id"] + n - 1}'
    small = R.get('small')
    if args.config == '2' and ff and mine and small and (n, size) == (small['streams'], small['size']):
        # a small config-2-shaped shard (the CPU tests' stand-in checks every rank against it)
        g = small['per_rank'][rank]
        return digest == g['sha256'], f'streams {g["first_id"]}..{g["first_id"] + n - 1}'
    if args.config == '2' and not ff and c2 and mine:
        # an encrypted repository's key (repository.py:174-181): the reference cut the first
        # 128 streams of every shard with synth.seeded_key(1) (tests/golden/make_golden.py)
        g = R['config2_seeded'][rank]
        from replicat_amd import synth
        assert synth.seeded_key(1).hex() == g['params']
        k = g['streams']
        return (G.cutlist_digest(ends[:k]) == g['sha256'],
                f'seeded key: streams {g["first_id"]}..{g["first_id"] + k - 1}')
    if args.config == '3iii' and ff and n == 65536 and mine:
        g = R['config3iii'][rank]
        return digest == g['sha256'], f'all 65536 streams ({g["first_id"]}..)'
    if args.config == '3iii' and ff and rank == 0 and n >= 4096:
        gold = {d['name']: d for d in G.load('digests.json')}
        return (G.cutlist_digest(ends[:4096]) == gold['config3iii_first4096']['sha256'],
                'first 4096 streams')
    if args.config == '3i' and ff:
        # the tail rule alone: one chunk per stream (adapters.cpp:50-51)
        return all(len(e) == 1 and int(e[0]) == size for e in ends), 'every stream'
    if long is not None and ff:
        # one stream split over the ranks: every rank holds the whole spliced list
        for g in [d for d in G.load('large.json') if d['name'] == 'config3ii'] + R.get('config3ii', []):
            if long.L == g['size'] and long.P == g['last_piece']:
                return digest == g['sha256'], f'the whole {long.L >> 30} GiB stream'
        return None, None
    if args.config == '4' and ff and n == 16 and size == 8 << 30 and rank < 8:
        c4 = G.load('config4.json')
        return digest == c4['per_gpu'][rank]['sha256'], 'streams r, r + 8, ..'
    if args.config == 'harness':
        return digest == G.load('harness.json')['sha256'], 'the whole harness stream'
    if edit is not None and ff and c2 and mine:
        dedup = edit.result = edit.dedup(ends)
        g5 = R['config5'][rank]
        return ((G.cutlist_digest([ends[i] for i in edit.edited]) == g5['edited_sha256']
                 and edit.orig_digest == g5['original_sha256']
                 and dedup['dup_bytes_edited'] == g5['dup_bytes_edited']
                 and dedup['total_bytes_edited'] == g5['total_bytes_edited']),
                f'{len(edit.edited)} edited streams of the shard + dedup')
    return None, None


def line_parity(per_rank, world):
    """The line's flag: the AND over every rank's own check, null when any rank has no fixture
    (a line whose cut lists were not all compared must not read true)."""
    flags = [r['parity'] for r in per_rank]
    if len(flags) == 1:
        return flags[0], per_rank[0]['parity_scope']
    if any(f is None for f in flags):
        unchecked = [r['rank'] for r in per_rank if r['parity'] is None]
        return None, f'no fixture for rank(s) {unchecked}'
    return all(flags), f'every rank ({world}) against its own shard: ' + '; '.join(
        f'rank {r["rank"]}: {r["parity_scope"]}' for r in per_rank)


def roofline(bytes_per_step, read, tile_avg, edge_avg, chain_avg, traffic, traffic_src, bid):
    """The tile kernel against the HBM read peak, on two bases: the stream bytes a launch
    covers (SURVEY §8 d's algorithmic bytes) and the bytes it must read (up to each stream's
    last needed key -- the tail rule's last ~max_length bytes are never read).  Null when the
    kernel reads nothing or the figure would pass the peak (then it is not a measurement)."""
    r = {'bound': 'hbm', 'kernel': 'rc_tile_kernel', 'unit': 'GB/s', 'peak': HBM_PEAK_GBS,
         'kernel_ms': round(tile_avg, 3), 'edge_kernel_ms': round(edge_avg, 3),
         'chain_kernel_ms': round(chain_avg, 3), 'algorithmic_bytes': bytes_per_step,
         'bytes_read': read, 'traffic': None if traffic is None else round(traffic),
         'traffic_source': traffic_src, 'build_id': bid,
         'basis': 'stream bytes per tile-kernel launch (SURVEY §8 d)',
         'basis_read': "bytes the tile kernel must read (to each stream's last needed key)"}
    ok = read > 0 and tile_avg > 0
    achieved = bytes_per_step / (tile_avg * 1e-3) / 1e9 if ok else None
    achieved_read = read / (tile_avg * 1e-3) / 1e9 if ok else None
    if ok and achieved_read > HBM_PEAK_GBS:
        ok = False
    r.update({'achieved': round(achieved, 1) if ok else None,
              'frac': round(achieved / HBM_PEAK_GBS, 4) if ok else None,
              'achieved_read': round(achieved_read, 1) if ok else None,
              'frac_read': round(achieved_read / HBM_PEAK_GBS, 4) if ok else None})
    if not ok:
        r['note'] = ('no key is hashed: every stream is cut by the tail rule alone '
                     '(adapters.cpp:48-55); no roofline') if read == 0 else 'not a measurement'
    # round 6: the same roofline from the committed rocprofv3 trace of this
    # build and workload (steady state: its first, cold launch dropped), beside the HIP-event one
    if ok and traffic_src and PROFILE.get('steady_ns'):
        pf = bytes_per_step / PROFILE['steady_ns'] / HBM_PEAK_GBS
        r.update({'profile_kernel_ms': round(PROFILE['steady_ns'] * 1e-6, 3),
                  'profile_frac': round(pf, 4),
                  'profile_frac_median': round(bytes_per_step / PROFILE['median_ns'] / HBM_PEAK_GBS, 4)
                  if PROFILE.get('median_ns') else None,
                  'profile_source': traffic_src.split(' [')[0] + ' (kernel trace, '
                  f'{PROFILE.get("launches")} launches, first dropped)',
                  'profile_vs_line': round(pf / r['frac'], 4)})
        if abs(pf / r['frac'] - 1) > 0.03:
            r['profile_note'] = ('the profiled process ran on another allocation (or box): '
                                 'HBM placement moves the tile kernel by up to ~5 % between '
                                 'allocations (DESIGN.md §4, placement), the profiler also '
                                 'serialises the pipelined kernels')
    return r


LAST = {}  # the last main() call's cut lists, device and parity (tests/test_bench_ranks.py)


def check_ranks(args, ranks, be):
    """Each rank's device, gathered; RankMismatch (every rank raises it alike) when the world
    is not --gpus ranks or, without --share-gpus, when two ranks hold the same device.
    Returns (identities, shared)."""
    if ranks.world != args.gpus:
        ranks.close()
        raise RankMismatch(f'{ranks.world} rank(s) running but --gpus {args.gpus} requested')
    ids = ranks.gather(dict(be.identity(), rank=ranks.rank))
    keys = [i.get('uuid') or i.get('pci') for i in ids]
    shared = len(set(keys)) < len(keys)
    if shared and not args.share_gpus:
        ranks.close()
        raise RankMismatch(f'{len(keys)} ranks on {len(set(keys))} distinct device(s) '
                           f'({", ".join(i["pci"] for i in ids)}); --share-gpus to rehearse')
    return ids, shared


def main(argv=None, backend=Backend):
    args = parse(argv)
    ranks = Ranks()
    world, rank = ranks.world, ranks.rank
    be = backend(ranks.local)
    if hasattr(be, 'use_own_stream'):
        be.use_own_stream()
    devices, shared = check_ranks(args, ranks, be)

    from replicat_amd import synth
    key = b'\xff' * 16 if args.key == 'ff' else synth.seeded_key(1)
    cfg = CONFIGS[args.config]
    n = args.streams or cfg[0]
    size = (args.stream_mib or cfg[1]) << 20
    min_len = cfg[2] if args.min_length is None else args.min_length
    max_len = cfg[3] if args.max_length is None else args.max_length
    custom = (min_len, max_len) != (cfg[2], cfg[3])
    ch = be.chunker(min_len, max_len, key)
    hs = be.stream()
    pipelined = args.pipeline == 'on'
    if pipelined and args.reserve_cus:
        ch.overlap(args.reserve_cus)  # otherwise the library's default, set up at the first call
    last = None
    edit = long = harness = None
    if args.config == '3ii':
        long = Config3ii(ch, size, ranks, be, pipelined)
        n, lens = 1, long.lens
        base_ptr = long.buf.data_ptr()
        last = [long.w.last_piece if not long.w.open else 0]
    elif args.config == 'harness':
        # the reference benchmark's stream, generated on the host as the reference does, copied
        # in once; the timed step chunks it on the device
        harness = list(synth.harness_buffers())
        L = sum(len(b) for b in harness)
        pool = be.empty(L + 64)
        off = 0
        for b in harness:
            be.upload(pool[off:], b)
            off += len(b)
        n, size, lens, last = 1, L, [L], [L - len(harness[-1])]
        base_ptr = pool.data_ptr()
        ptrs = [base_ptr]
    else:
        # stream slots 64-B aligned; config 5's inserts grow a stream by up to 4 bytes
        slot = (size + (64 if args.config == '5' else 0) + 63) // 64 * 64
        pool = be.empty(n * slot + 64)  # one arena
        base_ptr = pool.data_ptr()
        ptrs = [base_ptr + i * slot for i in range(n)]
        ids = shard_ids(args.config, rank, n)
        be.fill_streams(base_ptr, n, size, slot, synth.DEFAULT_SEED, ids[0],
                        ids[1] - ids[0] if n > 1 else 1)
        lens = [size] * n
        if args.config == '5':
            # the original set is chunked once (untimed); the step re-chunks the edited set
            edit = Config5(ch, pool, slot, n, size, rank, hs, be.device)
            ptrs, lens = edit.ptrs, edit.lens
    total_cap, caps = ch.capacity(lens)
    cuts = be.zeros_i64(total_cap)
    counts = be.zeros_i64(n)
    be.synchronize()
    # the stream arrays as the C ABI takes them (u64), built once: converting 65,536-entry
    # Python lists on every call is host time the device would wait for
    if long is None:
        ptrs_a = np.ascontiguousarray(ptrs, dtype=np.uint64)
        lens_a = np.ascontiguousarray(lens, dtype=np.uint64)
        last_a = np.ascontiguousarray(last if last is not None else np.zeros(n), dtype=np.uint64)

    def step(pipe=pipelined, end=False):
        # end: the last step of a pipelined run, whose chain has no tile kernel to hide behind
        # (RC_PIPELINE_END: it runs on every CU)
        if long is not None:
            if pipe == pipelined:
                long.step(last=end)
            else:
                long.enqueue(long.w, long.w.start, pipelined=pipe)
        else:
            ch.chunk_device(ptrs_a, lens_a, last_a, cuts.data_ptr(), counts.data_ptr(), hs,
                            pipelined=pipe, end=end)

    # warm-up: the requested steps, then more until the warm-up has kept the device busy for
    # WARM_MS (round 6): the clock ramps over the first ~30-40 ms of work,
    # which 2 sub-millisecond steps do not cover (profiles/r05/warmup/: the harness 0.857 ms per
    # tile kernel after 2 steps, 0.792 after 50); every rank runs the same number of steps (the
    # split line's steps exchange cuts), decided on the slowest rank's time
    warm_steps, warm_s, tw = 0, 0.0, time.perf_counter()
    batch = args.warmup
    while batch > 0:
        for i in range(batch):
            step(end=i == batch - 1)
        warm_steps += batch
        ch.wait(hs)
        be.synchronize()
        warm_s = ranks.max([time.perf_counter() - tw])[0]
        batch = 0 if warm_s * 1e3 >= WARM_MS or warm_steps >= WARM_MAX_STEPS else \
            min(max(8, warm_steps), WARM_MAX_STEPS - warm_steps)
    ch.wait(hs)
    be.synchronize()
    ranks.barrier()
    be.synchronize()
    ch.timing(True)
    piped0 = ch.pipelined_calls()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(end=i == args.steps - 1)
    ch.wait(hs)  # the outputs of every step (pipelined steps leave hs free)
    be.synchronize()
    ranks.barrier()
    be.synchronize()
    elapsed = time.perf_counter() - t0
    piped = ch.pipelined_calls() - piped0
    reserve = ch.overlap_cus() if pipelined else 0
    ch.timing(False)
    # every call so far (warm-up and timed): a tile kernel's fail-safe stop raises ChunkerFault
    # here, so the line is never printed over cuts that are not the reference's
    ch.check()
    tile_ms, edge_ms, chain_ms, calls = ch.read_kernel_timing()
    mine = {'rank': rank, 'elapsed_s': round(elapsed, 6),
            'tile_kernel_ms': round(tile_ms / max(calls, 1), 3)}
    elapsed, tile_ms, edge_ms, chain_ms = ranks.max([elapsed, tile_ms, edge_ms, chain_ms])

    bytes_per_step = sum(lens) if long is None else long.L // world
    value = world * bytes_per_step * args.steps / elapsed / GIB
    ms_per_step = elapsed * 1e3 / args.steps
    calls = max(calls, 1)

    parity, ends, scope = None, None, None
    if not args.no_verify:
        if long is not None:
            long.finish()
            ends = [np.asarray(long.ends, dtype=np.uint64)]
            digest = _golden().cutlist_digest(ends)
        else:
            digest, _, ends = cut_digest(cuts, counts, caps)
        if not custom:
            parity, scope = check_parity(args, n, size, rank, long, edit, ends, digest)
    LAST.update(device=be.index, ends=ends, parity=parity, rank=rank)
    # the same step unpipelined (every kernel on one stream in sequence), after the timed
    # region: what one call takes from its first kernel to its cuts
    seq_ms = None
    if pipelined and (long is None or world == 1):
        seq = max(1, min(3, args.steps))
        step(False)
        be.synchronize()
        t1 = time.perf_counter()
        for _ in range(seq):
            step(False)
        be.synchronize()
        seq_ms = (time.perf_counter() - t1) * 1e3 / seq
    mine['parity'] = parity
    mine['parity_scope'] = scope
    per_rank = ranks.gather(mine)
    parity, scope = line_parity(per_rank, world)
    for r, d in zip(per_rank, devices):
        r.update(device=d['device'], pci=d['pci'], uuid=d['uuid'])

    result = None
    if rank == 0:
        from replicat_amd.chunker import build_id
        bid = build_id()
        traffic, traffic_src = pmc_traffic(workload_key(args, n, size, custom, long), bid)
        roof = roofline(bytes_per_step, bytes_needed(max_len, lens, last), tile_ms / calls,
                        edge_ms / calls, chain_ms / calls, traffic, traffic_src, bid)
        if piped:
            roof['timing_note'] = (
                'pipelined steps: kernel_ms is the tile kernel on its CU-masked stream; '
                'edge_kernel_ms and chain_kernel_ms run on the reserved CUs beside the next '
                "step's tile kernel and span from the tile kernel's end (waits included)")
        if shared:
            # ranks on one device: each rank's HIP events also time the other ranks' kernels
            roof.update(achieved=None, frac=None, achieved_read=None, frac_read=None,
                        note='ranks share a device (--share-gpus): kernel times overlap, '
                             'no roofline')
        cpu = None
        # the CPU leg runs on rank 0 after the timed region, at every N (the other ranks wait
        # at the final barrier); its sample is rank 0's own streams
        if args.key == 'ff' and args.config == '2' and args.cpu_streams != 0:
            procs, seen = cpu_share(world)
            procs = args.cpu_procs or procs
            sample = min(args.cpu_streams or n, n)
            cpu, cpu_ends = cpu_baseline(sample, size, synth.DEFAULT_SEED, procs)
            cpu['affinity_cores'] = seen
            cpu['cores_basis'] = (
                f'{procs} = min(affinity mask {seen}, {world} GPU(s) x OMP_NUM_THREADS '
                f'{os.environ.get("OMP_NUM_THREADS")}) -- the host-core share the node grants '
                f'the line\'s GPUs (OMP_NUM_THREADS per GPU; nproc and the mask show the whole '
                f"machine); --cpu-procs overrides" if os.environ.get('OMP_NUM_THREADS')
                else f'{procs} = the affinity mask')
            if ends is not None:
                cpu['matches_gpu'] = bool(all(np.array_equal(np.asarray(cpu_ends[i], np.uint64),
                                                             ends[i]) for i in cpu_ends))
            if seen > procs and not args.cpu_procs:
                # beside the per-GPU share: the same scan on EVERY core of the affinity mask
                # (the box's whole host; value stays the share)
                whole, whole_ends = cpu_baseline(sample, size, synth.DEFAULT_SEED, seen,
                                                 extras=False)
                cpu['whole_mask'] = {k: whole[k] for k in ('value', 'unit', 'cores', 'kind',
                                                           'sample')}
                cpu['whole_mask']['matches_share'] = all(
                    list(whole_ends[i]) == list(cpu_ends[i]) for i in cpu_ends)
        elif harness is not None and args.cpu_streams != 0:
            cpu, lengths = harness_cpu(harness, min_len, max_len)
            if cpu is not None and ends is not None:
                cpu['matches_gpu'] = bool(np.array_equal(np.cumsum(lengths).astype(np.uint64),
                                                         ends[0]))
        result = {
            'metric': 'GiB/s chunked, device-resident streams',
            'value': round(value, 2),
            'unit': 'GiB/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'warmup_run': {'steps': warm_steps, 'ms': round(warm_s * 1e3, 1),
                           'rule': f'at least --warmup steps and {WARM_MS} ms of them'},
            'ms_per_step': round(ms_per_step, 3),
            'pipeline': {'on': pipelined, 'reserve_cus': reserve, 'pipelined_steps': piped,
                         'unpipelined_ms_per_step': None if seq_ms is None else round(seq_ms, 3),
                         'note': 'steps are RC_PIPELINED calls: step k\'s edge + chain kernels '
                                 'run on the reserved CUs beside step k+1\'s tile kernel (the '
                                 'library runs small-window batches, and batches with fewer '
                                 'tiles than the tile kernel has waves, in sequence: '
                                 'pipelined_steps counts the overlapped ones); every '
                                 'step still computes every cut'} if pipelined else {'on': False},
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'u8',
            'data': 'synthetic (splitmix64 counter streams generated in HBM)' if harness is None
                    else 'synthetic (Random(0): the reference harness stream, copied to HBM)',
            'config': {'workload': describe(args, long, n, size, min_len, max_len, world, edit),
                       'streams_per_gpu': n, 'stream_bytes': size,
                       'parallelism': f'streams/{world} ranks' if long is None
                       else f'one stream split over {world} ranks'},
            'roofline': roof,
            'cpu_baseline': cpu,
            'parity_sha256': parity,
            'parity_scope': scope,
            'devices': [d['pci'] for d in devices],
            'distinct_devices': len({d['uuid'] or d['pci'] for d in devices}),
            'ranks_seen': world,
            'shared_devices': shared,
            'per_rank': per_rank,
        }
        if harness is not None:
            result['rate_GBps'] = round(bytes_per_step * args.steps / elapsed / 1e9, 3)
        if edit is not None and getattr(edit, 'result', None) is not None:
            result['dedup'] = edit.result
        if args.e2e and long is None and harness is None:
            result['e2e_host_gibs'] = e2e_rates(ch, n, size)
        if args.calibrate:
            result['read_probe_gbs'] = be.read_probe_gbs(base_ptr, sum(lens))
        print(json.dumps(result), flush=True)
    ranks.barrier()
    ranks.close()
    # release the chunker's device state (its CU-masked streams) while the runtime is up
    close = getattr(ch, 'close', None)
    if close is not None:
        be.synchronize()
        close()
    return result


def describe(args, long, n, size, min_len, max_len, world, edit):
    if long is not None:
        return ('config3ii: ONE stream of %d GiB (last piece = final 1 MiB) split over %d '
                'rank(s), min %d, max %d, key %s' % (long.L >> 30, world, min_len, max_len,
                                                     args.key))
    if args.config == 'harness':
        return ('harness: Repository._benchmark_chunker stream, 10 x 512,000,000 B Random(0) '
                'as one stream of 10 pieces, min %d, max %d' % (min_len, max_len))
    w = ('config%s: %d x %d MiB streams per GPU, min %d, max %d, key %s'
         % (args.config, n, size >> 20, min_len, max_len, args.key))
    if edit is not None:
        w += ' (512 of the 1024 edited, re-chunk + dedup check)'
    return w


def e2e_rates(ch, n, size):
    """Host-resident streams: pinned copies in, chunking, cut offsets out (rc_chunk_host)."""
    import torch
    from replicat_amd import synth
    m = min(n, 64)
    hbufs = [synth.stream_bytes(size, synth.DEFAULT_SEED, i) for i in range(m)]
    pinned = torch.empty(m * size, dtype=torch.uint8).pin_memory()
    pv = pinned.numpy()
    for i, b in enumerate(hbufs):
        pv[i * size:(i + 1) * size] = b
    pbufs = [pv[i * size:(i + 1) * size] for i in range(m)]
    out = {}
    for label, bufs in (('pageable', hbufs), ('pinned', pbufs)):
        ch.chunk_host(bufs[:2])
        t1 = time.perf_counter()
        ch.chunk_host(bufs)
        out[label] = round(m * size / (time.perf_counter() - t1) / GIB, 2)
    out['streams'] = m
    return out


if __name__ == '__main__':
    sys.exit(cli())
