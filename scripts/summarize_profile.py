"""Condense a rocprofv3 run (kernel stats + PMC passes) into profiles/<tag>/: the kernel-trace
stats CSV as written by rocprofv3, plus per-kernel PMC means with the gfx950 HBM correction
applied (MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of a wide coalesced stream;
both counters are in KiB), stamped with the library build the profiled bench line printed.

    python scripts/summarize_profile.py r04 [gpurun_out/prof]          (config 2, the default bench)
    python scripts/summarize_profile.py r05 --workload harness gpurun_out/pmc/harness

Round 5: one summary file per round holds every BASELINE workload (``workloads``: config2,
config2_seeded, config3ii, config3iii, config4, config5, harness), each from its own bench
command; the read probe of that command (--calibrate) calibrates FETCH_SIZE on the same bytes.
bench.py pmc_traffic() reads the entry of the line's workload and refuses another build's.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TILE_BYTES = 4096 * 4  # rc_read_probe reads whole 16 KiB tiles


def short(name):
    for k in ('rc_tile_kernel', 'rc_edge_kernel', 'rc_chain_kernel', 'rc_spec_kernel',
              'rc_join_kernel', 'rc_fill_kernel', 'rc_read_probe_kernel', 'rc_merge_kernel',
              'rc_scan_kernel', 'rc_copy_kernel', 'rc_mark_kernel', 'rc_quad_chain_kernel',
              'rc_lane_chain_kernel', 'rc_fill_streams_kernel'):
        if k in name:
            return k
    return name[:60]


def bench_line(src):
    """The profiled bench command's JSON line (trace.log, else any *.log under src)."""
    for f in ['trace.log'] + sorted(x for x in os.listdir(src) if x.endswith('.log')):
        try:
            for line in open(os.path.join(src, f)):
                if line.startswith('{'):
                    return json.loads(line)
        except (OSError, ValueError):
            continue
    return None


def summarize(src, probe_bytes=None):
    out = {}
    stats = os.path.join(src, 'trace', 'run_kernel_stats.csv')
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            d = out.setdefault(short(r['Name']), {})
            # several template instances of one kernel: keep the busiest
            if int(r['Calls']) >= d.get('calls', 0):
                d['avg_ns'] = float(r['AverageNs'])
                d['calls'] = int(r['Calls'])
    # round 6: the per-launch trace too -- the average above includes the
    # first launch (a cold clock: config 2's 11.3 ms against ~9.5 after), so the steady-state
    # mean (first launch dropped) and the median are what the bench line's frac is checked on
    trace = os.path.join(src, 'trace', 'run_kernel_trace.csv')
    if os.path.exists(trace):
        per = collections.defaultdict(list)
        for r in csv.DictReader(open(trace)):
            per[short(r['Kernel_Name'])].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
        for k, v in per.items():
            d = out.setdefault(k, {})
            steady = v[1:] if len(v) > 1 else v
            d['launches'] = len(v)
            d['first_ns'] = v[0]
            d['steady_avg_ns'] = sum(steady) / len(steady)
            d['median_ns'] = float(sorted(v)[len(v) // 2])
            if k == 'rc_tile_kernel':
                d['launch_ns'] = v[:64]
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, 'run_counter_collection.csv')
        if p == 'trace' or not os.path.exists(f):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[(short(r['Kernel_Name']), r['Counter_Name'])].append(float(r['Counter_Value']))
        for (k, c), v in agg.items():
            d = out.setdefault(k, {})
            d[c] = sum(v) / len(v)
            if c == 'FETCH_SIZE' and k == 'rc_tile_kernel' and len(v) > 2:
                d['FETCH_SIZE_launches'] = len(v)
                d['FETCH_SIZE_min_max'] = [min(v), max(v)]
    for k, d in out.items():
        if 'FETCH_SIZE' in d:
            d['hbm_read_bytes_corrected'] = 2 * d['FETCH_SIZE'] * 1024
        if 'WRITE_SIZE' in d:
            d['hbm_write_bytes'] = d['WRITE_SIZE'] * 1024
        if 'GRBM_GUI_ACTIVE' in d and d.get('avg_ns'):
            d['effective_clock_ghz'] = d['GRBM_GUI_ACTIVE'] / 8 / d['avg_ns']
    # calibration on a known byte count in the same access pattern (MI355X_MICROARCH.md §HBM:
    # 'calibrate on a known byte count in your own access pattern'): the read probe streams
    # exactly probe_bytes of the same arena with the tile kernel's loads (bench.py --calibrate)
    probe = out.get('rc_read_probe_kernel', {})
    if probe.get('FETCH_SIZE') and probe_bytes:
        factor = probe_bytes / (probe['FETCH_SIZE'] * 1024)
        out['calibration'] = {'probe_bytes': probe_bytes, 'bytes_per_fetch_byte': factor}
        for d in out.values():
            if isinstance(d, dict) and 'FETCH_SIZE' in d:
                d['hbm_read_bytes_calibrated'] = d['FETCH_SIZE'] * 1024 * factor
    return out


def main():
    args = sys.argv[1:]
    tag = args.pop(0)
    workload = None
    if '--workload' in args:
        i = args.index('--workload')
        workload = args[i + 1]
        del args[i:i + 2]
    src = args[0] if args else os.path.join(ROOT, 'gpurun_out', 'prof')
    dst = os.path.join(ROOT, 'profiles', tag)
    os.makedirs(dst, exist_ok=True)
    line = bench_line(src)
    bid = (line or {}).get('roofline', {}).get('build_id')
    if bid is None:
        sys.path.insert(0, ROOT)
        from replicat_amd.build import embedded_id
        bid = embedded_id()
        print('warning: no bench line under', src, '; stamping the local library build', bid)
    if workload is None:  # the round-4 layout: config 2 only, at the top level
        out = summarize(src, 1024 * (64 << 20))
        shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'),
                    os.path.join(dst, 'kernel_stats.csv'))
        out['workload'] = 'config2'
        out['build_id'] = bid
        with open(os.path.join(dst, 'pmc_summary.json'), 'w') as f:
            json.dump(out, f, indent=1, sort_keys=True)
        print(json.dumps(out.get('rc_tile_kernel', {}), indent=1))
        return
    algo = (line or {}).get('roofline', {}).get('algorithmic_bytes')
    probe_bytes = algo // TILE_BYTES * TILE_BYTES if algo else None
    out = summarize(src, probe_bytes)
    t = out.get('rc_tile_kernel', {})
    if line:
        r = line['roofline']
        t['bytes_read_algorithmic'] = r.get('bytes_read')
        t['stream_bytes'] = r.get('algorithmic_bytes')
        if t.get('steady_avg_ns') and r.get('algorithmic_bytes'):
            # the roofline from the profile alone: stream bytes per launch / steady-state launch
            t['profile_frac'] = round(r['algorithmic_bytes'] / t['steady_avg_ns'] / 8000.0, 4)
            t['profile_frac_median'] = round(r['algorithmic_bytes'] / t['median_ns'] / 8000.0, 4)
            t['line_frac'] = r.get('frac')
        if t.get('hbm_read_bytes_corrected') and r.get('bytes_read'):
            t['traffic_over_bytes_read'] = round(
                (t['hbm_read_bytes_corrected'] + t.get('hbm_write_bytes', 0.0)) / r['bytes_read'], 4)
        out['bench_line'] = {k: line.get(k) for k in ('value', 'ms_per_step', 'config')}
    path = os.path.join(dst, 'pmc_summary.json')
    try:
        with open(path) as f:
            summary = json.load(f)
    except (OSError, ValueError):
        summary = {}
    if summary.get('build_id') not in (None, bid):
        print(f'warning: {path} holds build {summary.get("build_id")}; replacing it with {bid}')
        summary = {}
    summary['build_id'] = bid
    summary.setdefault('workloads', {})[workload] = out
    with open(path, 'w') as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    if os.path.exists(os.path.join(src, 'trace', 'run_kernel_stats.csv')):
        shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'),
                    os.path.join(dst, f'kernel_stats_{workload}.csv'))
    print(workload, json.dumps({k: t.get(k) for k in ('avg_ns', 'hbm_read_bytes_corrected',
                                                      'hbm_write_bytes', 'traffic_over_bytes_read')}))


if __name__ == '__main__':
    main()
