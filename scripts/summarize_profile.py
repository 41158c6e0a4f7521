"""Condense a rocprofv3 run (kernel stats + PMC passes under gpurun_out/prof) into
profiles/<tag>/: the kernel-trace stats CSV as written by rocprofv3, plus a per-kernel JSON of
PMC means with the gfx950 HBM correction applied (MI355X_MICROARCH.md §HBM: FETCH_SIZE counts
half the bytes of a wide coalesced stream; both counters are in KiB).

    python scripts/summarize_profile.py r01 [gpurun_out/prof]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOAD = 'config2'              # bench.py's default: 1024 x 64 MiB
PROBE_BYTES = 1024 * (64 << 20)   # rc_read_probe over the same arena (whole 16 KiB tiles)


def short(name):
    for k in ('rc_tile_kernel', 'rc_edge_kernel', 'rc_chain_kernel', 'rc_spec_kernel',
              'rc_join_kernel', 'rc_fill_kernel', 'rc_read_probe_kernel', 'rc_merge_kernel',
              'rc_scan_kernel', 'rc_copy_kernel', 'rc_mark_kernel'):
        if k in name:
            return k
    return name[:60]


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, 'gpurun_out', 'prof')
    dst = os.path.join(ROOT, 'profiles', tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'),
                os.path.join(dst, 'kernel_stats.csv'))
    out = {}
    for r in csv.DictReader(open(os.path.join(src, 'trace', 'run_kernel_stats.csv'))):
        out.setdefault(short(r['Name']), {})['avg_ns'] = float(r['AverageNs'])
        out[short(r['Name'])]['calls'] = int(r['Calls'])
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, 'run_counter_collection.csv')
        if p == 'trace' or not os.path.exists(f):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[(short(r['Kernel_Name']), r['Counter_Name'])].append(float(r['Counter_Value']))
        for (k, c), v in agg.items():
            out.setdefault(k, {})[c] = sum(v) / len(v)
    for k, d in out.items():
        if not isinstance(d, dict):
            continue
        if 'FETCH_SIZE' in d:
            d['hbm_read_bytes_corrected'] = 2 * d['FETCH_SIZE'] * 1024
        if 'WRITE_SIZE' in d:
            d['hbm_write_bytes'] = d['WRITE_SIZE'] * 1024
        if 'GRBM_GUI_ACTIVE' in d and d.get('avg_ns'):
            d['effective_clock_ghz'] = d['GRBM_GUI_ACTIVE'] / 8 / d['avg_ns']
    # calibration on a known byte count in the same access pattern (MI355X_MICROARCH.md §HBM:
    # 'calibrate on a known byte count in your own access pattern'): the read probe streams
    # exactly PROBE_BYTES with the tile kernel's loads (bench.py --calibrate, config 2)
    probe = out.get('rc_read_probe_kernel', {})
    if probe.get('FETCH_SIZE'):
        factor = PROBE_BYTES / (probe['FETCH_SIZE'] * 1024)
        out['calibration'] = {'probe_bytes': PROBE_BYTES, 'bytes_per_fetch_byte': factor}
        for k, d in out.items():
            if isinstance(d, dict) and 'FETCH_SIZE' in d:
                d['hbm_read_bytes_calibrated'] = d['FETCH_SIZE'] * 1024 * factor
    out['workload'] = WORKLOAD
    # the library build these counters are of (bench.py refuses a summary of another build):
    # the build id the profiled bench command printed (its JSON line in trace.log); the local
    # library's id only if that line is missing -- the tree may have been rebuilt since the run
    bid = None
    try:
        for line in open(os.path.join(src, 'trace.log')):
            if line.startswith('{'):
                bid = json.loads(line).get('roofline', {}).get('build_id') or bid
    except OSError:
        pass
    if bid is None:
        sys.path.insert(0, ROOT)
        from replicat_amd.build import embedded_id
        bid = embedded_id()
        print('warning: no bench line in trace.log; stamping the local library build', bid)
    out['build_id'] = bid
    with open(os.path.join(dst, 'pmc_summary.json'), 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out.get('rc_tile_kernel', {}), indent=1))


if __name__ == '__main__':
    main()
