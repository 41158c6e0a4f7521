"""Gaps between consecutive kernels per queue in a rocprofv3 kernel trace (CSV): for every
queue, the kernels in start order, and for the named kernel the idle time between one launch's
end and the next launch's start, with what ran on the queue in between.

    python scripts/trace_gaps.py <kernel_trace.csv> [kernel substring, default rc_tile_kernel]
"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else 'rc_tile_kernel'
rows = list(csv.DictReader(open(path)))
q = defaultdict(list)
for r in rows:
    q[r.get('Queue_Id', '?')].append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                                      r['Kernel_Name'][:60]))
t0 = min(k[0] for v in q.values() for k in v)
for qid, ks in sorted(q.items()):
    ks.sort()
    names = defaultdict(int)
    for k in ks:
        names[k[2]] += 1
    print(f'queue {qid}: {len(ks)} kernels: ' + ', '.join(f'{n} x{c}' for n, c in names.items()))
    idx = [i for i, k in enumerate(ks) if name in k[2]]
    gaps = []
    for a, b in zip(idx, idx[1:]):
        between = [k[2] for k in ks[a + 1:b]]
        gaps.append((ks[b][0] - ks[a][1]) / 1e3)
        print(f'  {name} end {(ks[a][1] - t0) / 1e3:.1f} us -> next start {(ks[b][0] - t0) / 1e3:.1f} us: '
              f'gap {gaps[-1]:.1f} us, between: {between}')
    if idx:
        d = [(ks[i][1] - ks[i][0]) / 1e3 for i in idx]
        print(f'  {name}: {len(idx)} launches, mean {sum(d) / len(d):.1f} us')
