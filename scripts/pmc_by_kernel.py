"""Mean PMC counter values per kernel (and per dispatch of it) over rocprofv3 --pmc output dirs.

    python scripts/pmc_by_kernel.py gpurun_out/ab/pmc_*
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.replace('(anonymous namespace)::', '')
    return name.split('(')[0][:40]


def main(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            for r in csv.DictReader(open(f)):
                agg[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
    for k in sorted(agg):
        if 'fill' in k or 'elementwise' in k:
            continue
        print(k)
        for c, v in sorted(agg[k].items()):
            print(f'   {c:24s} {sum(v) / len(v):16.1f}   (n={len(v)})')


if __name__ == '__main__':
    main(sys.argv[1:])
