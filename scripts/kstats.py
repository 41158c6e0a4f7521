"""Print kernel name / calls / average ms from a rocprofv3 kernel_stats.csv."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof/trace/run_kernel_stats.csv')):
    name = r['Name'].split('(')[0].replace('(anonymous namespace)::', '')
    if '::' in r['Name'] and 'rc_' in r['Name']:
        name = r['Name'].split('::')[1].split('(')[0]
    print(f"{name[:40]:40s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e6:9.4f} ms")
