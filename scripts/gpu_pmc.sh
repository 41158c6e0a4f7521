# PMC passes over a short bench (one rocprofv3 process per counter set).  Usage:
#   bash scripts/gpu_pmc.sh "SET1" "SET2" ...   (each SET = space-separated counters)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-streams 0 --no-verify ${BENCH_ARGS:-} > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; }
done
python3 - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob('gpurun_out/pmc/p*/run_counter_collection.csv')):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        k = k.split('::')[1].split('(')[0] if '::' in k else k[:30]
        agg[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
    for (k, c), v in sorted(agg.items()):
        if 'fill' in k or 'elementwise' in k:
            continue
        print(f'{k:18s} {c:40s} {sum(v)/len(v):.4g}')
PY
