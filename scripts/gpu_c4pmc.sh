# Config-4 attribution, counters: the tile kernel on 1024 x 64 MiB vs 8 x 8 GiB (same footprint).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4p
export TMPDIR=/tmp
for spec in "c2:--config 2" "c4_8x8g:--config 4 --streams 8"; do
  tag=${spec%%:*}; args=${spec#*:}
  B="bench.py --steps 3 --warmup 1 --cpu-streams 0 --no-verify $args"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c4p/$tag/fetch -o run -- python3 $B > gpurun_out/c4p/${tag}_fetch.log 2>&1 || { echo "fetch $tag failed"; exit 4; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS --output-format csv -d gpurun_out/c4p/$tag/sq -o run -- python3 $B > gpurun_out/c4p/${tag}_sq.log 2>&1 || { echo "sq $tag failed"; exit 5; }
  timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/c4p/$tag/ta -o run -- python3 $B > gpurun_out/c4p/${tag}_ta.log 2>&1 || echo "ta $tag failed (ignored)"
done
python3 - <<'PY'
import csv, glob, collections
for tag in ('c2', 'c4_8x8g'):
    acc = collections.defaultdict(list)
    for f in glob.glob(f'gpurun_out/c4p/{tag}/*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'rc_tile_kernel' in r['Kernel_Name']:
                acc[r['Counter_Name']].append(float(r['Counter_Value']))
    print(tag, {k: round(sum(v) / len(v)) for k, v in sorted(acc.items())})
PY
