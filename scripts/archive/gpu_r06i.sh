# round 6: AES-256 CTR keystream, bitsliced vs T-table (scripts/ubench/aes_bitslice.hip, built in
# the container into diag/aes_bitslice), correctness against the FIPS-197-pinned host AES; then
# one SQ counter pass over the same binary
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06i; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 diag/aes_bitslice 50 > $out/aes_bitslice.log 2>&1 || { cat $out/aes_bitslice.log; exit 3; }
cat $out/aes_bitslice.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $out/sq -o run -- diag/aes_bitslice 20 > $out/sq.log 2>&1 || { tail -5 $out/sq.log; exit 4; }
python3 - <<'PY'
import csv, collections, glob
f = glob.glob('gpurun_out/r06i/sq/**/run_counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()}, 'launches', len(next(iter(d.values()))))
PY
