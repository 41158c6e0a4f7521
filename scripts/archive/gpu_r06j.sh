# round 6: is config 3 (iii)'s quad chain latency- or throughput-bound?  The chain's time with
# 65,536 / 32,768 / 16,384 / 8,192 streams of 1 MiB (2,000 / 80,000), and one SQ counter pass
# restricted to the quad chain kernel on the full configuration
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06j; mkdir -p $out
export TMPDIR=/tmp
for n in 65536 32768 16384 8192; do
  timeout -k 10 200 python -u bench.py --config 3iii --streams $n --steps 10 --cpu-streams 0 --no-verify > $out/chain_$n.log 2>&1 || { tail -5 $out/chain_$n.log; exit 3; }
  tail -1 $out/chain_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print($n, d['ms_per_step'], r['kernel_ms'], r['edge_kernel_ms'], r['chain_kernel_ms'])"
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex "rc_quad_chain" --output-format csv -d $out/sq -o run -- python3 bench.py --config 3iii --steps 5 --cpu-streams 0 --no-verify > $out/sq.log 2>&1 || { tail -5 $out/sq.log; exit 4; }
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --kernel-include-regex "rc_quad_chain|rc_edge|rc_tile" --output-format csv -d $out/trace -o run -- python3 bench.py --config 3iii --steps 5 --cpu-streams 0 --no-verify > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 5; }
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob('gpurun_out/r06j/sq/**/*counter_collection.csv', recursive=True):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in sorted(acc.items()):
        print(k, len(v), sum(v) / len(v))
PY
