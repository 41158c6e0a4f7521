# round 6: the streaming-read ceiling with the simplest load patterns (scripts/ubench/read_ceiling.hip,
# built in the container into diag/read_ceiling) beside the bench's own read probe (config 2, --calibrate)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06k; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 diag/read_ceiling > $out/read_ceiling_a.log 2>&1 || { cat $out/read_ceiling_a.log; exit 3; }
cat $out/read_ceiling_a.log
timeout -k 10 300 python -u bench.py --steps 10 --calibrate --cpu-streams 0 > $out/bench_cal.log 2>&1 || { tail -5 $out/bench_cal.log; exit 4; }
tail -1 $out/bench_cal.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench', d['value'], d['read_probe_gbs'], r['kernel_ms'], r.get('achieved_read'))"
timeout -k 10 200 diag/read_ceiling > $out/read_ceiling_b.log 2>&1 || { cat $out/read_ceiling_b.log; exit 5; }
cat $out/read_ceiling_b.log
