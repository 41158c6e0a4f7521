# round 6: config 3 (iii) against config 2 on one allocation (clipped last tiles); the harness
# line with --warmup 5 against --warmup 50 (the busy-time warm-up floor), alternating; config 2
# with its read probe (--calibrate)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06h; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/c2_vs_3iii.py 4 10 > $out/c2_vs_3iii.log 2>&1; tail -1 $out/c2_vs_3iii.log | cut -c1-400
for w in 5 50 5 50; do
  timeout -k 10 200 python -u bench.py --config harness --warmup $w --steps 20 --cpu-streams 0 > $out/harness_w$w.log 2>&1 || exit 3
  tail -1 $out/harness_w$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('warmup', d['warmup'], d['warmup_run'], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python -u bench.py --calibrate --steps 20 --cpu-streams 0 > $out/c2_calibrate.log 2>&1 || exit 4
tail -1 $out/c2_calibrate.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r.get('read_probe'), r.get('frac'))"
