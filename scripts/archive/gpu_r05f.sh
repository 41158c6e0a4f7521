# Round 5, pass f: sweep of the workgroup-grab schedule (static share, unit size, group size)
# against the round-4 per-wave schedule, every configuration, one allocation each.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05f
mkdir -p $out
export TMPDIR=/tmp
B=100:12:128:0
timeout -k 10 500 python -u scripts/harness_sched_probe.py 2 3 $B 100:3:0:64 0:3:0:64 100:2:0:64 100:3:0:128 100:4:0:128 50:3:0:64 > $out/c2.log 2>&1 || { echo "c2 failed"; tail -5 $out/c2.log; exit 3; }
tail -1 $out/c2.log
timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 4 1000:12:128:0 100:3:0:64 0:3:0:64 100:2:0:128 100:3:0:128 0:2:0:64 > $out/harness.log 2>&1 || { echo "harness failed"; tail -5 $out/harness.log; exit 4; }
tail -1 $out/harness.log
timeout -k 10 500 python -u scripts/harness_sched_probe.py 3iii 3 $B 100:3:0:64 0:3:0:64 100:3:0:128 > $out/c3iii.log 2>&1 || { echo "3iii failed"; tail -5 $out/c3iii.log; exit 5; }
tail -1 $out/c3iii.log
timeout -k 10 500 python -u scripts/harness_sched_probe.py 3ii 3 $B 100:3:0:64 0:3:0:64 100:3:0:128 > $out/c3ii.log 2>&1 || { echo "3ii failed"; tail -5 $out/c3ii.log; exit 6; }
tail -1 $out/c3ii.log
timeout -k 10 600 python -u scripts/harness_sched_probe.py 4 2 $B 100:3:0:64 100:3:0:128 100:6:0:64 > $out/c4.log 2>&1 || { echo "4 failed"; tail -5 $out/c4.log; exit 7; }
tail -1 $out/c4.log
echo done
