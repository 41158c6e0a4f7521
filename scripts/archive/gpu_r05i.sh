# Round 5, pass i: workgroup grabs as the default candidate -- sweep of static share / unit /
# group on every configuration (tile kernel + read probe, one allocation each), and pipelined
# steps (one and two tile streams) on config 2, 3 (ii) and config 4.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05i
mkdir -p $out
export TMPDIR=/tmp
B=100:12:128:0
timeout -k 10 500 python -u scripts/harness_sched_probe.py 2 3 $B 0:3:0:64 0:2:0:64 0:2:0:128 0:4:0:64 0:3:0:32 0:3:0:128 > $out/c2_sched.log 2>&1 || { echo "c2 failed"; tail -5 $out/c2_sched.log; exit 3; }
tail -1 $out/c2_sched.log
timeout -k 10 500 python -u scripts/harness_sched_probe.py 3iii 3 $B 0:3:0:64 100:3:0:64 0:2:0:64 0:4:0:64 > $out/c3iii_sched.log 2>&1 || { echo "3iii failed"; tail -5 $out/c3iii_sched.log; exit 4; }
tail -1 $out/c3iii_sched.log
timeout -k 10 500 python -u scripts/harness_sched_probe.py 3ii 3 $B 0:3:0:64 100:3:0:64 0:2:0:64 > $out/c3ii_sched.log 2>&1 || { echo "3ii failed"; tail -5 $out/c3ii_sched.log; exit 5; }
tail -1 $out/c3ii_sched.log
timeout -k 10 600 python -u scripts/harness_sched_probe.py 4 2 $B 0:3:0:64 100:3:0:64 0:2:0:64 > $out/c4_sched.log 2>&1 || { echo "4 failed"; tail -5 $out/c4_sched.log; exit 6; }
tail -1 $out/c4_sched.log
timeout -k 10 500 python -u scripts/overlap_ab.py 2 3 p32 p32@0:3:0:64 p32x2@0:3:0:64 seq@0:3:0:64 > $out/ab_c2.log 2>&1 || { echo "ab c2 failed"; tail -5 $out/ab_c2.log; exit 7; }
tail -1 $out/ab_c2.log
timeout -k 10 500 python -u scripts/overlap_ab.py 3ii 3 p32 p32@0:3:0:64 p32x2@0:3:0:64 > $out/ab_c3ii.log 2>&1 || { echo "ab 3ii failed"; tail -5 $out/ab_c3ii.log; exit 8; }
tail -1 $out/ab_c3ii.log
echo done
