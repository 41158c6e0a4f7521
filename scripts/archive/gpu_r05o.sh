# Round 5, pass o: why the harness's masked tile launch is slower on some boxes -- pipelined steps
# (the previous step's chain beside the tile kernel) against "isolated" ones (mR: pipelined, but
# each step waits for its own chain) and sequential ones; config 2 the same.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05o
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/overlap_ab.py harness 6 seq p32 m32 p8 m8 > $out/ab_harness.log 2>&1 || { echo "ab harness failed"; tail -5 $out/ab_harness.log; exit 3; }
tail -1 $out/ab_harness.log
timeout -k 10 500 python -u scripts/overlap_ab.py 2 3 seq p32 m32 > $out/ab_c2.log 2>&1 || { echo "ab c2 failed"; tail -5 $out/ab_c2.log; exit 4; }
tail -1 $out/ab_c2.log
echo done
