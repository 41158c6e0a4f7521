# Round 5, pass p: the masked tile launch's fixed cost -- pipelined steps whose tile stream is
# masked (default), has a full mask, or is a plain stream (RC_TILE_MASK), against sequential
# steps: the harness (a 0.8 ms launch) and config 2; then the tests of pipelined calls under
# the fastest variant's setting.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05p
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/overlap_ab.py harness 6 seq p32 p32+full p32+plain m32+plain > $out/ab_harness.log 2>&1 || { echo "ab harness failed"; tail -5 $out/ab_harness.log; exit 3; }
tail -1 $out/ab_harness.log
timeout -k 10 500 python -u scripts/overlap_ab.py 2 3 seq p32 p32+full p32+plain > $out/ab_c2.log 2>&1 || { echo "ab c2 failed"; tail -5 $out/ab_c2.log; exit 4; }
tail -1 $out/ab_c2.log
timeout -k 10 500 python -u scripts/overlap_ab.py 3ii 3 seq p32 p32+plain > $out/ab_c3ii.log 2>&1 || { echo "ab 3ii failed"; tail -5 $out/ab_c3ii.log; exit 5; }
tail -1 $out/ab_c3ii.log
echo done
